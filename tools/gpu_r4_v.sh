#!/bin/bash
# Round 4, call V: the final tree's GPU tests, smoke and bench line (tools/round_end.sh), then the
# C4 kernel-trace summary and PMC passes on this build (the 65k step's GEMM PMC pass is left out:
# it dies inside rocprofv3, DESIGN round-4 table).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/tools/round_end.sh
O=$R/gpurun_out/r4prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/rocprof_summary.py $O/c4/c4_kernel_stats.csv $O/c4_summary.txt 25 > /dev/null
echo ok c4 stats
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc_$n -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4pmc_$n.log 2>&1
  echo ok c4 pmc $n
done
python3 $R/tools/pmc_c4.py $(ls $O/c4pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_WRITE_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_TCC_HIT_sum/*counter_collection.csv | head -1) --runs 3 --out $O/pmc_c4_r4.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum} -- python3 tools/c4_time.py --reps 1 32" > $O/pmc_c4.txt
echo done

#!/bin/bash
# Round-5 profiling on the GPU box (outputs under gpurun_out/r5prof; summaries copied to profiles/):
#  1. rocprofv3 --kernel-trace --stats of one timed 65k placement step (the bench's own command
#     with the C4 / VGP / sweep lines off), whose gemm_glds average is compared with the bench
#     line's live avg_launch_ms;
#  2. C4 (128^3, k = 50): kernel-trace stats of one run, and FETCH_SIZE / WRITE_SIZE /
#     TCC_HIT_sum + TCC_MISS_sum passes over its kernels -> pmc_c4_r5.json (hash-tied to
#     exact_greedy.hip).  The GEMM's PMC traffic comes from the PyTorch-free driver
#     (tools/step65k.cpp, profiles/traffic_r5.json) and is re-measured only when gemm.hip changes.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --no-sweep --steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o bench -- python3 $R/bench.py $ARGS > $O/step.log 2>&1
python3 $R/tools/rocprof_summary.py $O/step/bench_kernel_stats.csv $O/step_summary.txt > /dev/null
grep "^{" $O/step.log > $O/step_line.json
echo ok step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/rocprof_summary.py $O/c4/c4_kernel_stats.csv $O/c4_summary.txt 25 > /dev/null
echo ok c4 stats
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc_$n -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4pmc_$n.log 2>&1
  echo ok c4 pmc $n
done
python3 $R/tools/pmc_c4.py $(ls $O/c4pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_WRITE_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_TCC_HIT_sum/*counter_collection.csv | head -1) --runs 3 --out $O/pmc_c4_r5.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum} -- python3 tools/c4_time.py --reps 1 32" > $O/pmc_c4.txt
echo done

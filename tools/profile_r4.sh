#!/bin/bash
# Round-4 profiling on the GPU box (outputs under gpurun_out/r4prof; summaries copied to profiles/):
#  1. rocprofv3 --kernel-trace --stats of exactly one timed 65k placement step;
#  2. C4 (128^3, k = 50): kernel-trace stats of one run, and FETCH_SIZE / WRITE_SIZE /
#     TCC_HIT_sum + TCC_MISS_sum passes over its kernels -> pmc_c4_r4.json;
#  3. PMC passes, one counter per run (FETCH_SIZE, then WRITE_SIZE) over the 65k step for the
#     GEMM / mat-vec / assembly kernels -> traffic_r4.json (hash-tied to the kernel sources).
#     Last, because rocprofv3's counter-collection dispatch hook died with SIGSEGV on this step
#     twice in round 4 (profiles/r4_rocprof_pmc_*_segv.log), with and without a kernel filter.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --no-sweep --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o bench -- python3 $R/bench.py $ARGS > $O/step.log 2>&1
python3 $R/tools/rocprof_summary.py $O/step/bench_kernel_stats.csv $O/step_summary.txt > /dev/null
grep "^{" $O/step.log > $O/step_line.json
echo ok step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/rocprof_summary.py $O/c4/c4_kernel_stats.csv $O/c4_summary.txt 25 > /dev/null
echo ok c4 stats
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc_$n -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4pmc_$n.log 2>&1
  echo ok c4 pmc $n
done
python3 $R/tools/pmc_c4.py $(ls $O/c4pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_WRITE_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_TCC_HIT_sum/*counter_collection.csv | head -1) --runs 3 --out $O/pmc_c4_r4.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum} -- python3 tools/c4_time.py --reps 1 32" > $O/pmc_c4.txt
echo ok c4 traffic
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o p -- python3 $R/bench.py $ARGS > $O/pmc_$c.log 2>&1
  echo ok pmc $c
done
F=$(ls $O/pmc_FETCH_SIZE/*counter_collection.csv | head -1)
W=$(ls $O/pmc_WRITE_SIZE/*counter_collection.csv | head -1)
python3 $R/tools/pmc_traffic.py $F $W --N 65536 --shape 64 32 32 --k 50 --out $O/traffic_r4.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} -- python3 bench.py $ARGS" > /dev/null
echo done

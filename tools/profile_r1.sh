#!/bin/bash
# Round-1 profiling on the GPU box (outputs under gpurun_out/, summaries copied to profiles/):
#  1. rocprofv3 --kernel-trace --stats of exactly one timed bench step (no warm-up, no separate
#     potrf, no C2 / VGP lines), so rocprof's per-kernel averages are comparable with bench.py's
#     live HIP-event ones;
#  2. PMC passes, one counter per run, for the GEMM, the mat-vec and the kernel assembly of the
#     same step -> per-launch HBM bytes (tools/pmc_traffic.py).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r1 -o bench -- python3 $R/bench.py $ARGS > $O/prof_r1.log 2>&1
grep "^{" $O/prof_r1.log > $O/prof_r1_bench.json
echo ok kernel-trace
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "gemm_glds|greedy_trmv|kernel_matrix" --output-format csv -d $O/pmc_$c -o p -- python3 $R/bench.py $ARGS > $O/pmc_$c.log 2>&1
  echo ok $c
done
python3 $R/tools/pmc_traffic.py $O/pmc_FETCH_SIZE/p_counter_collection.csv \
  $O/pmc_WRITE_SIZE/p_counter_collection.csv --N 65536 --shape 64 32 32 --k 50 \
  --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-include-regex 'gemm_glds|greedy_trmv|kernel_matrix' -- python3 bench.py $ARGS" \
  --out $O/traffic_r1.json > /dev/null
python3 $R/tools/rocprof_summary.py $O/prof_r1/bench_kernel_stats.csv $O/prof_r1_summary.txt > /dev/null
echo done

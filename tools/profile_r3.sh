#!/bin/bash
# Round-3 profiling on the GPU box (outputs under gpurun_out/; summaries copied to profiles/):
#  1. rocprofv3 --kernel-trace --stats of exactly one timed 65k placement step (the bench's main
#     line) and of the C4 exact run (tools/bench_exact.py: setup + one timed + profiled runs);
#  2. PMC passes, one counter per run (FETCH_SIZE, then WRITE_SIZE) over the same 65k step for the
#     GEMM / mat-vec / assembly kernels -> gpurun_out/traffic_r3.json (tools/pmc_traffic.py,
#     (FETCH x 2 + WRITE) x 1 KiB per the gfx950 correction, tied to the kernel-source hashes).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --no-sweep --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r3 -o bench -- python3 $R/bench.py $ARGS > $O/prof_r3.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof_r3/bench_kernel_stats.csv $O/prof_r3_summary.txt > /dev/null
echo ok placement
# C4 profile kept from the earlier run of this script
# REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r3_c4 -o c4 -- python3 $R/tools/bench_exact.py 128 50 512 > $O/prof_r3_c4.log 2>&1
# python3 $R/tools/rocprof_summary.py $O/prof_r3_c4/c4_kernel_stats.csv $O/prof_r3_c4_summary.txt 25 > /dev/null
# echo ok c4
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'gemm_glds|greedy_trmv|kernel_matrix' --output-format csv -d $O/pmc_r3_$c -o p -- python3 $R/bench.py $ARGS > $O/pmc_r3_$c.log 2>&1
  echo ok pmc $c
done
F=$(ls $O/pmc_r3_FETCH_SIZE/*counter_collection.csv | head -1)
W=$(ls $O/pmc_r3_WRITE_SIZE/*counter_collection.csv | head -1)
python3 $R/tools/pmc_traffic.py $F $W --N 65536 --shape 64 32 32 --k 50 --out $O/traffic_r3.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --kernel-include-regex 'gemm_glds|greedy_trmv|kernel_matrix' -- python3 bench.py $ARGS" > /dev/null
echo done

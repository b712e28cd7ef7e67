#!/bin/bash
# Round-2 profiling on the GPU box (outputs under gpurun_out/, summaries copied to profiles/ by
# hand): rocprofv3 --kernel-trace --stats of
#  1. exactly one timed 65k placement step (no warm-up, no side lines);
#  2. the C3 and C5 VGP training steps (tools/bench_vgp.py, 2 warm-up + 5 timed graph steps, then
#     5 eager profiled steps).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r2 -o bench -- python3 $R/bench.py $ARGS > $O/prof_r2.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof_r2/bench_kernel_stats.csv $O/prof_r2_summary.txt > /dev/null
echo ok placement
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r2_c3 -o vgp -- python3 $R/tools/bench_vgp.py --steps 5 > $O/prof_r2_c3.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof_r2_c3/vgp_kernel_stats.csv $O/prof_r2_c3_summary.txt 25 > /dev/null
echo ok c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r2_c5 -o vgp -- python3 $R/tools/bench_vgp.py --c5 --steps 5 > $O/prof_r2_c5.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof_r2_c5/vgp_kernel_stats.csv $O/prof_r2_c5_summary.txt 25 > /dev/null
echo done

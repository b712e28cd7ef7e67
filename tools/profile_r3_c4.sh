#!/bin/bash
# rocprofv3 --kernel-trace --stats of the C4 bounded-lazy form (tools/bench_bounds.py: two timed
# runs + one profiled run of 128^3, k = 50) -> gpurun_out/prof_r3_c4b_summary.txt.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r3_c4b -o c4b -- python3 $R/tools/bench_bounds.py 128 50 > $O/prof_r3_c4b.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof_r3_c4b/c4b_kernel_stats.csv $O/prof_r3_c4b_summary.txt 25 > /dev/null
echo ok c4b

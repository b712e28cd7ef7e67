#!/bin/bash
# Round 4, call E: kernel trace of one C4 run (per-launch durations and gaps of the rounds).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/timeline.py $O/tr/c4_kernel_trace.csv --marker exact_gersh_final --step -1 > $O/c4_timeline.txt
echo ok

#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench's 65k placement step on the final round-6 tree
# (step 1 of tools/profile_r6.sh; outputs under gpurun_out/r6prof_final).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6prof_final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --no-sweep --steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o bench -- python3 $R/bench.py $ARGS > $O/step.log 2>&1
python3 $R/tools/rocprof_summary.py $O/step/bench_kernel_stats.csv $O/step_summary.txt > /dev/null
grep "^{" $O/step.log > $O/step_line.json
echo ok step

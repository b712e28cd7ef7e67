#!/bin/bash
# Launch timeline of one graph-replayed VGP training step (C3, then C5) under rocprofv3
# --kernel-trace; tools/timeline.py prints every launch of the second-to-last timed step.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_c3 -o vgp -- python3 $R/tools/bench_vgp.py --steps 4 > $O/tl_c3.log 2>&1
python3 $R/tools/timeline.py $O/tl_c3/vgp_kernel_trace.csv --step 4 > $O/tl_c3.txt
echo ok c3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_c5 -o vgp -- python3 $R/tools/bench_vgp.py --c5 --steps 4 > $O/tl_c5.log 2>&1
python3 $R/tools/timeline.py $O/tl_c5/vgp_kernel_trace.csv --step 4 > $O/tl_c5.txt
echo ok c5

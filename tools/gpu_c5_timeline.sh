#!/bin/bash
# Launch timelines of one graph-replayed C5 step (matern52): fp64, then mixed with 2 refinement
# steps (rocprofv3 --kernel-trace; tools/timeline.py) -> gpurun_out/r4c5/tl_c5{f,m}.txt
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4c5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_c5f -o vgp -- python3 $R/tools/bench_vgp.py --c5 --kernel matern52 --steps 4 > $O/tl_c5f.log 2>&1
python3 $R/tools/timeline.py $O/tl_c5f/vgp_kernel_trace.csv --step 4 > $O/tl_c5f.txt
echo ok fp64
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_c5m -o vgp -- python3 $R/tools/bench_vgp.py --c5 --kernel matern52 --mixed --mixed-iters 2 --steps 4 > $O/tl_c5m.log 2>&1
python3 $R/tools/timeline.py $O/tl_c5m/vgp_kernel_trace.csv --step 4 > $O/tl_c5m.txt
echo ok mixed
rm -rf $O/tl_c5f $O/tl_c5m

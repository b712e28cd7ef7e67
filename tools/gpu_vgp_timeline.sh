#!/bin/bash
# Launch timeline of one graph-replayed VGP training step (C3, C5 Matern 5/2 fp64, C5 mixed with
# two refinement steps) under rocprofv3 --kernel-trace; tools/timeline.py prints every launch of
# the second-to-last timed step.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, bench_vgp args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl_$n -o vgp -- python3 $R/tools/bench_vgp.py --steps 4 "$@" > $O/tl_$n.log 2>&1
  python3 $R/tools/timeline.py $O/tl_$n/vgp_kernel_trace.csv --step 4 > $O/tl_$n.txt
  echo ok $n
}
run c3
run c5 --c5 --kernel matern52
# run c5m --c5 --kernel matern52 --mixed --mixed-iters 2

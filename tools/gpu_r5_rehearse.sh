#!/bin/bash
# Round 5, final build: bench.py --gpus 2 started plainly (it launches its own two ranks), gloo on
# one GPU (VGPOSP_BENCH_DEVICE=0): the sharded headline, the distributed Cholesky and C4's sharded
# bounds, with the committed picks.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5reh
mkdir -p $O
cd $R
VGPOSP_BENCH_DEVICE=0 timeout -k 10 700 python -u bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 \
  --no-cpu --no-vgp --no-sweep --no-c4-selinv --no-splits --no-c2 > $O/bench_2ranks.log 2>&1
grep "^{" $O/bench_2ranks.log > $O/bench_2ranks.json
echo ok launcher

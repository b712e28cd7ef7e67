#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: 2 ranks over gloo, both pinned to cuda:0
# (the driver's SCALE run uses RCCL, one GPU per rank).  Shape 32^3 keeps the gloo host staging
# of the distributed Cholesky short.
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
VGPOSP_BENCH_DEVICE=0 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --shape 32 32 32 \
  --steps 1 --warmup 1 > gpurun_out/rehearse2.log 2>&1
echo rc=$?

#!/bin/bash
# Rehearse bench.py's N > 1 path on a one-GPU box: NP ranks (default 2) over gloo, all pinned to
# cuda:0 (the driver's SCALE run uses RCCL, one GPU per rank).  Shape 32^3 keeps the gloo host
# staging of the distributed Cholesky short.  Output: gpurun_out/rehearse$NP.log
NP=${1:-2}
LIMIT=${2:-500}
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
VGPOSP_BENCH_DEVICE=0 timeout -k 10 $LIMIT python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $NP --backend gloo --shape 32 32 32 \
  --steps 1 --warmup 1 > gpurun_out/rehearse$NP.log 2>&1
echo rc=$?

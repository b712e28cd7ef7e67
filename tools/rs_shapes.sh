#!/bin/bash
# per-shape GEMM times of one 65k Cholesky + inverse under each GEMM kernel choice
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
for rs in 0 1 2; do
  VGPOSP_GEMM_RS=$rs timeout -k 10 200 python -u -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import gemm_shapes as g; g.main(top=80)" > gpurun_out/shapes_rs$rs.txt 2>&1
  echo ok $rs
done

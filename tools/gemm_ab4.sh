#!/bin/bash
# A/B of the GEMM tile-group size (row tiles per XCD band): the 16384^3 layout sweep and the
# 65k placement step for the default build and each tools/variants/lib_group*.so
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
for lib in default tools/variants/lib_group*.so; do
  if [ $lib = default ]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/$lib; fi
  echo "== $lib" >> gpurun_out/ab4_layouts.txt
  timeout -k 10 300 python -u tools/gemm_layouts.py >> gpurun_out/ab4_layouts.txt 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 2>&1 | grep '^{' | cut -c1-200 >> gpurun_out/ab4_layouts.txt
  echo ok $lib
done

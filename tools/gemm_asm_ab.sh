#!/bin/bash
# A/B of the explicitly sequenced GEMM K-loop variants (tools/variants/lib_asm*.so) against the
# default build: GEMM parity tests, the 16384^3 layout sweep, the 65k placement step and the C3 /
# C5 VGP steps.
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
out=gpurun_out/$1; shift
for lib in "$@"; do
  if [ $lib = default ]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/lib_$lib.so; fi
  echo "== $lib" >> $out
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linalg.py >> $out 2>&1
  timeout -k 10 300 python -u tools/gemm_layouts.py >> $out 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --no-c4 --no-sweep --steps 2 --warmup 1 2>&1 | grep '^{' | cut -c1-200 >> $out
  timeout -k 10 200 python -u tools/bench_vgp.py --steps 10 2>&1 | tail -2 | cut -c1-300 >> $out
  timeout -k 10 200 python -u tools/bench_vgp.py --c5 --kernel matern52 --steps 10 2>&1 | tail -2 | cut -c1-300 >> $out
  echo ok $lib
done

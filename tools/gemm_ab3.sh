#!/bin/bash
# A/B of GEMM library variants on one box: parity of the b128 variant, then the 16384^3 layout
# sweep and the 65k placement step for the default build and every tools/variants/*.so
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
VGPOSP_LIB=$PWD/tools/variants/lib_b128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_placement.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1
echo ok tests
for lib in default tools/variants/lib_b128.so tools/variants/lib_prio.so tools/variants/lib_b128prio.so; do
  if [ $lib = default ]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/$lib; fi
  echo "== $lib" >> gpurun_out/ab3_layouts.txt
  timeout -k 10 300 python -u tools/gemm_layouts.py >> gpurun_out/ab3_layouts.txt 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 2>&1 | grep '^{' | cut -c1-200 >> gpurun_out/ab3_layouts.txt
  echo ok $lib
done

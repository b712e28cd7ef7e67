#!/bin/bash
# A/B of GEMM variants (tools/build_gemm_variant.sh) on one box: the 16384^3 layout sweep and the
# 65k placement step, default build first.  Usage: tools/gemm_ab_r3.sh OUT lib_a lib_b ...
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
out=gpurun_out/$1; shift
for lib in default "$@"; do
  if [ $lib = default ]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/$lib.so; fi
  echo "== $lib" >> $out
  timeout -k 10 300 python -u tools/gemm_layouts.py >> $out 2>&1
  timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --no-c4 --no-sweep --steps 2 --warmup 1 2>&1 | grep '^{' | cut -c1-160 >> $out
  echo ok $lib
done

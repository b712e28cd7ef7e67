#!/bin/bash
# GPU A/B of the one-wave-per-SIMD register-staged GEMM (VGPOSP_GEMM_RS=1: 128x256, 2: 256x128):
# The RS kernel lives in tools/variants/gemm_experiments.hip: build tools/variants/lib_rs.so on
# the CPU first (bash tools/build_variant.sh rs).
# linalg parity tests under each, GEMM micro-benchmarks, one bench step.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
for rs in 1 2; do
  VGPOSP_LIB=$R/tools/variants/lib_rs.so VGPOSP_GEMM_RS=$rs timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py -x -q --timeout 200 --timeout-method thread > $O/rs${rs}_tests.log 2>&1
  echo ok tests rs=$rs
done
for rs in 0 1 2; do
  VGPOSP_LIB=$R/tools/variants/lib_rs.so VGPOSP_GEMM_RS=$rs timeout -k 10 300 python -u tools/bench_gemm.py > $O/rs${rs}_gemm.jsonl 2>&1
  echo ok gemm rs=$rs
done
for rs in 1 2; do
  VGPOSP_LIB=$R/tools/variants/lib_rs.so VGPOSP_GEMM_RS=$rs timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 > $O/rs${rs}_bench.log 2>&1
  echo ok bench rs=$rs
done

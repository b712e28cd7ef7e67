#!/bin/bash
# trtri with the split triangular-A TRMM: parity (GEMM/potrf/placement + full-size 65k checks),
# then the 65k placement step
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_placement.py tests/test_gpu_fullsize.py tests/test_gpu_gp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tc_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 > gpurun_out/tc_bench.log 2>&1
echo ok bench

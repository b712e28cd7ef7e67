#!/bin/bash
# One iteration of the VGP / GEMM work on the GPU box: linear-algebra + VGP GPU tests, the GEMM
# rate on the step's shapes, then tools/gpu_vgp.sh (VGP step times + timelines).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_vgp_train.py -x -q --timeout 200 --timeout-method thread > $O/iter_tests.log 2>&1
echo ok lin tests
timeout -k 10 200 python -u tools/bench_gemm.py > $O/gemm_rates.log 2>&1
echo ok gemm
bash tools/gpu_vgp.sh

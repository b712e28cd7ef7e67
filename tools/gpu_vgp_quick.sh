#!/bin/bash
# Grouped-GEMM test, VGP GPU tests, then C3 / C5 / C5-mixed step times with the grouped M x M
# products on / off (tools/vgp_ab.py).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_linalg.py -k "group or batched or beta01" -x -q --timeout 120 --timeout-method thread > $O/group_tests.log 2>&1
echo ok group tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_vgp_train.py tests/test_gpu_configs.py tests/test_gpu_mixed.py tests/test_gpu_vgp_dp.py tests/test_gpu_gp.py -x -q --timeout 200 --timeout-method thread > $O/vgp_tests.log 2>&1
echo ok vgp tests
timeout -k 10 200 python -u tools/vgp_ab.py VGPOSP_GEMM_GROUP=1,0 > $O/q_c3.jsonl 2>$O/q_c3.err
timeout -k 10 200 python -u tools/vgp_ab.py --c5 VGPOSP_GEMM_GROUP=1,0 > $O/q_c5.jsonl 2>$O/q_c5.err
timeout -k 10 200 python -u tools/vgp_ab.py --c5 --mixed VGPOSP_GEMM_GROUP=1,0 > $O/q_c5m.jsonl 2>$O/q_c5m.err
echo ok times

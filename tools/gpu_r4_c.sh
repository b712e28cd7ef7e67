#!/bin/bash
# Round 4, call C: C4 with the refine-or-pick decision on the device (tests + timing).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_linalg.py tests/test_gpu_placement.py tests/test_gpu_fullsize.py tests/test_gpu_vgp_dp.py tests/test_gpu_vgp_train.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 8 4 > $O/c4_time.jsonl 2> $O/c4_time.err
echo ok time

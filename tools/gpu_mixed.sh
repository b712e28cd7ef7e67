#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mixed_tests.log 2>&1
echo ok mixed tests
timeout -k 10 200 python -u tools/bench_vgp.py --c5 --mixed --steps 5 > gpurun_out/vgp_c5_mixed.log 2>&1
echo ok bench
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v -k "c5" --timeout 400 --timeout-method thread > gpurun_out/c5_tests.log 2>&1
echo ok c5 tests

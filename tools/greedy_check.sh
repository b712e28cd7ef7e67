#!/bin/bash
# greedy kernels: parity tests + one bench step
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_sharded.py tests/test_gpu_tf_variant.py tests/test_gpu_fullsize.py tests/test_integration_stub.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gr_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 > gpurun_out/gr_bench.log 2>&1
echo ok bench

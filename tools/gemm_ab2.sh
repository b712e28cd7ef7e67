#!/bin/bash
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_placement.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/gemm_layouts.py > gpurun_out/layouts.jsonl 2>&1
echo ok layouts
timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --steps 2 --warmup 1 > gpurun_out/ab2_bench.log 2>&1
echo ok bench

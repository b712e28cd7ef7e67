#!/bin/bash
# kernel assembly: parity tests + C2 line (assembly GB/s) + one bench step
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_gp.py tests/test_gpu_placement.py -x -q --timeout 200 --timeout-method thread > gpurun_out/km_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['bench.py']; import bench, torch; torch.cuda.set_device(0)
print(json.dumps(bench.c2_line(reps=3)))" > gpurun_out/km_c2.log 2>&1
echo ok c2

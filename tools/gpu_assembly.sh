#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 5 200 python tools/bench_assembly.py > gpurun_out/assembly.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kernel or covariance or local or c2 or matvec or gp" > gpurun_out/assembly_tests.log 2>&1

#!/bin/bash
# Round 4, call B: the sharded GPU tests (backend built on an unassembled Sigma), then the full
# default bench line with the per-class GEMM breakdown.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > $O/sharded_tests.log 2>&1
echo ok tests
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log > $O/bench_line.json
echo ok bench

#!/bin/bash
# Round 4, call D: C4 rounds as two launches, parallel refinement end, fast top-B, the 7-point CG
# on the Manhattan ball, bounds neighbour slots in registers: tests + timing per batch size, and
# the bounds A/B (neighbour slots read from LDS: tools/variants/lib_nbl.so).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 8 16 32 > $O/c4_time.jsonl 2> $O/c4_time.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_nbl.so timeout -k 10 300 python -u tools/c4_time.py 16 32 > $O/c4_time_nbl.jsonl 2> $O/c4_time_nbl.err
echo ok ab

#!/bin/bash
# Round 5, call J: grouped bounds grid capped at 16,384, the stall kernel's top-B merge by rank:
# C4 GPU tests, the 128^3 run (3 x 10 runs), stall / step / window stamps.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 120 python -u tools/exact_dbg.py > $O/c4_dbg.json 2>&1
echo ok dbg

#!/bin/bash
# Round 5, call Q: the 7-point CG as one launch per iteration (VGPOSP_CG_AB=1: part B of it - 1 and
# part A of it together, |r|^2 by recurrence): C4 GPU tests on the variant, then 128^3 timings
# against the product.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
VGPOSP_LIB=$R/tools/variants/lib_cgab.so timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_cgab.log 2>&1 || echo "tests failed"
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$R/tools/variants/lib_cgab.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"cgab\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4

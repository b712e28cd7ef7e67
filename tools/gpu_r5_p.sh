#!/bin/bash
# Round 5, call P: the CG start kernel clearing r / p0 / p1 only on the Manhattan ball it can read
# (product) against the whole box (fullzero); the CG walk at 8 / 32 lanes per diamond row (seg8 /
# seg32) against 16.  C4 GPU tests on the product first.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5p
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  for v in fullzero seg8 seg32; do
    VGPOSP_LIB=$R/tools/variants/lib_$v.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4

#!/bin/bash
# Round 5, call W: the CG start kernel on the CG columns' XCD mapping (product) against the
# previous commit (lib_prev); the window kernel's working workgroups all on XCD 0, beside the
# single-workgroup step kernel that reads what they write (x0c2 / x0c4: 2 / 4 candidates per
# workgroup).  C4 GPU tests on the product and on x0c2 first.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5w
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
VGPOSP_LIB=$R/tools/variants/lib_x0c2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_x0c2.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  for v in prev x0c2 x0c4; do
    VGPOSP_LIB=$R/tools/variants/lib_$v.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4

#!/bin/bash
# Round 5, call K: the whole CG solve of a column in one workgroup (VGPOSP_CG_WG=1 variant) against
# the per-phase launches: C4 GPU tests on the variant, then interleaved 128^3 timings.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
V=$R/tools/variants/lib_cgwg.so
VGPOSP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_cgwg.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$V timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"cgwg\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4

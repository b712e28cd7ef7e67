#!/bin/bash
# Round 5, call Y: the step kernel issues the window entries. loads before the block-key staging and the
# window list before the superblock-key copy: C4 GPU tests on this
# build, then 128^3 timings against the previous commit (lib_prev).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5y
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"prev\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4

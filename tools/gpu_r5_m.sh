#!/bin/bash
# Round 5, call M: the window kernel at 14 candidates per workgroup (1,024 threads), and with the
# next round's step fused into its last workgroup (ticket after a device-scope fence): C4 GPU tests
# on the fused variant, then 128^3 timings interleaved with the product.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5m
mkdir -p $O
cd $R
VGPOSP_LIB=$R/tools/variants/lib_fuse.so timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_fuse.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  for v in win14 fuse; do
    VGPOSP_LIB=$R/tools/variants/lib_$v.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4

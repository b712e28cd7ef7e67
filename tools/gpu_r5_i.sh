#!/bin/bash
# Round 5, call I: the bounds decode by multiply-high division; grid caps 65,536 (product) /
# 16,384 / 8,192 workgroups for the grouped bounds launch.  C4 GPU tests first.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  for v in product grid16384 grid8192; do
    if [ $v = product ]; then L=$R/vgposp_amd/libvgposp.so; else L=$R/tools/variants/lib_$v.so; fi
    VGPOSP_LIB=$L timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 \
      | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4 ab

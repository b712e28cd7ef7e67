#!/bin/bash
# Round 5, call F: factor rows read through LDS-typed pointers (ds_read, not flat loads) in the
# window / rows kernels: C4 GPU tests, the 128^3 run against lib_bnda2, stamps, then one full
# default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  for v in product bnda2; do
    if [ $v = product ]; then L=$R/vgposp_amd/libvgposp.so; else L=$R/tools/variants/lib_$v.so; fi
    VGPOSP_LIB=$L timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 \
      | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4 ab
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 120 python -u tools/exact_dbg.py > $O/c4_dbg.json 2>&1
echo ok dbg
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log > $O/bench.json
echo ok bench

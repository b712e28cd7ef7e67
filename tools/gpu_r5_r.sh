#!/bin/bash
# Round 5, call R: the stall kernel's top-B with coalesced chunk-interleaved item loads, an
# unrolled rank merge and a parallel output; the slot ranking unrolled and the batch write by
# one wave: C4 GPU tests on this build, level stamps (-DVGPOSP_EXACT_DBG=3), then 128^3 timings
# against the previous commit (lib_prev).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
VGPOSP_LIB=$R/tools/variants/lib_dbg3.so timeout -k 10 200 python tools/exact_dbg.py --dbg3 > $O/dbg3.json 2> $O/dbg3.err
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"prev\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4

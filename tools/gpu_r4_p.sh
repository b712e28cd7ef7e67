#!/bin/bash
# Round 4, call P: interleaved two-pass top-B, pre-tightening of the round-0 top candidates (two
# bound levels): C4 parity, timing of one level and of two levels by first-level bracket and
# pre-tightened count, phase stamps.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4p
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
for lt in 3e-5 5e-4; do
  for pt in 0 4096 16384; do
    timeout -k 10 300 python -u tools/c4_time.py --two-level --lo-target $lt --pt $pt 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
  done
done
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py --one-level > $O/dbg1.json 2> $O/dbg1.err
echo ok dbg

#!/bin/bash
# Round 4, call Q: three-pass radix select for the pre-tightening, two bound levels by default:
# C4 parity, timing by pre-tightened count, one level beside it.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4q
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
for pt in 4096 2048 8192; do
  timeout -k 10 300 python -u tools/c4_time.py --pt $pt 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
done
timeout -k 10 300 python -u tools/c4_time.py --one-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py > $O/dbg2.json 2> $O/dbg2.err
echo ok dbg

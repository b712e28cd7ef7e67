#!/bin/bash
# Round 4, call J: encoded (branch-free) key arg-max, deduplicated window keys: checks, C4 parity,
# timing, phase stamps; the leading-dimension A/B of the 65k Cholesky + inverse.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -v --timeout 120 --timeout-method thread > $O/wave_test.log 2>&1
echo ok wave
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_placement.py tests/test_gpu_tf_variant.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --one-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py --one-level > $O/dbg1.json 2> $O/dbg1.err
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py > $O/dbg2.json 2> $O/dbg2.err
echo ok dbg
timeout -k 10 400 python -u tools/lda_ab.py 65536 0 64 128 > $O/lda65k.jsonl 2> $O/lda65k.err
echo ok lda65k

#!/bin/bash
# Round 4, call N: two-pass top-B of the stall kernel: C4 parity, timing (one / two levels), phase
# stamps; then the round-4 profiles (tools/profile_r4.sh, PMC passes without kernel filters: the
# filtered FETCH_SIZE pass of call M died in rocprofv3's dispatch hook, SIGSEGV on the first
# copy_leaf_kernel launch).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --two-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py --one-level > $O/dbg1.json 2> $O/dbg1.err
echo ok dbg
bash $R/tools/profile_r4.sh
echo ok profile

#!/bin/bash
# Round 4, call K: component-wise key selects (no scratch), CG walk with 4 diamond rows per wave,
# Gauss-Radau bounds (A/B: Chebyshev):
# checks, C4 parity, timing (and the one-row-per-wave CG as A/B), phase stamps.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4k
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -v --timeout 120 --timeout-method thread > $O/wave_test.log 2>&1
echo ok wave
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_placement.py tests/test_gpu_tf_variant.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --one-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --cheb 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --cheb --one-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
VGPOSP_LIB=$R/tools/variants/lib_seg64.so timeout -k 10 300 python -u tools/c4_time.py --one-level 32 > $O/c4_time_seg64.jsonl 2> $O/c4_time_seg64.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py > $O/dbg2.json 2> $O/dbg2.err
echo ok dbg
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/timeline.py $O/tr/c4_kernel_trace.csv --marker exact_gersh_final --step -1 > $O/c4_timeline.txt
rm -rf $O/tr
echo ok trace

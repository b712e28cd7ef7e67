#!/bin/bash
# Round 4, call L: 32-bit bounds index math with hoisted offsets, the pick's factor rows computed
# in the window kernel: C4 parity, timing (one / two levels), phase stamps, one kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4l
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --two-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py --one-level > $O/dbg1.json 2> $O/dbg1.err
echo ok dbg
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/timeline.py $O/tr/c4_kernel_trace.csv --marker exact_gersh_final --step -1 > $O/c4_timeline.txt
rm -rf $O/tr
echo ok trace

#!/bin/bash
# Round 4, call H: DPP / permlane wave reductions (no ds_bpermute): bit-identity check, C4 and
# greedy parity, C4 timing (one and two bound levels), one kernel trace.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4h
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -v --timeout 120 --timeout-method thread > $O/wave_test.log 2>&1
echo ok wave
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py tests/test_gpu_placement.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py --one-level 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o c4 -- python3 $R/tools/c4_time.py --reps 1 --one-level 32 > $O/c4.log 2>&1
python3 $R/tools/timeline.py $O/tr/c4_kernel_trace.csv --marker exact_gersh_final --step -1 > $O/c4_timeline.txt
rm -rf $O/tr
echo ok trace
cd $R
VGPOSP_LIB=$R/tools/variants/lib_wpe4.so timeout -k 10 300 python -u tools/c4_time.py --one-level 32 > $O/c4_time_wpe4.jsonl 2> $O/c4_time_wpe4.err
echo ok wpe4

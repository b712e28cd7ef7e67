#!/bin/bash
# Round 5, call V: the CG columns of a batch mapped one XCD per column (its blocks on workgroup ids = j mod 8): C4 GPU tests, then 128^3 timings
# against the previous commit (lib_prev), and the start kernel's duration under --kernel-trace.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5v
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"prev\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/rocprof_summary.py $O/c4/c4_kernel_stats.csv $O/c4_summary.txt 25 > /dev/null
rm -f $O/c4/c4_kernel_trace.csv
echo ok stats

#!/bin/bash
# Round 4, call S: the radix select's pick kernel as one wave over LDS; the bounds launch's
# workgroup cap (A/B 4,096 / 16,384 / 65,536), the re-score loads before the new row: C4 parity,
# timing; then the C5 launch timelines (tools/gpu_c5_timeline.sh).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
for g in 4096 16384; do
  VGPOSP_LIB=$R/tools/variants/lib_grid$g.so timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
done
timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
bash $R/tools/gpu_c5_timeline.sh
echo ok c5

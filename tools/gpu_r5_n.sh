#!/bin/bash
# Round 5, call N: window candidates per workgroup 1 / 2 / 3 / 6 against the product's 4
# (128^3 k = 50 timings interleaved, 2 repeats; picks checked in every run).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5n
mkdir -p $O
cd $R
for rep in 1 2; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  for v in win1 win2 win3 win6; do
    VGPOSP_LIB=$R/tools/variants/lib_$v.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4

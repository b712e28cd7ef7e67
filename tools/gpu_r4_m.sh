#!/bin/bash
# Round 4, call M: the one-level bracket target (K = 3 / 4 / 5 Radau steps) on the current build,
# then the round-4 profiles (tools/profile_r4.sh: rocprof summary of one 65k step, PMC traffic of
# the GEMM / mat-vec / assembly and of the C4 kernels).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
for t in 3e-5 1e-6 4e-8; do
  timeout -k 10 300 python -u tools/c4_time.py --target $t 32 >> $O/c4_target.jsonl 2>> $O/c4_target.err
done
echo ok target
bash $R/tools/profile_r4.sh
echo ok profile

#!/bin/bash
# Round 4, call I: phase stamps inside the C4 stall / step kernels (debug build), and the
# leading-dimension A/B of the 65k Cholesky + inverse.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4i
mkdir -p $O
cd $R
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py --one-level > $O/dbg1.json 2> $O/dbg1.err
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 300 python -u tools/exact_dbg.py > $O/dbg2.json 2> $O/dbg2.err
echo ok dbg
timeout -k 10 400 python -u tools/lda_ab.py 65536 0 64 128 > $O/lda65k.jsonl 2> $O/lda65k.err
echo ok lda65k
timeout -k 10 200 python -u tools/lda_ab.py 32768 0 64 > $O/lda32k.jsonl 2> $O/lda32k.err
echo ok lda32k

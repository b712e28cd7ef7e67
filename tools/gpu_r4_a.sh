#!/bin/bash
# Round 4, call A: the GPU suite on the round-4 tree (epsilon-local path retired, no environment
# switches, alg-3 reference-arithmetic fixtures), then the original round-3 crash sweep once on
# the fixed build (explicit split depth and streams), under faulthandler: C3 and C5 mixed.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4a
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -X faulthandler -u tools/vgp_ab.py streams=1,0 split=64,32,16 > $O/ab_splitk_c3.jsonl 2> $O/ab_splitk_c3.err
echo ok c3
timeout -k 10 300 python -X faulthandler -u tools/vgp_ab.py --c5 --mixed streams=7,1,0 split=64,32,16 > $O/ab_splitk_c5m.jsonl 2> $O/ab_splitk_c5m.err
echo ok c5m

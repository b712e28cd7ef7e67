#!/bin/bash
# Round-4 reproduction of the round-3 host segfault (gpurun_out/call_ab2.txt, rc 139) on the
# UNCHANGED round-3 build, once, under faulthandler so that the Python stack of the crash is kept.
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/segv
mkdir -p $O
cd $R
timeout -k 10 300 python -X faulthandler -u tools/vgp_ab.py VGPOSP_VGP_STREAMS=1,0 VGPOSP_SPLIT_MIN_K=64,32,16 > $O/ab_c3.jsonl 2> $O/ab_c3.err
rc=$?
echo "rc=$rc"
tail -60 $O/ab_c3.err
exit $rc

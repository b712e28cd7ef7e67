#!/bin/bash
# C3 / C5 step times with the fused softplus parameter launches on / off (tools/vgp_ab.py).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/vgp_ab.py VGPOSP_FUSED_PARAMS=1,0 > $O/q_c3.jsonl 2>$O/q_c3.err
timeout -k 10 200 python -u tools/vgp_ab.py --c5 VGPOSP_FUSED_PARAMS=1,0 > $O/q_c5.jsonl 2>$O/q_c5.err
echo ok times

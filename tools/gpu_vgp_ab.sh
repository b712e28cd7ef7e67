#!/bin/bash
# One-process A/Bs (tools/vgp_ab.py) of the VGP step's side streams per segment (bitmask
# VGPOSP_VGP_STREAMS: 1 Kzb, 2 middle chains, 4 tail VJPs / reductions), split depth 16.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
export VGPOSP_SPLIT_MIN_K=16
timeout -k 10 200 python -u tools/vgp_ab.py VGPOSP_VGP_STREAMS=0,1,2,4,7 > $O/ab2_c3.jsonl 2>$O/ab2_c3.err
echo ok c3
timeout -k 10 200 python -u tools/vgp_ab.py --c5 VGPOSP_VGP_STREAMS=0,1,2,4,7 > $O/ab2_c5.jsonl 2>$O/ab2_c5.err
echo ok c5
timeout -k 10 200 python -u tools/vgp_ab.py --c5 --mixed VGPOSP_VGP_STREAMS=0,2,4,7 > $O/ab2_c5m.jsonl 2>$O/ab2_c5m.err
echo ok c5m

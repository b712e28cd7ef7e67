#!/bin/bash
# A/B of the VGP step's side streams (VGPOSP_VGP_STREAMS=0: every launch on the main stream),
# C3 and C5 (Matern 5/2) fp64 and C5 mixed:2, three interleaved repeats.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
: > $O/vgp_ab.txt
for rep in 1 2 3; do
  for st in 1 0; do
    for cfg in "" "--c5 --kernel matern52" "--c5 --kernel matern52 --mixed --mixed-iters 2"; do
      ms=$(VGPOSP_VGP_STREAMS=$st timeout -k 10 120 python -u tools/bench_vgp.py $cfg 2>/dev/null | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
      echo "rep=$rep streams=$st cfg='$cfg' ms=$ms" | tee -a $O/vgp_ab.txt
    done
  done
done

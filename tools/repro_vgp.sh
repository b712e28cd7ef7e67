#!/bin/bash
# The graph-replay status check of the VGP step: back-to-back replays in bench.py's loop shape
# (tools/repro_vgp2.py), against the eager step.  Both lines must print the same losses.
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/repro_vgp2.py plain > gpurun_out/rep1.log 2>&1; echo rc1=$?
VGPOSP_GRAPH=0 timeout -k 10 200 python -u tools/repro_vgp2.py plain > gpurun_out/rep2.log 2>&1; echo rc2=$?

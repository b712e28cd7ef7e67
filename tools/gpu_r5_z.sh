#!/bin/bash
# Round 5, call Z: the 128-leaf's panel factor broadcasting each scaled column through LDS instead
# of a v_readlane pair per row: leaf phase stamps (stamped build), the linear-algebra / placement /
# VGP GPU tests on the product, then the 65k step and C3 / C5 timings.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5z
mkdir -p $O
cd $R
VGPOSP_LIB=$R/tools/variants/lib_stamps.so timeout -k 10 200 python tools/leaf_probe.py > $O/leaf_probe.json 2> $O/leaf_probe.err
echo ok probe
timeout -k 10 900 python -u -m pytest tests/test_gpu_linalg.py tests/test_gpu_placement.py tests/test_gpu_vgp_train.py tests/test_gpu_gp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
timeout -k 10 600 python -u bench.py --no-cpu --no-c4 --no-sweep --no-c2 --vgp-steps 20 > $O/bench.log 2>&1
grep "^{" $O/bench.log > $O/bench.json
echo ok bench

#!/bin/bash
# VGP step iteration on the GPU box: the VGP GPU tests, the C3 / C5 / C5-mixed step times, then
# the launch timeline of one graph-replayed C3 and C5 step (tools/gpu_vgp_timeline.sh).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_vgp_train.py tests/test_gpu_configs.py tests/test_gpu_mixed.py tests/test_gpu_vgp_dp.py -x -q --timeout 200 --timeout-method thread > $O/vgp_tests.log 2>&1
echo ok tests
timeout -k 10 120 python -u tools/bench_vgp.py > $O/vgp_c3.json 2>/dev/null
timeout -k 10 120 python -u tools/bench_vgp.py --c5 --kernel matern52 > $O/vgp_c5.json 2>/dev/null
timeout -k 10 120 python -u tools/bench_vgp.py --c5 --kernel matern52 --mixed --mixed-iters 2 > $O/vgp_c5m.json 2>/dev/null
echo ok bench
bash tools/gpu_vgp_timeline.sh

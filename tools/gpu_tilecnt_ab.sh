#!/bin/bash
# Round-6 A/B of the in-launch split-K reduction (gemm.hip tile_cnt) against the previous build
# (tools/variants/lib_head.so): GPU parity subset, the 65k step twice each, the per-rank R = 8 step.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/tcab
mkdir -p $O
tools/gpu_ab.sh $O --tests "tests/test_gpu_linalg.py tests/test_gpu_placement.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_exact.py" default
for i in 1 2; do
  for lib in head default; do
    if [[ $lib == default ]]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/lib_head.so; fi
    timeout -k 10 400 python -u bench.py --no-cpu --no-vgp --no-c2 --no-c4 --no-sweep --steps 2 --warmup 1 > $O/step_${lib}_$i.json 2> $O/step_${lib}_$i.err
    echo "$lib $i $(cut -c1-140 $O/step_${lib}_$i.json)"
  done
done
for lib in head default; do
  if [[ $lib == default ]]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/lib_head.so; fi
  timeout -k 10 300 python -u tools/bench_sharded_step.py --ranks 8 --out $O/sharded_$lib.json > $O/sharded_$lib.log 2>&1
  echo "$lib sharded $(tail -1 $O/sharded_$lib.log)"
done

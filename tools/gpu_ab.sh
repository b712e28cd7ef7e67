#!/bin/bash
# A/B of libvgposp builds on ONE GPU box (the parameterised replacement of the per-call
# tools/gpu_r*_*.sh one-offs).  Usage, from the repo root on the box:
#   tools/gpu_ab.sh OUT_DIR [--tests "pytest files"] [--gemm] [--step] LIB...
# LIB is "default" (the in-tree libvgposp.so) or a path to a variant .so (VGPOSP_LIB).  For every
# LIB: the GPU tests named by --tests (parity first: any failure stops the script), the 16384^3
# layout sweep + 8192^3 NT (--gemm), the 65k placement step (--step: bench.py main line only,
# 2 timed steps).  Every GPU step has its own time limit;
# the first failure ends the script (set -e).
set -euo pipefail
out=$1; shift
tests=""; gemm=0; step=0
while [[ $# -gt 0 && $1 == --* ]]; do
  case $1 in
    --tests) tests=$2; shift 2 ;;
    --gemm) gemm=1; shift ;;
    --step) step=1; shift ;;
    *) echo "unknown option $1"; exit 2 ;;
  esac
done
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p "$out"
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  if [[ $lib == default ]]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/$lib; fi
  if [[ -n $tests ]]; then
    timeout -k 10 600 python -u -m pytest $tests -x -q --timeout 300 --timeout-method thread \
      > "$out/tests_$tag.log" 2>&1
    echo "tests ok $tag: $(tail -1 "$out/tests_$tag.log")"
  fi
  if [[ $gemm == 1 ]]; then
    timeout -k 10 300 python -u tools/gemm_layouts.py > "$out/layouts_$tag.jsonl" 2>&1
    timeout -k 10 120 python -u -c "
import sys, json; sys.path.insert(0, 'tools'); sys.path.insert(0, '.')
from bench_gemm import run
print(json.dumps(run(8192, 8192, 8192, 0, 1, False, 0.0, reps=5)))" >> "$out/layouts_$tag.jsonl" 2>&1
    echo "gemm ok $tag"
  fi
  if [[ $step == 1 ]]; then
    timeout -k 10 400 python -u bench.py --no-cpu --no-vgp --no-c2 --no-c4 --no-sweep --steps 2 \
      --warmup 1 > "$out/step_$tag.json" 2> "$out/step_$tag.err"
    echo "step ok $tag: $(cut -c1-160 "$out/step_$tag.json")"
  fi
done

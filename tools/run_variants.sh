#!/bin/bash
# A/B timing of library builds on one box: the current build (BMW 2 and BMW 1) and any
# tools/variants/*.so, 8192^3 NT GEMM + the 65k Cholesky+inverse.
run() {
  timeout -k 10 200 python tools/bench_gemm.py > /tmp/bg.txt 2>/dev/null || exit 1
  grep '"m": 8192, "n": 8192, "k": 8192, "ta": 0' /tmp/bg.txt | cut -c100-170
  timeout -k 10 200 python tools/prof_overhead.py 2>/dev/null || exit 1
}
for round in 1 2; do
  echo "== current"; unset VGPOSP_GEMM_BMW; unset VGPOSP_LIB; run
  echo "== current BMW2"; export VGPOSP_GEMM_BMW=2; run; unset VGPOSP_GEMM_BMW
  for lib in tools/variants/*.so; do [ -e "$lib" ] || continue; echo "== $lib"; VGPOSP_LIB=$PWD/$lib run; done
done

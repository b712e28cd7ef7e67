#!/bin/bash
# A/B timing of library build variants (tools/variants/*.so) on the GPU box.
for lib in vgposp_amd/libvgposp.so tools/variants/*.so; do
  echo "== $lib"
  VGPOSP_LIB=$PWD/$lib timeout -k 10 200 python tools/bench_gemm.py > /tmp/bg.txt 2>/dev/null || exit 1
  grep '"m": 8192' /tmp/bg.txt | head -2
  VGPOSP_LIB=$PWD/$lib timeout -k 10 200 python tools/prof_overhead.py 2>/dev/null || exit 1
done

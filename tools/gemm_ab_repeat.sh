#!/bin/bash
# Interleaved repeats of the 65k placement step for the default build and one GEMM variant.
set -e
cd ${GRAFT_REPO_ROOT:-$PWD}; mkdir -p gpurun_out
out=gpurun_out/$1; var=$2; reps=${3:-3}
for i in $(seq $reps); do
  for lib in default $var; do
    if [ $lib = default ]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/$lib.so; fi
    v=$(timeout -k 10 300 python -u bench.py --no-cpu --no-vgp --no-c2 --no-c4 --no-sweep --steps 2 --warmup 1 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'])")
    echo "$lib $v" >> $out
  done
done

#!/bin/bash
# PMC passes (one counter per run) over one timed bench step, GEMM kernels only
cd ${GRAFT_REPO_ROOT:-$PWD}; R=$PWD; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --steps 1 --warmup 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex gemm_glds --output-format csv -d $R/gpurun_out/pmcg_$c -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcg_$c.log 2>&1
  echo "rc $c $?"
done
ls -la $R/gpurun_out/pmcg_FETCH_SIZE/ 2>/dev/null | head

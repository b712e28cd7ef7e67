#!/bin/bash
# Round 5, call B: the grouped bounds kernel (G candidates per wave, exact_bounds_grp_kernel)
# against the one-candidate-per-wave kernel (G = 1): bounds GPU tests under each variant, then
# the 128^3 k = 50 run time, variants interleaved, three repeats.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
for G in 8 4 2; do
  VGPOSP_LIB=$R/tools/variants/lib_bndg$G.so timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -x -q \
    -k "bounds or bounded or regression or two_bound" --timeout 200 --timeout-method thread > $O/tests_g$G.log 2>&1
  echo "ok tests G=$G"
done
for rep in 1 2 3; do
  for G in 1 8 4 2; do
    VGPOSP_LIB=$R/tools/variants/lib_bndg$G.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 \
      | sed "s/^{/{\"G\": $G, \"rep\": $rep, /" >> $O/c4_bndg.jsonl
  done
done
echo done
# the 65k step without PyTorch (tools/step65k.cpp): timing + picks, then its GEMM PMC passes
(while sleep 45; do echo "heartbeat $(date +%T)"; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 120 tools/_build/step65k tools/_build/x65k.bin 2 50 > $O/step65k.json 2> $O/step65k.log
echo ok step65k
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o p -- $R/tools/_build/step65k $R/tools/_build/x65k.bin 1 50 > $O/pmc_$c.log 2>&1
  echo "ok pmc $c"
done
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
  --kernel-include-regex gemm_glds --output-format csv -d $O/pmc_gemm_sq -o p -- $R/tools/_build/step65k $R/tools/_build/x65k.bin 1 50 > $O/pmc_gemm_sq.log 2>&1
echo "ok pmc gemm sq"

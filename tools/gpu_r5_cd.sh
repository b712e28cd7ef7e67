#!/bin/bash
# Round 5, calls C + D in one: the GPU suite on this tree (column-oriented re-scores, window
# kernel overlap, pick records, grouped bounds with neighbour addresses); bounds A/B (G = 1 / 2 /
# 4); window A/B (this tree against lib_bnda2: same bounds, previous window kernel); the window
# kernel's stamps; the PyTorch-free 65k step's WRITE_SIZE and GEMM SQ passes.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5c
mkdir -p $O
cd $R
(while sleep 45; do echo "heartbeat $(date +%T)"; done) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  for v in product bndg1 bnda2 bnda4; do
    if [ $v = product ]; then L=$R/vgposp_amd/libvgposp.so; else L=$R/tools/variants/lib_$v.so; fi
    VGPOSP_LIB=$L timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 \
      | sed "s/^{/{\"variant\": \"$v\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  done
done
echo ok c4 ab
VGPOSP_LIB=$R/tools/variants/lib_dbg.so timeout -k 10 120 python -u tools/exact_dbg.py > $O/c4_dbg_new.json 2>&1
VGPOSP_LIB=$R/tools/variants/lib_dbg_old.so timeout -k 10 120 python -u tools/exact_dbg.py > $O/c4_dbg_old.json 2>&1
echo ok dbg
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_WRITE_SIZE -o p -- $R/tools/_build/step65k $R/tools/_build/x65k.bin 1 50 > $O/pmc_WRITE_SIZE.log 2>&1
echo "ok pmc WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM \
  --kernel-include-regex gemm_glds --output-format csv -d $O/pmc_gemm_sq -o p -- $R/tools/_build/step65k $R/tools/_build/x65k.bin 1 50 > $O/pmc_gemm_sq.log 2>&1
echo "ok pmc gemm sq"

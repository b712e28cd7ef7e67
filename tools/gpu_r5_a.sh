#!/bin/bash
# Round 5, call A: the GPU suite on this tree (new GPRM fixture test, k = 110 bounded case,
# reduce_keys guard), the bench's own rank launcher rehearsed with 2 gloo ranks on one GPU, the
# C4 bounds pass's SQ counters, then (LAST: it may die) the PMC SIGSEGV probe with the maps dump.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
VGPOSP_BENCH_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 1 --warmup 1 \
  --no-cpu --no-vgp --no-sweep --no-c4-selinv --no-splits --no-c2 > $O/bench_2ranks.log 2>&1
grep "^{" $O/bench_2ranks.log > $O/bench_2ranks.json
echo ok launcher
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES \
  --kernel-include-regex exact_bounds --output-format csv -d $O/c4sq -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4sq.log 2>&1
echo ok c4 sq
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 \
  --kernel-include-regex exact_bounds --output-format csv -d $O/c4sq2 -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4sq2.log 2>&1 || echo "c4 sq2 rc $?"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/probe -o p -- \
  python3 $R/tools/pmc_segv_probe.py $O/segv_maps.txt 4096 16384 65536 > $O/probe.log 2>&1
echo ok probe

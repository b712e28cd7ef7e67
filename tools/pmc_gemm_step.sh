#!/bin/bash
# PMC of the GEMM instantiations over ONE 65k placement step (the actual tri-A / tri-B / NT step
# shapes, not a square benchmark): MFMA busy and wave wait fractions, one counter group per run.
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex gemm_glds --output-format csv -d $R/gpurun_out/pmcs_a -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcs_a.log 2>&1
echo "rc a $?"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex gemm_glds --output-format csv -d $R/gpurun_out/pmcs_b -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmcs_b.log 2>&1
echo "rc b $?"
python3 $R/tools/pmc_gemm_step.py $R/gpurun_out/pmcs_a $R/gpurun_out/pmcs_b > $R/gpurun_out/pmc_gemm_step.txt 2>&1
echo "rc py $?"

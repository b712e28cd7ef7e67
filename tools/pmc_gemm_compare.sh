set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcg
for prog in gemm_one vendor_gemm_one; do
  timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmcg/${prog}_a -- python3 $R/tools/$prog.py > $R/gpurun_out/pmcg/${prog}_a.log 2>&1
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmcg/${prog}_b -- python3 $R/tools/$prog.py > $R/gpurun_out/pmcg/${prog}_b.log 2>&1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmcg/${prog}_t -- python3 $R/tools/$prog.py > $R/gpurun_out/pmcg/${prog}_t.log 2>&1
done

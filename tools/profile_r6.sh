#!/bin/bash
# Round-6 profiling on the GPU box (outputs under gpurun_out/r6prof; summaries copied to profiles/):
#  1. rocprofv3 --kernel-trace --stats of the bench's 65k placement step (C4 / VGP / sweep off);
#  2. the PyTorch-free 65k step (tools/step65k.cpp, per-phase progress lines on stderr) under
#     --pmc FETCH_SIZE and --pmc WRITE_SIZE (HBM traffic, tools/pmc_traffic.py) and under
#     MFMA-busy counters for the GEMM instantiations (tools/pmc_sum.py);
#  3. C4 (128^3, k = 50): kernel-trace stats, FETCH / WRITE / TCC passes (tools/pmc_c4.py, hash-tied
#     to exact_greedy.hip) and the SQ counters of the shipped bounds kernel.
# Every GPU step has its own kill timeout; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r6prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-vgp --no-potrf --no-c2 --no-c4 --no-splits --no-sweep --steps 1 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o bench -- python3 $R/bench.py $ARGS > $O/step.log 2>&1
python3 $R/tools/rocprof_summary.py $O/step/bench_kernel_stats.csv $O/step_summary.txt > /dev/null
grep "^{" $O/step.log > $O/step_line.json
echo ok step
S="$R/tools/_build/step65k $R/tools/_build/x65k.bin 1 50"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/s65_fetch -o p -- $S > $O/s65_fetch.log 2>&1
echo ok fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/s65_write -o p -- $S > $O/s65_write.log 2>&1
echo ok write
python3 $R/tools/pmc_traffic.py $(ls $O/s65_fetch/*counter_collection.csv | head -1) $(ls $O/s65_write/*counter_collection.csv | head -1) --N 65536 --shape 64 32 32 --k 50 --out $O/traffic_r6.json > $O/traffic.txt
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex gemm_glds --output-format csv -d $O/s65_mfma -o p -- $S > $O/s65_mfma.log 2>&1
python3 $R/tools/pmc_sum.py $O/r6_pmc_gemm_mfma.json $(ls $O/s65_mfma/*counter_collection.csv | head -1) --command "rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex gemm_glds -- tools/_build/step65k tools/_build/x65k.bin 1 50" --note "dispatch-summed over one 65k placement step" > $O/pmc_gemm_mfma.txt
echo ok mfma
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4.log 2>&1
python3 $R/tools/rocprof_summary.py $O/c4/c4_kernel_stats.csv $O/c4_summary.txt 25 > /dev/null
echo ok c4 stats
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc_$n -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4pmc_$n.log 2>&1
  echo ok c4 pmc $n
done
python3 $R/tools/pmc_c4.py $(ls $O/c4pmc_FETCH_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_WRITE_SIZE/*counter_collection.csv | head -1) $(ls $O/c4pmc_TCC_HIT_sum/*counter_collection.csv | head -1) --runs 3 --out $O/pmc_c4_r6.json --command "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE|TCC_HIT_sum TCC_MISS_sum} -- python3 tools/c4_time.py --reps 1 32" > $O/pmc_c4.txt
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex exact_bounds --output-format csv -d $O/c4sq -o p -- python3 $R/tools/c4_time.py --reps 1 32 > $O/c4sq.log 2>&1
python3 $R/tools/pmc_sum.py $O/r6_pmc_c4_bounds_sq.json $(ls $O/c4sq/*counter_collection.csv | head -1) --command "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex exact_bounds -- python3 tools/c4_time.py --reps 1 32" --note "dispatch-summed over 3 runs of 128^3 k = 50 (c4_time.py's reps: warm-up + timed)" > $O/pmc_c4_sq.txt
echo done

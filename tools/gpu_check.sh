#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke(), the default bench line, and a rocprofv3
# kernel-trace summary of one timed bench step. Every GPU step is time-limited and the
# script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo ok smoke
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
grep "^{" $O/bench.log > $O/bench_line.json
echo ok bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 $R/bench.py --no-cpu --no-vgp --no-potrf --no-c2 --steps 1 --warmup 0 > $O/prof.log 2>&1
python3 $R/tools/rocprof_summary.py $O/prof/bench_kernel_stats.csv $O/prof_summary.txt > /dev/null
echo done

#!/bin/bash
# the round's evidence in one GPU call: GPU tests, smoke(), rocprof kernel trace + PMC traffic of
# one bench step, then the default bench line (which reads the fresh traffic file)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo ok smoke
bash tools/profile_r1.sh
cd $R
cp $O/traffic_r1.json profiles/traffic_r1.json
timeout -k 10 600 python -u bench.py > $O/bench_final.log 2>&1
grep "^{" $O/bench_final.log > $O/bench_final.json
echo final

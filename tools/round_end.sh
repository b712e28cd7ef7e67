#!/bin/bash
# The round's evidence in one GPU call: GPU tests, smoke(), then the default bench line.
# (Profiles: tools/profile_r2.sh, tools/pmc_gemm_step.sh, tools/gpu_vgp_timeline.sh.)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${ROUND_END_TAG:-r6end}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo ok smoke
timeout -k 10 600 python -u bench.py > $O/bench_final.log 2>&1
grep "^{" $O/bench_final.log > $O/bench_final.json
echo final

#!/bin/bash
# Round-6 check of the per-factorization partials area (potrf.hip PART_ELEMS / _BATCHED): the GPU
# suite, the VGP and headline lines against the 16 MB build (tools/variants/lib_part2.so, built
# by SRC=build/var/potrf_part2.hip tools/build_potrf_variant.sh part2), and the per-rank sharded step.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/partchk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests: $(tail -1 $O/gpu_tests.log)"
for i in 1 2; do
  for lib in default part2; do
    if [[ $lib == default ]]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/tools/variants/lib_part2.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu --no-c2 --no-c4 --no-sweep --steps 1 --warmup 1 > $O/${lib}_$i.json 2> $O/${lib}_$i.err
    python -c "import json; d=json.load(open('$O/${lib}_$i.json')); print('$lib', $i, round(d['value'],3), [round(d[k]['ms_per_step'],3) for k in ('vgp_c3','vgp_c5','vgp_c5_mixed')])"
  done
done
unset VGPOSP_LIB
timeout -k 10 300 python -u tools/bench_sharded_step.py --ranks 1 8 --out $O/sharded.json > $O/sharded.log 2>&1
tail -1 $O/sharded.log

#!/bin/bash
# A/B of GEMM runtime switches on one box: 8192^3 NT and the three 16384^3 triangular shapes.
run() { timeout -k 10 200 python tools/bench_gemm.py 2>/dev/null | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if d['k'] >= 8192: print(d['m'], d['ta'], d['tb'], d['lower'], d['tri'], round(d['tflops'], 2))
" || exit 1; }
for cfg in "$@"; do echo "== $cfg"; env $cfg bash -c "$(declare -f run); run" || exit 1; done

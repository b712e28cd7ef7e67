#!/bin/bash
# Round 4, call Y: the 7-point coefficient table written through LDS (exact_coef8_kernel):
# bounds bit-identical to the previous build
# (tools/variants/lib_prev.so), C4 timing A/B, then the final tree's evidence (tools/gpu_r4_v.sh:
# all GPU tests, smoke, bench line, C4 kernel stats and PMC).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/bnd_dump.py $O/bnd_new.npz > $O/bnd.log 2>&1
VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 300 python -u tools/bnd_dump.py $O/bnd_prev.npz >> $O/bnd.log 2>&1
python -c "
import numpy as np, sys
a, b = np.load('$O/bnd_new.npz'), np.load('$O/bnd_prev.npz')
bad = 0
for k in a.files:
    same = np.array_equal(a[k].view(np.int64), b[k].view(np.int64))
    bad += not same
    print(k, 'identical' if same else 'DIFFER %d' % (a[k] != b[k]).sum())
sys.exit(1 if bad else 0)
" >> $O/bnd.log 2>&1
rm -f $O/bnd_new.npz $O/bnd_prev.npz
echo ok bnd
timeout -k 10 300 python -u -m pytest tests/test_gpu_wave.py -x -v --timeout 120 --timeout-method thread > $O/wave_tests.log 2>&1
echo ok wave
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time
bash $R/tools/gpu_r4_v.sh

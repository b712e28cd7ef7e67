#!/bin/bash
# Round 4, call T: the tiled all-candidate bounds kernel (exact_bounds_tile_kernel): bounds
# bit-identical to the register kernel's (tools/variants/lib_notile.so), C4 parity, timing A/B.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/bnd_dump.py $O/bnd_tile.npz > $O/bnd.log 2>&1
VGPOSP_LIB=$R/tools/variants/lib_notile.so timeout -k 10 300 python -u tools/bnd_dump.py $O/bnd_notile.npz >> $O/bnd.log 2>&1
python -c "
import numpy as np
a, b = np.load('$O/bnd_tile.npz'), np.load('$O/bnd_notile.npz')
for k in a.files: print(k, 'identical' if np.array_equal(a[k].view(np.int64), b[k].view(np.int64)) else 'DIFFER %d' % (a[k] != b[k]).sum())
" >> $O/bnd.log 2>&1
rm -f $O/bnd_tile.npz $O/bnd_notile.npz
echo ok bnd
timeout -k 10 900 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -x -v --timeout 300 --timeout-method thread > $O/exact_tests.log 2>&1
echo ok tests
timeout -k 10 300 python -u tools/c4_time.py 32 > $O/c4_time.jsonl 2> $O/c4_time.err
VGPOSP_LIB=$R/tools/variants/lib_notile.so timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
timeout -k 10 300 python -u tools/c4_time.py 32 >> $O/c4_time.jsonl 2>> $O/c4_time.err
echo ok time

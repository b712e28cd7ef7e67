#!/bin/bash
# Round 5, call X: the coefficient rows and sigma_off on 32-bit grid coordinates (no 64-bit divisions; the
# same values): bounds bit-identity against the previous commit (lib_prev, tools/bnd_dump.py), C4 GPU
# tests, then 128^3 timings interleaved with lib_prev.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
timeout -k 10 120 python tools/bnd_dump.py $O/bnd_new.npz > $O/bnd_new.log 2>&1
VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 120 python tools/bnd_dump.py $O/bnd_prev.npz > $O/bnd_prev.log 2>&1
python -c "
import numpy as np
a=np.load('$O/bnd_new.npz'); b=np.load('$O/bnd_prev.npz')
print({k: bool(np.array_equal(a[k], b[k])) for k in a.files})
" > $O/bnd_identity.log 2>&1
rm -f $O/bnd_new.npz $O/bnd_prev.npz
echo ok identity
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_alg3_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo ok tests
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"product\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
  VGPOSP_LIB=$R/tools/variants/lib_prev.so timeout -k 10 120 python -u tools/c4_time.py --reps 10 32 | sed "s/^{/{\"variant\": \"prev\", \"rep\": $rep, /" >> $O/c4_ab.jsonl
done
echo ok c4

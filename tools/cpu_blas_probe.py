"""Which (N, BLAS threads) combinations of the CPU baseline's LAPACK calls crash numpy/scipy's
OpenBLAS on this host (CPU only, no GPU): each case in its own process.
python tools/cpu_blas_probe.py -> one line per case: N, threads, return code, seconds."""
import os
import subprocess
import sys
import time

CASE = r"""
import sys, time, numpy as np
sys.path.insert(0, {root!r})
from threadpoolctl import threadpool_limits
from oracle import gp as ogp, placement as op
from vgposp_amd.data_generation import grid_points, grid_spacing
shape = {shape!r}
X = grid_points(shape, jitter=0.05, seed=0)
S = ogp.kernel_matrix('eq', X, X, 1.0, 2 * grid_spacing(shape))[0]
S[np.diag_indices(len(X))] += 1e-2 + 1e-6
with threadpool_limits(limits={th}, user_api='blas'):
    op.placement_lazy_incremental(S, 50)
"""

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for shape in [(16, 16, 32), (16, 16, 16)]:
    for th in [256, 64, 32, 16]:
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-c",
                            CASE.format(root=root, shape=shape, th=th)],
                           capture_output=True, text=True, timeout=300)
        print(f"N={shape[0] * shape[1] * shape[2]} threads={th} rc={r.returncode} "
              f"{time.perf_counter() - t0:.1f}s {r.stderr.strip().splitlines()[-1:] if r.returncode else ''}",
              flush=True)

# the same LAPACK path with the thread count changed INSIDE one process (64, then 16, then 64)
SEQ = CASE.replace("with threadpool_limits(limits={th}, user_api='blas'):\n    op.placement_lazy_incremental(S, 50)",
                   "for th in (64, 16, 64):\n    with threadpool_limits(limits=th, user_api='blas'):\n"
                   "        op.placement_lazy_incremental(S, 50)\n    print('ok', th, flush=True)")
if "--sequence" in sys.argv:
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c",
                        SEQ.format(root=root, shape=(16, 16, 32))],
                       capture_output=True, text=True, timeout=300)
    print("sequence 64 -> 16 -> 64 at N=8192:", r.returncode, r.stdout.split(), r.stderr[-300:])

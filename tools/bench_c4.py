"""Time config C4 (128^3 local-kernel greedy, k = 50) on one GPU: whole step, then the per-kernel
split from the library's event timing.  Usage: python tools/bench_c4.py [beta ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.local_placement import HipLocalBackend, LocalGreedyPlacement  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402

betas = [float(b) for b in sys.argv[1:]] or [4.0, 2.5]
X, shape, ls = c4_grid()
for beta in betas:
    b = HipLocalBackend(X, shape, 50, 3, beta, ls=ls, diag_shift=0.01 + 1e-6)
    g = LocalGreedyPlacement(b)
    for _ in range(2):
        g.run(50)
    torch.cuda.synchronize()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        g.run(50)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    _lib.prof_enable(True)
    g.run(50)
    prof = _lib.prof_dump()
    _lib.prof_enable(False)
    b.check()
    print(f"beta {beta} m {b.m}: {dt * 1e3:.3f} ms/step, {50 / dt:.0f} placements/s, "
          f"picks {b.picks[:4].tolist()}")
    for name, (ms, n, fl, by) in sorted(prof.items()):
        print(f"   {name:16s} {ms:8.3f} ms {n:4d} launches  {by / max(ms, 1e-9) / 1e6:9.1f} GB/s")

if os.environ.get("C4_PHASES"):
    import ctypes
    import numpy as np
    b = HipLocalBackend(X, shape, 50, 3, 4.0, ls=ls, diag_shift=0.01 + 1e-6)
    g = LocalGreedyPlacement(b)
    g.run(50)
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 64)()
    _lib.load().vgposp_local_debug_times(buf)
    t = np.array(buf[:], dtype=np.int64).reshape(8, 8)
    print("phase times (us) per round: touched, blocks, supers, reduce, pick+sync, window, sync")
    for r in range(1, 8):
        print(r, np.diff(t[r]) / 100.0, "round total", (t[r][7] - t[r][0]) / 100.0)

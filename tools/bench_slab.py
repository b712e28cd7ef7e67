"""Per-rank work of the candidate-sharded 65k placement on ONE GPU: for R = 1, 2, 4, 8 time every
rank's assembly + vgposp_greedy_init_slab (replicated Cholesky + its slab of L^-1) and its 50
rounds of slab updates (mat-vec + update over its columns, the pick taken from the full problem).
The max over ranks, plus the measured collectives' cost, predicts the N-GPU step (collectives are
not included here)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vgposp_amd import linalg  # noqa: E402
from vgposp_amd.sharded_placement import HipGreedyBackend, inverse_slabs  # noqa: E402
from vgposp_amd.workloads import placement_split  # noqa: E402

X, ls = placement_split((64, 32, 32), 0)
N, k = len(X), 50
Xd = linalg.as_device(X)
Sigma = torch.empty((N, N), dtype=torch.float64, device="cuda")
b = HipGreedyBackend(Sigma, k)


def assemble():
    linalg.kernel_matrix("eq", Xd, None, 1.0, ls, diag_shift=0.01 + 1e-6, out=Sigma[None])


# reference picks of the full problem (selected[] drives the slab rounds below)
assemble()
b.init()
for r in range(k):
    b.update(r, 0, N)
    b.select(r, True, 0, N)
picks = b.g.selected.clone()
for R in (1, 2, 4, 8):
    times = []
    for (c0, c1) in inverse_slabs(N, R):
        assemble()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.init_slab(c0, c1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        b.g.selected.copy_(picks)
        for r in range(k):
            if r:
                b.extract(r, 0, N)  # stands in for the xcol all-reduce (full column on one GPU)
            b.update(r, c0, c1, extract=False)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        times.append((t1 - t0, t2 - t1))
    tmax = max(a + r for a, r in times)
    print(f"R={R}: per-rank init+rounds (s) {[(round(a, 3), round(r, 3)) for a, r in times]} "
          f"-> max {tmax:.3f} s, {k / tmax:.1f} placements/s before collectives", flush=True)

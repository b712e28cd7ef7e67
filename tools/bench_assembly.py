"""Kernel-assembly rates (vgposp_kernel_matrix): the 65k placement Sigma (full, EQ), C2's 32^3
lower triangle (EQ), and the 65k full Sigma with Matern 5/2; GB/s of algorithmic bytes, best of 5."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vgposp_amd import linalg  # noqa: E402
from vgposp_amd.workloads import c2_data, placement_split  # noqa: E402


def rate(kind, X, ls, lower, reps=5):
    n, d = X.shape
    Xd = linalg.as_device(X)
    A = torch.empty((1, n, n), dtype=torch.float64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e30
    for _ in range(reps + 1):
        ev[0].record()
        linalg.kernel_matrix(kind, Xd, None, 1.0, ls, diag_shift=0.01 + 1e-6, lower=lower, out=A)
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]))
    nbytes = (4.0 * n * (n + 1) if lower else 8.0 * n * n) + 8.0 * d * n
    del A
    torch.cuda.empty_cache()
    return best, nbytes / (best * 1e-3) / 1e9


X, ls = placement_split((64, 32, 32), 0)
for kind in ("eq", "matern52"):
    ms, gbs = rate(kind, X, ls, False)
    print(f"65k full {kind:9s} {ms:7.3f} ms {gbs:8.1f} GB/s", flush=True)
X2, ls2 = c2_data()
ms, gbs = rate("eq", X2, ls2, True)
print(f"C2 32k lower eq   {ms:7.3f} ms {gbs:8.1f} GB/s", flush=True)

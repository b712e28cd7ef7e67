"""Time the fused 512-block kernel inside a plain potrf (n = 8192: 16 blocks) and check the factor.
  python tools/b512_probe.py   (run under rocprofv3 --kernel-trace --stats for per-kernel times)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import linalg  # noqa: E402

n = 8192
rng = np.random.default_rng(0)
X = rng.standard_normal((n, 3))
d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
S = np.exp(-0.5 * d2) + 0.1 * np.eye(n)
A0 = torch.tensor(S, device="cuda")
for it in range(4):
    A = A0.clone()
    torch.cuda.synchronize()
    t = time.perf_counter()
    L, _, _ = linalg.cholesky_(A)
    torch.cuda.synchronize()
    print("potrf ms", (time.perf_counter() - t) * 1e3, flush=True)
Ln = np.linalg.cholesky(S)
Lg = torch.tril(L).cpu().numpy()
print("max rel err", float(np.abs(Lg - Ln).max() / np.abs(Ln).max()))

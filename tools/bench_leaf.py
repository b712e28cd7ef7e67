"""Time the 128x128 leaf (Cholesky + inverse) alone: n = 128 single and batched."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from vgposp_amd import linalg

rng = np.random.default_rng(0)
out = {}
for n, B in [(128, 1), (128, 256), (96, 1), (512, 1)]:
    M = rng.normal(size=(B, n, n))
    S = torch.as_tensor(M @ M.transpose(0, 2, 1) + n * np.eye(n), device="cuda")
    for _ in range(3):
        linalg.cholesky_(S.clone(), invert=True)
    A = [S.clone() for _ in range(20)]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for a in A:
        linalg.cholesky_(a, invert=True, check=False)
    e1.record()
    torch.cuda.synchronize()
    out[f"n{n}_b{B}_us"] = e0.elapsed_time(e1) * 1e3 / len(A)
print(json.dumps(out))

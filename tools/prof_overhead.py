"""Wall time of the fused Cholesky + inverse with and without the library's event profiling."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import _lib, linalg
from vgposp_amd.data_generation import grid_points, grid_spacing

shape = tuple(int(v) for v in (sys.argv[1:4] or (64, 32, 32)))
X = grid_points(shape)
n = X.shape[0]
A = torch.empty((n, n), dtype=torch.float64, device="cuda")
ls = 2 * grid_spacing(shape)
res = {"n": n}
for rep, prof in enumerate([False, True, False, True]):
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    torch.cuda.synchronize()
    _lib.prof_enable(prof)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    linalg.cholesky_(A, invert=True, check=False)
    e1.record()
    torch.cuda.synchronize()
    _lib.prof_enable(False)
    res[f"run{rep}_prof{int(prof)}_s"] = e0.elapsed_time(e1) * 1e-3
print(json.dumps(res))

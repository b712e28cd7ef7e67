"""Isolate the bench step's parts: potrf+inverse on jittered vs regular grids, via cholesky_ and
via GreedyPlacement.init(), with the GEMM share from the library's event timing."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import _lib, linalg
from vgposp_amd.data_generation import grid_points, grid_spacing
from vgposp_amd.placement_algorithm2 import GreedyPlacement

shape = (64, 32, 32)
h = grid_spacing(shape)
res = {}
S = torch.empty((65536, 65536), dtype=torch.float64, device="cuda")
g = GreedyPlacement(S, 50)


def timed(fn):
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    gm = _lib.prof_query("gemm_f64")[0]
    _lib.prof_enable(False)
    return round(e0.elapsed_time(e1), 1), round(gm, 1)


for jit in (0.0, 0.05):
    X = grid_points(shape, jitter=jit, seed=0)
    for full in (False, True):
        for how in ("cholesky_", "greedy_init"):
            linalg.kernel_matrix("eq", X, None, 1.0, 2 * h, diag_shift=0.010001, lower=not full,
                                 out=S[None])
            if how == "cholesky_":
                res[f"jit{jit}_full{int(full)}_{how}"] = timed(lambda: linalg.cholesky_(S, invert=True, check=False))
            else:
                res[f"jit{jit}_full{int(full)}_{how}"] = timed(g.init)
            print(json.dumps(res), flush=True)

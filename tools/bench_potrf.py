"""Micro-benchmark of the recursive Cholesky (+ inverse) with the library's per-kernel timing."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import _lib, linalg
from vgposp_amd.data_generation import grid_points, grid_spacing


def run(shape, invert):
    X = grid_points(shape)
    n = X.shape[0]
    A = torch.empty((n, n), dtype=torch.float64, device="cuda")
    ls = 2 * grid_spacing(shape)
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    linalg.cholesky_(A, invert=invert)  # warm-up
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    linalg.cholesky_(A, invert=invert, check=False)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e-3
    prof = {k: _lib.prof_query(k) for k in ("gemm_f64", "potrf_diag", "trtri_leaf")}
    _lib.prof_enable(False)
    flops = n ** 3 / 3 * (2 if invert else 1)
    return {"n": n, "invert": invert, "s": t, "tflops": flops / t / 1e12,
            "gemm_ms": prof["gemm_f64"][0], "gemm_tflops": prof["gemm_f64"][2] / prof["gemm_f64"][0] / 1e9,
            "gemm_launches": prof["gemm_f64"][1], "diag_ms": prof["potrf_diag"][0],
            "leaf_ms": prof["trtri_leaf"][0]}


if __name__ == "__main__":
    for shape in [(32, 16, 16), (32, 32, 32), (64, 32, 32)]:
        for inv in (False, True):
            print(json.dumps(run(shape, inv)), flush=True)

"""Leading-dimension A/B for the fused Cholesky + inverse: the same n x n covariance stored with
row stride n (a power of two at the bench's n = 65,536: every row of a tile panel starts at the
same offset modulo 512 KiB) and with a padded stride n + pad.
python tools/lda_ab.py [n] [pad ...] -> one JSON line per (pad, repeat): seconds, GEMM TF/s."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import _lib, linalg
from vgposp_amd.data_generation import grid_points, grid_spacing

SHAPES = {65536: (64, 32, 32), 32768: (32, 32, 32), 16384: (32, 16, 32)}


def run(n, pad, X, ls):
    buf = torch.empty((n, n + pad), dtype=torch.float64, device="cuda")
    A = buf[:, :n]
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    linalg.cholesky_(A, invert=True, check=False)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e-3
    g = _lib.prof_query("gemm_f64")
    _lib.prof_enable(False)
    diag = float(A.diagonal().sum())  # the same factor whatever the stride
    del buf, A
    torch.cuda.empty_cache()
    return {"n": n, "pad": pad, "s": t, "tflops": 2 * n ** 3 / 3 / t / 1e12,
            "gemm_ms": g[0], "gemm_tflops": g[2] / g[0] / 1e9, "gemm_launches": g[1],
            "diag_sum": diag}


if __name__ == "__main__":
    args = [int(a) for a in sys.argv[1:]]
    n = args[0] if args else 65536
    pads = args[1:] or [0, 64, 128]
    X = grid_points(SHAPES[n])
    ls = 2 * grid_spacing(SHAPES[n])
    run(n, 0, X, ls)  # warm-up
    for rep in range(2):
        for pad in pads:
            print(json.dumps(run(n, pad, X, ls)), flush=True)

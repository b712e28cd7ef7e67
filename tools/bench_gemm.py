"""Micro-benchmark of the fp64 MFMA GEMM (vgposp_gemm) on the shapes the Cholesky sweep uses."""
import argparse
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import linalg


def run(m, n, k, ta, tb, lower, beta, reps=5, tri_a=False, tri_b=False):
    A = torch.randn((k, m) if ta else (m, k), dtype=torch.float64, device="cuda")
    B = torch.randn((n, k) if tb else (k, n), dtype=torch.float64, device="cuda")
    C = torch.randn((m, n), dtype=torch.float64, device="cuda")
    kw = dict(alpha=-1.0, beta=beta, transa=ta, transb=tb, lower_c=lower, tri_a=tri_a, tri_b=tri_b)
    linalg.gemm(A, B, C, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        linalg.gemm(A, B, C, **kw)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    outs = m * (m + 1) / 2 if lower else m * n
    frac = (1 / 3 if tri_a and tri_b else 0.5 if (tri_a or tri_b) else 1.0)
    return {"m": m, "n": n, "k": k, "ta": ta, "tb": tb, "lower": lower, "tri": [tri_a, tri_b],
            "ms": t * 1e3, "tflops": 2 * k * outs * frac / t / 1e12}


if __name__ == "__main__":
    shapes = [
        (8192, 8192, 8192, 0, 1, False, 0.0),
        (16384, 16384, 128, 0, 1, True, 1.0),    # trailing SYRK, K = 128
        (16384, 16384, 256, 0, 1, True, 1.0),    # trailing SYRK, K = 256
        (32768, 32768, 128, 0, 1, True, 1.0),
        (16384, 16384, 128, 0, 0, False, 1.0),   # GJ update (NN)
        (65536, 128, 128, 0, 1, False, 0.0),     # panel
        (8192, 8192, 8192, 1, 0, True, 0.0),     # M^T M
    ]
    for s in shapes:
        print(json.dumps(run(*s)), flush=True)
    # trtri TRMMs: W = L21 X11 (tri_b), X21 = -X22 W (tri_a); GPRM V = K M^T (tri_b, NT)
    print(json.dumps(run(16384, 16384, 16384, 0, 0, False, 0.0, tri_b=True)), flush=True)
    print(json.dumps(run(16384, 16384, 16384, 0, 0, False, 0.0, tri_a=True)), flush=True)
    print(json.dumps(run(16384, 16384, 16384, 0, 1, False, 0.0, tri_b=True)), flush=True)

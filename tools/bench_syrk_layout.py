"""Kzx Kzx^T (M = 512, K = N = 262,144) from the [M, N] layout (row pitch 2 MiB, NT) against the
[N, M] layout (row pitch 4 KiB, TN): does the 2 MiB row stride (one page per row) cost?"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import linalg

M, N = 512, 262144
A = torch.randn(M, N, dtype=torch.float64, device="cuda")
At = A.t().contiguous()
C = torch.empty(M, M, dtype=torch.float64, device="cuda")
res = {}
for name, fn in [("NT_MxN", lambda: linalg.gemm(A, A, C, transb=True, lower_c=True)),
                 ("TN_NxM", lambda: linalg.gemm(At, At, C, transa=True, lower_c=True)),
                 ("NT_MxN_full", lambda: linalg.gemm(A, A, C, transb=True)),
                 ("TN_NxM_full", lambda: linalg.gemm(At, At, C, transa=True))]:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    full = "full" in name
    fl = 2.0 * M * M * N * (1.0 if full else 0.5 * (M + 1) / M)
    res[name] = {"ms": ms, "tflops": fl / (ms * 1e-3) / 1e12}
ref = (A @ A.t()).tril()
linalg.gemm(At, At, C, transa=True, lower_c=True)
res["tn_err"] = float((C.tril() - ref).abs().max())
print(json.dumps(res))

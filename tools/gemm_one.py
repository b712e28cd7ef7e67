"""Run one GEMM shape a few times (for rocprofv3 PMC passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import linalg

m, n, k = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (8192, 8192, 8192)
A = torch.randn((m, k), dtype=torch.float64, device="cuda")
B = torch.randn((n, k), dtype=torch.float64, device="cuda")
C = torch.zeros((m, n), dtype=torch.float64, device="cuda")
for _ in range(3):
    linalg.gemm(A, B, C, transb=True)
torch.cuda.synchronize()
print("done")

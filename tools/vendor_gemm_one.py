"""One fp64 8192^3 NT product through torch (hipBLASLt / rocBLAS) — for reading its kernel name."""
import torch
n = 8192
a = torch.randn(n, n, dtype=torch.float64, device="cuda")
b = torch.randn(n, n, dtype=torch.float64, device="cuda")
for _ in range(3):
    c = a @ b.t()
torch.cuda.synchronize()

"""Phase cycles of the 128-leaf Cholesky + inverse kernel (potrf_leaf_kernel) in a plain N = 8,192
factorization, from a -DVGPOSP_STAMPS build (SRC=../../tools/variants/potrf_stamps.hip tools/build_potrf_variant.sh stamps -DVGPOSP_STAMPS;
VGPOSP_LIB=$PWD/tools/variants/lib_stamps.so python tools/leaf_probe.py).  Thread 0 of every leaf
workgroup accumulates s_memtime deltas: panel updates | panel factors | diagonal-block inverses |
off-diagonal inverse chains | output; printed per leaf, in microseconds at the measured clock."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import _lib, linalg  # noqa: E402
from vgposp_amd.data_generation import grid_points, grid_spacing  # noqa: E402

shape = (32, 16, 16)
X = grid_points(shape, jitter=0.05, seed=0)
N = X.shape[0]
Xd = linalg.as_device(X)
S = torch.empty((N, N), dtype=torch.float64, device="cuda")
lib = _lib.load()
buf = (ctypes.c_longlong * 16)()


def run():
    linalg.kernel_matrix("eq", Xd, None, linalg.as_device([1.0]),
                         linalg.as_device([2 * grid_spacing(shape)]),
                         diag_shift=linalg.as_device([1e-2 + 1e-6]), lower=True, out=S[None])
    linalg.cholesky_(S, invert=True, check=False)
    torch.cuda.synchronize()


run()
lib.vgposp_potrf_stamps(buf)  # clear
t0 = time.perf_counter()
run()
lib.vgposp_potrf_stamps(buf)
leaves = N // 128
names = {3: "panel_update", 1: "panel_factor", 2: "diag_inverse", 4: "offdiag_inverse", 5: "output"}
# s_memtime counts at the shader clock; MI355X runs the leaf near 2.4 GHz
out = {v: round(buf[k] / leaves / 2400.0, 2) for k, v in names.items()}
out["leaves"] = leaves
print(json.dumps({"us_per_leaf_at_2.4GHz": out}), flush=True)

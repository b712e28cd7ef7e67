"""Per-shape GEMM time histogram of one fused Cholesky + inverse (VGPOSP_PROF_SHAPES=1)."""
import json
import os
import sys

os.environ["VGPOSP_PROF_SHAPES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from vgposp_amd import _lib, linalg
from vgposp_amd.data_generation import grid_points, grid_spacing


def main(shape=(64, 32, 32), invert=True, top=40):
    X = grid_points(shape)
    n = X.shape[0]
    A = torch.empty((n, n), dtype=torch.float64, device="cuda")
    ls = 2 * grid_spacing(shape)
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    linalg.cholesky_(A, invert=invert)  # warm-up
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=0.010001, lower=True, out=A[None])
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    linalg.cholesky_(A, invert=invert, check=False)
    torch.cuda.synchronize()
    d = _lib.prof_dump()
    _lib.prof_enable(False)
    rows = [(k, v) for k, v in d.items() if k.startswith("gemm:")]
    rows.sort(key=lambda kv: -kv[1][0])
    tot = sum(v[0] for _, v in rows)
    print(json.dumps({"n": n, "gemm_ms_total": tot, "other": {k: v for k, v in d.items()
                                                              if not k.startswith("gemm:")}}))
    for k, (ms, cnt, fl, _) in rows[:top]:
        print(f"{k:40s} {ms:9.3f} ms {cnt:5d} x  {fl / (ms * 1e-3) / 1e12:6.1f} TF/s  "
              f"{100 * ms / tot:5.1f}%")


if __name__ == "__main__":
    main()

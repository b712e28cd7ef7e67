"""Debug: bench.py's vgp_line loop shape (all feed indices precomputed, no per-step host read)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph  # noqa: E402

torch.cuda.set_device(0)
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
X, y, Z = vgp_c3_data()
N = len(X)
B = N // 8
train_op, loss, xb, yb = vgp_c3_graph(X, y, Z, B)
Xd = torch.as_tensor(X, device="cuda")
yd = torch.as_tensor(y, device="cuda")
rng = np.random.default_rng(1)
steps = int(os.environ.get("REP_N", "30"))
idx = [torch.as_tensor(rng.integers(0, N, B), device="cuda") for _ in range(steps + 2)]
first = float(train_op.run({xb: Xd[idx[0]], yb: yd[idx[0]]}))
train_op.run({xb: Xd[idx[1]], yb: yd[idx[1]]})
torch.cuda.synchronize()
keep = []
for i in range(2, steps + 2):
    fx, fy = Xd[idx[i]], yd[idx[i]]
    last = train_op.run({xb: fx, yb: fy})
    if mode == "sync":
        torch.cuda.synchronize()
    if mode == "ssync":
        torch.cuda.current_stream().synchronize()
    if mode == "keep":
        keep.append((fx, fy, last))
torch.cuda.synchronize()
print(mode, "ok", first, float(last), flush=True)

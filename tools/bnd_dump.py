"""Dump C4's all-candidate Q_yy upper bounds (vgposp_exact_bounds, 128^3, the default Gauss-Radau
steps, and one to three explicit steps) to an .npz, for a bit-identity A/B of two builds
(VGPOSP_LIB=... python tools/bnd_dump.py out.npz)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd.sparse_placement import ExactTaperPlacement  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402

X, shape, ls = c4_grid()
run = ExactTaperPlacement(X, shape, 50, 3, 4.0, ls=ls, diag_shift=0.01 + 1e-6, method="bounds")
run.run()
g = run.greedy
out = {}
q = torch.zeros(g.p.n, dtype=torch.float64, device="cuda")
b = g.bound_qdiag(q)
out["default"] = q.cpu().numpy().copy()
for K in (1, 2, 3):
    q.zero_()
    g.bound_qdiag(q, steps=(K, 1.0 + 1e-12, 0.0), mu=g.gershgorin(q)[0])
    out["K%d" % K] = q.cpu().numpy().copy()
# a sub-range (a shard's [c0, c1)): the candidates outside keep their zeros
q.zero_()
n = g.p.n
g.bound_qdiag(q, c0=n // 3 + 5, c1=2 * n // 3 + 17)
out["range"] = q.cpu().numpy().copy()
np.savez(sys.argv[1], **out)
print("bounds", b, {k: float(np.abs(v).sum()) for k, v in out.items()}, flush=True)

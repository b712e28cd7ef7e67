"""A/B debug of the one-launch CG (VGPOSP_LIB=tools/variants/lib_cgab.so): one column on a small grid
against the dense inverse, with the iterations used."""
import sys
import numpy as np
sys.path.insert(0, '.')
from oracle import taper as lp
from vgposp_amd.data_generation import grid_points, grid_spacing
from vgposp_amd.sparse_placement import ExactTaperPlacement
shape = (12, 11, 10)
X = grid_points(shape, jitter=0.05, seed=3)
ls = 2 * grid_spacing(shape)
for method in ("selinv", "bounds"):
    run = ExactTaperPlacement(X, shape, 3, 3, ls=ls, diag_shift=0.01 + 1e-6, leaf=128, method=method)
    p = run.run().cpu().numpy()
    C = lp.tapered_cov(X, shape, 4.0, ls=ls, diag_shift=0.01 + 1e-6)
    Qi = np.linalg.inv(C + 1e-6 * np.eye(len(C)))
    cols = run.greedy.q_columns().cpu().numpy()
    print(method, 'picks', p, 'cg', run.greedy.cg_iters, run.greedy.cg_iterations_used())
    for t in range(2):
        e = cols[t] - Qi[:, p[t]]
        print(' col', t, 'maxerr', np.abs(e).max(), 'at center', cols[t][p[t]], Qi[p[t], p[t]],
              'nnz', int((np.abs(cols[t]) > 0).sum()))

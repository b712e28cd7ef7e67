import sys, numpy as np
sys.path.insert(0, '.')
from oracle import taper as lp
from oracle import placement as op
from vgposp_amd.data_generation import grid_points, grid_spacing
from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
shape=(8,8,8); k=8
X=grid_points(shape,jitter=0.05,seed=8*7+k); ls=2*grid_spacing(shape)
A, deltas, dci = tapered_placement_algorithm_3(X, k, shape, 3, 4.0, ls=ls, diag_shift=0.01+1e-6, snapshots=True, leaf=96)
C=lp.tapered_cov(X,shape,4.0,ls=ls,diag_shift=0.01+1e-6)
rA,_,rdci=op.placement_window_precision(C,k,shape,3)
print(A, rA)
for c in range(k):
    d=np.abs(dci[:,c]-rdci[:,c]); bad=np.flatnonzero(d>1e-12)
    print(c, d.max(), len(bad), bad[:10], [int(np.abs(np.array(np.unravel_index(b,shape))-np.array(np.unravel_index(rA[c-1],shape))).max()) if c>0 else -1 for b in bad[:10]])
from vgposp_amd.sparse_placement import ExactTaperPlacement
import torch
run = ExactTaperPlacement(X, shape, k, 3, ls=ls, diag_shift=0.01+1e-6, leaf=96)
snaps=[]
p = run.run(snaps).cpu().numpy()
Qi = np.linalg.inv(C + 1e-6*np.eye(len(C)))
cols = run.greedy.q_columns().cpu().numpy()
for t in range(k-1):
    print('col', t, p[t], np.abs(cols[t]-Qi[:,p[t]]).max())
qd = run.qdiag.cpu().numpy(); print('qdiag', np.abs(qd-np.diag(Qi)).max())
print('cg', run.greedy.cg_iters, run.greedy.cg_iterations_used())
# rerun deterministic?
snaps2=[]
p2 = run.run(snaps2).cpu().numpy()
print('rerun equal', np.array_equal(p,p2), max(float((a-b).abs().max()) for a,b in zip(snaps,snaps2)))

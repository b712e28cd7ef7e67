"""The hot-path computations of `main_architecture_2_sampledistribution.py` in its call order, on
the MI355X drop-in modules.  The reference restores a trained VGP and builds cov_vv pair by pair in
TF while loops. It then filters cov_vv with the beta-decay local kernel and places sensors. Its
datasets and saved variables are absent, so synthetic 5-D data stand in (the C5 field of
`vgposp_amd.workloads`):

    :188-265    VGP on (x, y, z, T, P) -> tfd.VariationalGaussianProcess.optimal_variational_posterior
                -> variational_loss(kl_weight = B / N) -> AdamOptimizer(0.01).minimize -> sess.run
    :423-542    cov_vv[i][j] = tfp.stats.covariance over the T/P samples of the VGP mean at
                locations i and j   (covariance.cov_vv_from_vgp: every pair at once)
    :361-421    local_kernel_filter: cov_vv *= exp(-(beta delta_ij)^2 / 2 pi), zeroed below 0.01
                (covariance.index_taper_)
    :871        snippets_a2.sparse_placement_algorithm_2(cov_vv, K_SENSORS, COVER_spatial)
    :915-932    selection / delta_cached_iters CSVs  (snippets_save)
    (and snippets_a3.sparse_placement_algorithm_3, the windowed variant of the same greedy)

    python examples/main_architecture_2.py [--cover 6 6 6] [--steps 200] [--k 7] [--out DIR]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vgposp_amd import snippets_save  # noqa: E402
from vgposp_amd.covariance import empirical_cov, index_taper_, vgp_tracer_samples  # noqa: E402
from vgposp_amd.snippets_a2 import sparse_placement_algorithm_2  # noqa: E402
from vgposp_amd.snippets_a3 import sparse_placement_algorithm_3  # noqa: E402
from vgposp_amd.workloads import vgp_c3_graph, vgp_c5_data  # noqa: E402

BETA_val = 4.0  # TEST_cov_buckets(..., BETA_val=4.)


def run(cover=(6, 6, 6), n_obs=8192, m=3, batch=1024, steps=200, tp_samples=None, k=7,
        cutoff=2, seed=0, out_dir=None):
    t0 = time.perf_counter()
    X, y, Z = vgp_c5_data(n=n_obs, m=m, seed=seed)
    train_op, loss, xb, yb = vgp_c3_graph(X, y, Z, batch)
    rng = np.random.default_rng(seed + 1)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    losses = []
    for _ in range(steps):
        idx = torch.as_tensor(rng.integers(0, len(X), batch), device="cuda")
        losses.append(train_op.run({xb: Xd[idx], yb: yd[idx]}))
    losses = torch.stack([torch.as_tensor(v).reshape(()) for v in losses]).cpu().numpy()
    t_train = time.perf_counter() - t0

    # locations on the cover grid (linsp over [-2, 2] per axis, C order) and T/P samples
    lin = [np.linspace(-2.0, 2.0, c) for c in cover]
    locs = np.stack(np.meshgrid(*lin, indexing="ij"), -1).reshape(-1, 3)
    S = tp_samples or 4 * len(locs)
    tp = rng.uniform(-2.0, 2.0, (S, 2))
    vgp = loss.vgp
    T = vgp_tracer_samples(vgp, locs, tp)  # covariance.cov_vv_from_vgp, in its two steps
    cov_vv = empirical_cov(T)
    cov_raw = cov_vv.cpu().numpy()
    index_taper_(cov_vv, cover, BETA_val)
    t1 = time.perf_counter()
    A, len_A, dci, sel = sparse_placement_algorithm_2(cov_vv, k, cover)
    A3, cache3, dci3 = sparse_placement_algorithm_3(cov_vv, k, cover, cutoff)
    t_place = time.perf_counter() - t1
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        snippets_save.save_cov_vv(cov_vv.cpu().numpy(), os.path.join(out_dir, "cov_vv.csv"))
        snippets_save.save_selection(sel, os.path.join(out_dir, "selection.csv"))
        snippets_save.save_delta_cached_iters(dci, os.path.join(out_dir, "delta_cached_iters.csv"))
    amp, ls = (float(v[0]) for v in vgp.kernel.params())
    return dict(losses=losses, locs=locs, tp=tp, T=T.cpu().numpy(), cov_raw=cov_raw, cov_vv=cov_vv.cpu().numpy(),
                alg2=[int(v) for v in sel[:, 0]], alg3_set=sorted(int(v) for v in A3.values),
                dci=dci, amp=amp, ls=ls, Z=vgp._Z().cpu().numpy(), vgp=vgp, t_train=t_train,
                t_place=t_place)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cover", type=int, nargs=3, default=[6, 6, 6])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    r = run(tuple(a.cover), steps=a.steps, k=a.k, out_dir=a.out)
    print(json.dumps({"cover": a.cover, "loss_first": float(r["losses"][0]),
                      "loss_last": float(r["losses"][-1]), "amp": r["amp"], "ls": r["ls"],
                      "alg2": r["alg2"], "alg3": r["alg3_set"], "train_s": r["t_train"],
                      "placement_s": r["t_place"]}))


if __name__ == "__main__":
    main()

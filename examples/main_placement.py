"""The computations of the reference drivers `main_GP_fit.py` and `main.py`, in their call order,
on the MI355X drop-in modules (the reference scripts themselves stop before the hot
path; their data files and VAE checkpoint are absent).  Synthetic inputs replace the CSVs:

    main_GP_fit.py:186-245   tf_Placeholder_assign_test -> create_cov_kernel -> fit_gp ->
                             log_prob -> tf_train_gp_adam -> tf_optimize_model_params (lls)
    main_GP_fit.py:249-262   create_meshgrid -> tf_gp_regression_model -> sample ;  calc_H
    main.py:125-350, :597    cov_vv = pairwise tfp.stats.covariance of per-location samples
                             (here: GPRM posterior samples on the cover grid) -> cov_vv.csv
    main.py:605              placement_algorithm2.placement_algorithm_2(cov_vv_, K)
    main.py:493, :608        snippets_a2.sparse_placement_algorithm_2(cov_vv, K, COVER)
    main.py:610-613          py_get_coord_idxs -> selected coordinates

Config C1 of BASELINE.json (8 x 8 x 8 grid, 3-D sinusoid, batch-2 kernel) is the default.
`run()` returns every intermediate so tests can check each one against the oracle.

    python examples/main_placement.py [--cover 8 8 8] [--iters 1000] [--k 7] [--out DIR]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vgposp_amd import gp_functions as gpf  # noqa: E402
from vgposp_amd import snippets_save  # noqa: E402
from vgposp_amd.covariance import empirical_cov  # noqa: E402
from vgposp_amd.data_generation import grid_points, grid_observations  # noqa: E402
from vgposp_amd.placement_algorithm2 import placement_algorithm_2  # noqa: E402
from vgposp_amd.snippets_a2 import sparse_placement_algorithm_2  # noqa: E402

AMPLITUDE_INIT = np.array([.1, .1])      # main_GP_fit.py:117
LENGTHSCALE_INIT = np.array([.1, .1])    # main_GP_fit.py:118
LEARNING_RATE = .1                       # main_GP_fit.py:119
INIT_OBSNOISEVAR = 1e-6                  # main_GP_fit.py:120
XEDGES = YEDGES = 60                     # main_GP_fit.py:122-123
PRED_FRACTION = 50                       # main_GP_fit.py:126
NUM_SAMPLES = 20                         # main_GP_fit.py:128


def run(cover=(8, 8, 8), num_iters=1000, k=7, num_train=200, cov_samples=None, xedges=XEDGES,
        yedges=YEDGES, seed=0, out_dir=None):
    t0 = time.perf_counter()
    rng = np.random.default_rng(seed)
    # the cover grid (C-order flattening, main.py:259-267) and noisy 3-D sinusoid observations
    X = grid_points(cover, jitter=0.05, seed=seed)
    y = grid_observations(X, seed=seed + 1)
    train = np.sort(rng.choice(len(X), size=min(num_train, len(X)), replace=False))
    Xtr, ytr = X[train], y[train]

    # ---- main_GP_fit.py: hyperparameter fit ----
    sess = gpf.reset_session()
    amp, amp_assign, amp_p, lensc, lensc_assign, lensc_p, emb, emb_assign, emb_p, obs_noise_var = \
        gpf.tf_Placeholder_assign_test(AMPLITUDE_INIT, LENGTHSCALE_INIT, INIT_OBSNOISEVAR)
    kernel = gpf.create_cov_kernel(amp, lensc)
    gp = gpf.fit_gp(kernel, Xtr, obs_noise_var)
    log_likelihood = gp.log_prob(ytr)
    train_op = gpf.tf_train_gp_adam(log_likelihood, LEARNING_RATE)
    summ, writer, saver = gpf.tf_summary_writer_saver(sess, None)
    lls = gpf.tf_optimize_model_params(sess, num_iters, train_op, log_likelihood, summ, writer,
                                       saver, None, None, ytr, None)
    t_fit = time.perf_counter() - t0

    # ---- main_GP_fit.py: GPRM on a prediction mesh (first two coordinates, z = 0 plane) ----
    pred = np.linspace(-2, 2, PRED_FRACTION, dtype=np.float64)
    xy_pred = gpf.create_meshgrid(pred, pred)
    xyz_pred = np.concatenate([xy_pred, np.zeros((len(xy_pred), 1))], axis=1)
    gprm_mesh = gpf.tf_gp_regression_model(kernel, xyz_pred, Xtr, ytr, obs_noise_var, 0.)
    samples_mesh = gprm_mesh.sample(NUM_SAMPLES, seed=seed).cpu().numpy()

    # ---- main.py: cov_vv from per-location samples (posterior samples on the cover grid) ----
    # 4 N samples keep the empirical covariance full rank (the Cholesky-based greedy, like the
    # reference's pinv, then sees a well-posed problem)
    cov_samples = cov_samples or 4 * len(X)
    gprm_cover = gpf.tf_gp_regression_model(kernel, X, Xtr, ytr, obs_noise_var, 0.)
    T = gprm_cover.sample(cov_samples, seed=seed + 2)[:, 0, :].t().contiguous()  # [N, S]
    cov_vv = empirical_cov(T)
    cov_vv_ = cov_vv.cpu().numpy()
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        snippets_save.save_cov_vv(cov_vv_, os.path.join(out_dir, "cov_vv.csv"))

    # ---- main.py: placements ----
    t1 = time.perf_counter()
    np_algo2 = [int(a) for a in placement_algorithm_2(cov_vv_, k)]
    A, len_A, dci, sel_delta = sparse_placement_algorithm_2(cov_vv, k, cover)
    t_place = time.perf_counter() - t1
    sel_coord = gpf.py_get_coord_idxs(np_algo2, X)
    if out_dir:
        snippets_save.save_selection(sel_delta, os.path.join(out_dir, "selection.csv"))
        snippets_save.save_delta_cached_iters(dci, os.path.join(out_dir, "delta_cached_iters.csv"))

    # ---- main.py:575 / main_GP_fit.py:260: the LML surface ----
    H = gpf.calc_H(xedges, yedges, lensc, lensc_assign, lensc_p, amp, amp_assign, amp_p,
                   log_likelihood, sess, None, ytr)
    return dict(X=X, y=y, train=train, lls=lls, samples_mesh=samples_mesh, T=T.cpu().numpy(),
                cov_vv=cov_vv_, np_algo2=np_algo2, tf_algo2=[int(a) for a in sel_delta[:, 0]],
                dci=dci, sel_coord=sel_coord, H=H, t_fit=t_fit, t_place=t_place,
                noise=float(obs_noise_var.numpy()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cover", type=int, nargs=3, default=[8, 8, 8])
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--k", type=int, default=7)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    r = run(tuple(a.cover), a.iters, a.k, out_dir=a.out)
    print(json.dumps({"cover": a.cover, "iters": a.iters, "lml_first": r["lls"][0].tolist(),
                      "lml_last": r["lls"][-1].tolist(), "np_algo2": r["np_algo2"],
                      "tf_algo2": r["tf_algo2"], "sel_coord": r["sel_coord"].tolist(),
                      "H_max": float(np.max(r["H"])), "fit_s": r["t_fit"],
                      "placement_s": r["t_place"]}))


if __name__ == "__main__":
    main()

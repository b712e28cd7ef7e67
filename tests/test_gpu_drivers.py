"""The reference drivers' call sequence end to end (examples/main_placement.py: main_GP_fit.py's
fit / GPRM / calc_H, then main.py's cov_vv -> placements -> coordinates) on the GPU modules,
every intermediate checked against the oracle restatements on the same data."""
import os
import sys

import numpy as np
import pytest

from oracle import covariance as ocov
from oracle import gp as ogp
from oracle import placement as op

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "examples"))


def test_main_placement_pipeline(tmp_path):
    import main_placement
    cover, k = (6, 6, 6), 5
    r = main_placement.run(cover=cover, num_iters=30, k=k, num_train=120, xedges=8, yedges=6,
                           out_dir=str(tmp_path))
    X, y, tr = r["X"], r["y"], r["train"]
    # main_GP_fit.py: the Adam fit trajectory of the batch-2 Matern 1/2 GP
    ref_lls, _ = ogp.fit_gp_adam("matern12", X[tr], y[tr], [.1, .1], [.1, .1], 1e-6, 0.1, 30)
    np.testing.assert_allclose(r["lls"], ref_lls, rtol=1e-7)
    assert r["samples_mesh"].shape == (main_placement.NUM_SAMPLES, 2, 50 * 50)
    assert np.isfinite(r["samples_mesh"]).all()
    # main.py: cov_vv = pairwise tfp.stats.covariance of the per-location samples
    np.testing.assert_allclose(r["cov_vv"], ocov.empirical_cov(r["T"]), rtol=1e-10, atol=1e-14)
    # placements: the reference's numpy greedy (pinv) and its TF-graph variant, exact indices
    assert r["np_algo2"] == [int(a) for a in op.placement_algorithm_2(r["cov_vv"], k)]
    _, _, _, ref_sel = op.sparse_placement_algorithm_2(r["cov_vv"], k, cover)
    assert r["tf_algo2"] == [int(v) for v in ref_sel[:, 0]]
    np.testing.assert_array_equal(r["sel_coord"], X[r["np_algo2"]])
    # the CSV outputs of snippets_save
    for f in ("cov_vv.csv", "selection.csv", "delta_cached_iters.csv"):
        assert (tmp_path / f).stat().st_size > 0
    # main.py:575: the LML surface at the fitted noise
    ref_H = ogp.calc_H("matern12", X[tr], y[tr], r["noise"], 8, 6)
    np.testing.assert_allclose(r["H"], ref_H, rtol=1e-8)


def test_main_architecture_2_pipeline(tmp_path):
    import main_architecture_2 as arch2
    cover, k = (4, 4, 4), 6
    r = arch2.run(cover=cover, n_obs=2048, m=3, batch=256, steps=20, k=k, cutoff=1,
                  out_dir=str(tmp_path))
    assert np.isfinite(r["losses"]).all() and r["losses"][-1] < r["losses"][0]
    # cov_vv over the T/P samples of the VGP tracer field, then the beta-decay filter
    np.testing.assert_allclose(r["cov_raw"], ocov.empirical_cov(r["T"]), rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(r["cov_vv"], ocov.index_taper(r["cov_raw"], cover, arch2.BETA_val),
                               rtol=1e-12, atol=1e-15)
    # arch2:871 and the windowed variant: exact selections vs the restated TF graphs
    _, _, _, ref_sel = op.sparse_placement_algorithm_2(r["cov_vv"], k, cover)
    assert r["alg2"] == [int(v) for v in ref_sel[:, 0]]
    ref3, _, _ = op.sparse_placement_algorithm_3(r["cov_vv"], k, cover, 1)
    assert r["alg3_set"] == sorted(int(v) for v in ref3)
    assert (tmp_path / "selection.csv").stat().st_size > 0

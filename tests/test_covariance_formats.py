"""CPU checks: the cov_vv builders' oracle against the reference's pairwise definitions, and the
CSV formats (snippets_save.py:18-31) round trip."""
import numpy as np
import pytest

from oracle import covariance as oc


def test_empirical_cov_matches_pairwise_tfp_covariance():
    rng = np.random.default_rng(0)
    T = rng.normal(size=(7, 40)) * 3.0 + 1.0
    C = oc.empirical_cov(T, tr_mean=0.0018, tr_stdev=2.5)
    for i in range(7):
        for j in range(7):
            ti, tj = (T[i] - 0.0018) / 2.5, (T[j] - 0.0018) / 2.5
            assert C[i, j] == pytest.approx(oc.tfp_covariance(ti, tj), rel=1e-12)


def test_index_taper_definition():
    C = np.ones((27, 27))
    out = oc.index_taper(C, (3, 3, 3), beta=2.0)
    # (0,0,0) vs (0,0,1): delta 1 -> exp(-4/(2 pi)); vs (2,2,2): delta^2 = 12 -> 5e-4 < 0.01 -> 0
    assert out[0, 1] == pytest.approx(np.exp(-4.0 / (2 * np.pi)))
    assert out[0, 26] == 0.0
    assert np.allclose(out, out.T)


def test_cov_vv_csv_round_trip(tmp_path):
    from vgposp_amd import snippets_save
    rng = np.random.default_rng(1)
    U = rng.normal(1, 1, size=(11, 11))
    cov = U @ U.T + 0.001 * np.eye(11)
    f = tmp_path / "cov_vv.csv"
    snippets_save.save_cov_vv(cov, str(f))
    head = f.read_text().splitlines()[0]
    assert head == "," + ",".join(str(i) for i in range(11))  # DataFrame.to_csv header
    back = snippets_save.load_cov_vv(str(f))
    # the same DataFrame.to_csv call as the reference, so the same (last-digit) text rounding
    np.testing.assert_allclose(back, cov, rtol=1e-15)
    g = tmp_path / "sel.csv"
    snippets_save.save_selection(np.array([3, 1, 2]), str(g))
    assert g.read_text().splitlines() == [",0", "0,3", "1,1", "2,2"]

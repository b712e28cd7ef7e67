"""CPU checks of the TF-variant oracle (snippets_a2.sparse_placement_algorithm_2 restatement).

TensorFlow is absent, so the variant cannot be run; its restatement is anchored two ways:
with placement_algorithm_2's constants (jitter 0, threshold 1e-8, INF = inf) it must reproduce
the golden vectors recorded from the reference's own placement_algorithm2; and with the TF
constants it must agree with the precision-matrix restatement the HIP path implements."""
import numpy as np
import pytest

from oracle import gp as ogp
from oracle import placement as op
from tests.golden_io import placement_cases, placement_cov

CASES = placement_cases()
SMALL = [n for n in ("cov4x4", "randcov11", "spd11", "spd40", "grid4", "grid5") if n in CASES]


@pytest.mark.parametrize("name", SMALL)
def test_tf_oracle_with_alg2_constants_reproduces_goldens(name):
    e = CASES[name]
    cov = placement_cov(name, e)
    N = cov.shape[0]
    A, n, dci, sel = op.sparse_placement_algorithm_2(cov, e["k"], (N, 1, 1), jitter=0.0,
                                                     small=1e-8, inf=np.inf)
    assert [int(v) for v in sel[:, 0]] == e["alg2"]
    assert A == sorted(e["alg2"]) and n == e["k"]


def _grid_cov(shape, nugget, ls_h=2.0, seed=0):
    from vgposp_amd.data_generation import grid_points, grid_spacing
    X = grid_points(shape, jitter=0.05, seed=seed)
    K = ogp.kernel_matrix("eq", X, X, 1.0, ls_h * grid_spacing(shape))[0]
    return K + nugget * np.eye(len(X))


@pytest.mark.parametrize("shape,k,nugget,ls_h", [((4, 4, 4), 8, 1e-2 + 1e-6, 2.0),
                                                 ((4, 4, 4), 10, 1e-7, 1.5),
                                                 ((5, 4, 3), 12, 0.0, 1.5)])
def test_tf_oracle_matches_precision_restatement(shape, k, nugget, ls_h):
    cov = _grid_cov(shape, nugget, ls_h)
    A, n, dci, sel = op.sparse_placement_algorithm_2(cov, k, shape)
    snaps = []
    B = op.placement_lazy_precision(cov, k, jitter=op.TF_JITTER, thr=op.TF_SMALL,
                                    cache_init=op.TF_INF, snapshots=snaps)
    assert [int(v) for v in sel[:, 0]] == B
    d = np.array(snaps).T
    assert ((dci == op.TF_INF) == (d == op.TF_INF)).all()
    fin = dci != op.TF_INF
    np.testing.assert_allclose(d[fin], dci[fin], rtol=1e-6, atol=1e-9 * np.abs(dci[fin]).max())
    # snapshot semantics: a selected entry reads 0 in every later column
    for r, y in enumerate(B[:-1]):
        assert (dci[y, r + 1:] == 0).all()
        assert dci[y, r] == sel[r, 1]


def test_tf_oracle_cover_assert():
    with pytest.raises(ValueError):
        op.sparse_placement_algorithm_2(np.eye(8), 2, (2, 2, 3))


def test_product_cover_assert_before_device_work():
    from vgposp_amd.snippets_a2 import sparse_placement_algorithm_2
    with pytest.raises(ValueError):
        sparse_placement_algorithm_2(np.eye(8), 2, (2, 2, 3))


@pytest.mark.parametrize("shape,k,cutoff,nugget", [((4, 4, 4), 6, 1, 1e-2), ((5, 4, 3), 8, 2, 1e-2),
                                                   ((4, 4, 4), 8, 0, 1e-6)])
def test_alg3_oracle_forms_agree(shape, k, cutoff, nugget):
    """snippets_a3 restatement (pinv tf_nominator) vs the precision-matrix form the HIP path
    implements: same picks, same per-round cache snapshots."""
    cov = _grid_cov(shape, nugget)
    order = []
    A, cache, dci = op.sparse_placement_algorithm_3(cov, k, shape, cutoff, order=order)
    B, cache2, dci2 = op.placement_window_precision(cov, k, shape, cutoff)
    assert order == B and A == sorted(B)
    fin = dci < op.TF_INF
    assert (fin == (dci2 < op.TF_INF)).all()
    np.testing.assert_allclose(dci2[fin], dci[fin], rtol=1e-5, atol=1e-8 * np.abs(dci[fin]).max())
    np.testing.assert_allclose(cache2, dci[:, -1], rtol=1e-5, atol=1e-8 * np.abs(dci[fin]).max())


def test_alg3_window_bounds_are_half_open():
    """The reference's while loops run j in [i - cutoff, min(i + cutoff, I)): 2*cutoff wide."""
    w = sorted(op._window(0, (4, 4, 4), 2))
    assert w == sorted(j0 * 16 + j1 * 4 + j2 for j0 in range(2) for j1 in range(2) for j2 in range(2))
    # cutoff 1 around (1, 1, 1): j in [0, 2) per axis, so the window is lopsided toward 0
    w = sorted(op._window(1 * 16 + 1 * 4 + 1, (4, 4, 4), 1))
    assert w == sorted(j0 * 16 + j1 * 4 + j2 for j0 in range(2) for j1 in range(2) for j2 in range(2))

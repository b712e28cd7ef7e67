"""CPU checks of oracle/c4_exact.c (the C restatement of config C4's exact algorithm 3 in the
bounded-lazy form): its picks and pick deltas equal the dense oracle's algorithm 3
(oracle.placement.placement_window_precision on the dense tapered covariance) on small grids —
also with brackets so wide that most candidates get refined — and at 128^3 it reproduces the picks
committed in tests/golden/c4_picks.json (which the GPU tests and bench.py compare against), so the
GPU picks at the north-star size are pinned to a CPU run."""
import json
import os

import numpy as np
import pytest

from oracle import c4_exact as ce
from oracle import taper as lp
from oracle import placement as op
from vgposp_amd.data_generation import grid_points, grid_spacing

SHIFT = 0.01 + 1e-6


@pytest.mark.parametrize("shape,k,cutoff,kind,K", [
    ((6, 6, 6), 8, 3, "eq", None),
    ((7, 5, 6), 10, 2, "eq", 1),            # K = 1: nearly every candidate refined
    ((9, 8, 7), 20, 3, "matern52", None),
    ((10, 10, 10), 30, 4, "eq", 2),
    ((8, 9, 10), 25, 2, "matern32", None),
    ((1, 1, 40), 12, 3, "eq", None),        # a line
    ((2, 3, 50), 15, 5, "matern12", None),
    ((3, 3, 3), 27, 2, "eq", None),         # k = N
    ((5, 5, 5), 1, 2, "eq", None),          # one pick
    ((6, 5, 4), 10, 0, "eq", None),         # cutoff 0: no window re-score
])
def test_c_oracle_matches_dense_alg3(shape, k, cutoff, kind, K):
    X = grid_points(shape, jitter=0.05, seed=sum(shape))
    ls = 2.0 * grid_spacing(shape)
    C = lp.tapered_cov(X, shape, 4.0, kind=kind, ls=ls, diag_shift=SHIFT)
    st = {}
    picks, deltas = ce.exact_alg3(X, shape, k, cutoff, kind=kind, ls=ls, diag_shift=SHIFT, K=K,
                                  stats=st)
    rA, _, rdci = op.placement_window_precision(C, k, shape, cutoff)
    assert [int(a) for a in picks] == [int(a) for a in rA]
    np.testing.assert_allclose(deltas, [rdci[a, i] for i, a in enumerate(rA)], rtol=1e-12)
    assert st["rounds"] == k and st["refinements"] >= k


def test_c_oracle_refuses_without_diagonal_dominance():
    shape = (5, 5, 5)
    X = grid_points(shape, jitter=0.05, seed=0)
    with pytest.raises(ValueError, match="diagonally dominant"):
        ce.exact_alg3(X, shape, 5, 2, beta=1.0, ls=4.0 * grid_spacing(shape), diag_shift=1e-4)


def test_c_oracle_128cube_reproduces_committed_picks():
    """Config C4 at full size (128^3 = 2,097,152 candidates, k = 50, cutoff 3): a few seconds on
    the host's cores."""
    from vgposp_amd.workloads import c4_grid
    with open(os.path.join(os.path.dirname(__file__), "golden", "c4_picks.json")) as f:
        want = json.load(f)["picks"]
    X, shape, ls = c4_grid()
    st = {}
    picks, deltas = ce.exact_alg3(X, shape, 50, 3, ls=ls, diag_shift=SHIFT, stats=st)
    assert [int(a) for a in picks] == want
    assert np.all(np.isfinite(deltas)) and np.all(deltas > 0)
    assert st["refinements"] <= 2 * 50

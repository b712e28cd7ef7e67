"""CPU: the algorithm-3 restatements are pinned to fixtures produced by the REFERENCE's arithmetic
(tests/golden/make_golden_alg3.py: placement_algorithm2.nominator / denominator on Sigma + 1e-6 I
minus 1e-6, argmax_cache_linear, the window loop of snippets_a3.py:43-364).

* oracle.placement.sparse_placement_algorithm_3 (the pinv restatement of snippets_a3.py);
* oracle.placement.placement_window_precision (the precision-matrix algebra the GPU uses);
* oracle/c4_exact.c (the bounded-lazy C restatement behind the 128^3 picks), on the diagonally
  dominant beta = 4 cases;
* the fixture's covariance equals the tapered covariance rebuilt from its grid points, so the GPU
  tests (tests/test_gpu_alg3_golden.py), which assemble Sigma from X, see the same input."""
import numpy as np
import pytest

from golden_alg3 import NAMES, load
from oracle import c4_exact as ce
from oracle import taper as lpo
from oracle import placement as op


@pytest.mark.parametrize("name", NAMES)
def test_fixture_cov_is_tapered_cov_of_X(name):
    m, z = load(name)
    C = lpo.tapered_cov(z["X"], tuple(m["shape"]), m["beta"], kind=m["kernel"], ls=m["ls"],
                        diag_shift=m["diag_shift"])
    np.testing.assert_array_equal(C, z["cov"])


# the pinv restatement costs what the reference's arithmetic does (one SVD-pinv of Sigma_AbarAbar per
# delta: ~20 CPU-minutes for the 8^3 k = 24 case), so it runs on the grids up to 7^3; the 8^3 case
# (config C4's own parameters) pins the precision form and the C oracle, which the others tie to it
@pytest.mark.parametrize("name", [n for n in NAMES if np.prod(load(n)[0]["shape"]) <= 343])
def test_pinv_restatement_matches_reference_arithmetic(name):
    m, z = load(name)
    order = []
    _, cache, dci = op.sparse_placement_algorithm_3(z["cov"], m["k"], m["shape"], m["cutoff"],
                                                    order=order)
    assert order == [int(a) for a in z["order"]]
    np.testing.assert_allclose(dci, z["dci"], rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(cache, z["cache"], rtol=1e-10, atol=1e-13)


def test_pinv_restatement_at_c4_parameters_sampled():
    """Config C4's own parameters (8^3, EQ, beta 4, cutoff 3) against the reference's arithmetic
    directly, at a cost the CPU suite can carry: the pinv restatement's delta (tf_nominator /
    tf_denominator, snippets_a2.py:138-213, threshold snippets_a2.py:480) for 24 sampled candidates
    of round 0 (A = {}) and 24 of the first pick's window in round 1 (A = {a_0},
    snippets_a3.py:196-308) equals the fixture's delta_cached_iters columns 0 and 1.  (The full
    k = 24 run costs ~20 CPU-minutes; the precision form and the C oracle run it below.)"""
    m, z = load("g888_eq_b4_c3")
    cov, N = z["cov"], len(z["cov"])

    def delta(y, A):
        nom = op.tf_nominator(y, A, cov)
        den = op.tf_denominator(y, [v for v in range(N) if v not in A], cov)
        return 0.0 if (abs(den) < op.TF_SMALL or abs(nom) < op.TF_SMALL) else nom / den

    rng = np.random.default_rng(0)
    for y in rng.choice(N, 24, replace=False):
        np.testing.assert_allclose(delta(int(y), []), z["dci"][y, 0], rtol=1e-10)
    a0 = int(z["order"][0])
    win = [y for y in op._window(a0, tuple(m["shape"]), m["cutoff"]) if y != a0]
    for y in rng.choice(win, 24, replace=False):
        np.testing.assert_allclose(delta(int(y), [a0]), z["dci"][y, 1], rtol=1e-10)


@pytest.mark.parametrize("name", NAMES)
def test_precision_form_matches_reference_arithmetic(name):
    m, z = load(name)
    order, cache, dci = op.placement_window_precision(z["cov"], m["k"], m["shape"], m["cutoff"])
    assert [int(a) for a in order] == [int(a) for a in z["order"]]
    np.testing.assert_allclose(dci, z["dci"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name", [n for n in NAMES if load(n)[0]["beta"] >= 4.0])
def test_c_oracle_matches_reference_arithmetic(name):
    m, z = load(name)
    picks, deltas = ce.exact_alg3(z["X"], m["shape"], m["k"], m["cutoff"], beta=m["beta"],
                                  kind=m["kernel"], ls=m["ls"], diag_shift=m["diag_shift"])
    assert [int(a) for a in picks] == [int(a) for a in z["order"]]
    np.testing.assert_allclose(deltas, m["pick_deltas"], rtol=1e-10)

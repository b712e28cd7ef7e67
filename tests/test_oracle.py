"""The CPU oracle against the reference's own golden vectors (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import placement as op
from tests.golden_io import placement_cases, placement_cov

CASES = placement_cases()
SMALL = [n for n, e in CASES.items() if e["N"] <= 64]


@pytest.mark.parametrize("name", SMALL)
def test_pinv_oracle_reproduces_reference_trace(name):
    e = CASES[name]
    cov = placement_cov(name, e)
    trace = []
    A = op.placement_algorithm_2(cov, e["k"], trace=trace)
    assert [int(a) for a in A] == e["alg2"]
    ref = [tuple(t) for t in e["trace"]]
    assert len(trace) == len(ref)
    for got, exp in zip(trace, ref):
        assert got[0] == exp[0]
        if got[0] != "select":
            assert got[1] == exp[1]  # bit-exact: same pinv calls on the same slices


@pytest.mark.parametrize("name", [n for n in SMALL if "alg1" in CASES[n]])
def test_pinv_oracle_alg1(name):
    e = CASES[name]
    cov = placement_cov(name, e)
    assert [int(a) for a in op.placement_algorithm_1(cov, e["k"])] == e["alg1"]


@pytest.mark.parametrize("name", list(CASES))
def test_precision_oracle_matches_reference(name):
    e = CASES[name]
    cov = placement_cov(name, e)
    assert op.placement_lazy_precision(cov, e["k"]) == e["alg2"]
    if "alg1" in e:
        assert op.placement_lazy_precision(cov, e["k"], lazy=False) == e["alg1"]


@pytest.mark.parametrize("name", ["grid5", "grid654", "spd40"])
def test_precision_deltas_match_trace(name):
    """Every delta the reference evaluated, recomputed with Cholesky/precision algebra."""
    e = CASES[name]
    cov = placement_cov(name, e)
    A, pos = [], 0
    trace = e["trace"]
    while pos < len(trace):
        delta, _, _ = op.all_deltas(cov, A)
        while trace[pos][0] != "select":
            y, d = trace[pos]
            assert delta[y] == pytest.approx(d, rel=1e-9, abs=1e-12)
            pos += 1
        A.append(trace[pos][1])
        pos += 1


@pytest.mark.parametrize("name", list(CASES))
def test_incremental_oracle_matches_reference(name):
    """The O(N^2)-per-round restatement (used by the GPU test at N = 16k) against the goldens."""
    e = CASES[name]
    cov = placement_cov(name, e)
    assert op.placement_lazy_incremental(cov, e["k"]) == e["alg2"]
    if "alg1" in e:
        assert op.placement_lazy_incremental(cov, e["k"], lazy=False) == e["alg1"]


@pytest.mark.parametrize("jitter,thr,cinit", [(0.0, 1e-8, np.inf), (1e-6, 1e-7, 1e8)])
def test_incremental_oracle_matches_precision(jitter, thr, cinit):
    from vgposp_amd.data_generation import grid_points, grid_spacing
    from oracle import gp as ogp
    shape = (9, 8, 7)
    X = grid_points(shape, jitter=0.05, seed=11)
    K = ogp.kernel_matrix("matern32", X, X, 1.0, 2 * grid_spacing(shape))[0] + 0.01 * np.eye(len(X))
    a = op.placement_lazy_incremental(K, 20, jitter=jitter, thr=thr, cache_init=cinit)
    b = op.placement_lazy_precision(K, 20, jitter=jitter, thr=thr, cache_init=cinit)
    assert a == b

"""CPU checks of the bounded-lazy form of exact algorithm 3 (sparse_placement.ExactWindowGreedy
.run_bounded / exact_greedy.hip): the reach tables, the CG bracket of Q_yy, and the lazy loop's
bookkeeping, restated in numpy on the dense tapered covariance and compared with the oracle's
algorithm 3 (oracle.placement.placement_window_precision)."""
import itertools
import math

import numpy as np
import pytest

from oracle import taper as lp
from oracle import placement as op
from vgposp_amd.data_generation import grid_points, grid_spacing
from vgposp_amd.taper import taper_support
from vgposp_amd.sparse_placement import bound_steps, reach_table

SHIFT = 0.01 + 1e-6
EPS, THR = 1e-6, 1e-7


@pytest.mark.parametrize("beta,K", [(4.0, 1), (4.0, 5), (4.0, 8), (3.0, 2)])
def test_reach_table_is_the_k_step_ball(beta, K):
    offs, _ = taper_support(beta)
    tab, cnt, nb = reach_table(offs, K)
    assert tuple(tab[0]) == (0, 0, 0) and cnt[0] == 1 and cnt[-1] == len(tab)
    # brute force: offsets reachable in <= d steps
    reach = {(0, 0, 0): 0}
    for d in range(1, K + 1):
        for v in [v for v, s in reach.items() if s == d - 1]:
            for o in offs:
                w = tuple(int(a + b) for a, b in zip(v, o))
                reach.setdefault(w, d)
    assert {tuple(t) for t in tab} == set(reach)
    steps = np.array([reach[tuple(t)] for t in tab])
    assert np.all(np.diff(steps) >= 0)
    for d in range(K + 1):
        assert cnt[d] == (steps <= d).sum()
    pos = {tuple(t): i for i, t in enumerate(tab)}
    for i, j in itertools.product(range(len(tab)), range(len(offs))):
        w = tuple(int(a + b) for a, b in zip(tab[i], offs[j]))
        assert nb[i, j] == pos.get(w, -1)


def _problem(shape, beta=4.0, kind="eq", seed=1):
    X = grid_points(shape, jitter=0.05, seed=seed)
    ls = 2.0 * grid_spacing(shape)
    C = lp.tapered_cov(X, shape, beta, kind=kind, ls=ls, diag_shift=SHIFT)
    return C, C + EPS * np.eye(len(C))


def _gershgorin(Ce):
    off = np.abs(Ce).sum(1) - np.abs(np.diag(Ce))
    return float((np.diag(Ce) - off).min()), float((np.diag(Ce) + off).max())


def _cg_bounds(Ce, shape, offs, K, scale, mu=0.0):
    """exact_bounds_kernel restated: K CG steps from e_y on the reach-table nodes around y
    (clipped to the grid), g = sum alpha_i |r_i|^2, upper bound scale * g (mu = 0) or the
    Gauss-Radau bound scale * (g + gamma^mu_K |r_K|^2) (0 < mu <= lambda_min)."""
    tab, cnt, nb = reach_table(offs, K)
    I0, I1, I2 = shape
    out = np.zeros(len(Ce))
    for y in range(len(Ce)):
        c = np.array(np.unravel_index(y, shape))
        g = c + tab
        ok = np.all((g >= 0) & (g < np.array(shape)), axis=1)
        idx = np.ravel_multi_index(g[ok].T, shape)
        A = Ce[np.ix_(idx, idx)]
        r = np.zeros(len(idx))
        r[0] = 1.0
        p = r.copy()
        rr, acc, gmu = 1.0, 0.0, (1.0 / mu if mu > 0 else 0.0)
        for _ in range(K):
            q = A @ p
            alpha = rr / (p @ q)
            acc += alpha * rr
            r = r - alpha * q
            rn = r @ r
            if mu > 0:
                d = gmu - alpha
                gmu = d / (mu * d + rn / rr)
            p = r + (rn / rr) * p
            rr = rn
        out[y] = scale * (acc + gmu * rr) if mu > 0 else scale * acc
    return out


@pytest.mark.parametrize("shape,kind", [((6, 7, 8), "eq"), ((5, 9, 4), "matern52")])
def test_cg_bounds_bracket_q(shape, kind):
    C, Ce = _problem(shape, kind=kind)
    offs, _ = taper_support(4.0)
    Q = np.diag(np.linalg.inv(Ce))
    lo, hi = _gershgorin(Ce)
    K, scale, width = bound_steps(offs, lo, hi)
    qhi = _cg_bounds(Ce, shape, offs, K, scale)
    assert np.all(qhi >= Q) and np.all(qhi <= Q * scale * (1 + 1e-13))
    for K in (1, 2, 3):   # wider brackets hold too
        _, scale, _ = bound_steps(offs, lo, hi, kmax=K)
        qhi = _cg_bounds(Ce, shape, offs, K, scale)
        assert np.all(qhi >= Q)


@pytest.mark.parametrize("shape,kind", [((6, 7, 8), "eq"), ((5, 9, 4), "matern32")])
def test_radau_bounds_bracket_q(shape, kind):
    """The Gauss-Radau upper bound (mu = the Gershgorin lambda_min) holds at every K and after K
    steps brackets Q_yy at least as tightly as the Chebyshev bound after K (on the beta = 4 taper,
    about as tightly as Chebyshev after K + 1: sparse_placement.radau_steps)."""
    C, Ce = _problem(shape, kind=kind)
    offs, _ = taper_support(4.0)
    Q = np.diag(np.linalg.inv(Ce))
    lo, hi = _gershgorin(Ce)
    assert 0 < lo <= np.linalg.eigvalsh(Ce)[0]
    for K in (1, 2, 3, 4, 5):
        _, cscale, cwidth = bound_steps(offs, lo, hi, kmax=K)
        rad = _cg_bounds(Ce, shape, offs, K, 1.0 + 1e-12, mu=lo)
        cheb = _cg_bounds(Ce, shape, offs, K, cscale)
        assert np.all(rad >= Q), K
        assert np.all(rad <= cheb * (1 + 1e-13)), K
        _, _, wnext = bound_steps(offs, lo, hi, kmax=K + 1)
        assert (rad / Q - 1).max() <= 4 * wnext, (K, (rad / Q - 1).max(), wnext)


def _delta_ub(nom, P, exact):
    den = 1.0 / P - EPS
    if exact:
        return 0.0 if (abs(nom) < THR or abs(den) < THR) else nom / den
    return 0.0 if abs(nom) < THR else nom / max(den, THR)


def bounded_lazy_alg3(C, Ce, shape, k, cutoff, qhi):
    """The host loop of ExactWindowGreedy.run_bounded with the device kernels' arithmetic restated
    on the dense matrix: cache = upper bounds; refine the arg-max until it is refined (its entry
    re-scored with the A of its last re-score, lastA); pick; window re-score (bounds for
    unrefined).  -> (picks, pick deltas, refinements)."""
    N = len(C)
    Qd = np.diag(np.linalg.inv(Ce))
    exact = np.zeros(N, dtype=bool)
    lastA = np.zeros(N, dtype=np.int64)
    sel = np.zeros(N, dtype=bool)
    A = []
    qd = qhi.copy()
    _, nom0, den0 = op.all_deltas(C, [], EPS, THR)
    cache = np.array([_delta_ub(nom0[y], qd[y], False) for y in range(N)])
    picks, pdelta, nref = [], [], 0

    def score(y, nA):
        _, nom, den = op.all_deltas(C, A[:nA], EPS, THR)
        P = 1.0 / (den[y] + EPS)                  # the exact P_yy
        corr = Qd[y] - P                          # |LQ^-1 q_Ay|^2, exact on the device too
        return _delta_ub(nom[y], qd[y] - corr, exact[y])

    for t in range(k):
        while True:
            m = np.where(sel, -np.inf, cache)
            c = int(np.flatnonzero(m == m.max())[0])
            if exact[c]:
                break
            qd[c] = Qd[c]
            exact[c] = True
            cache[c] = score(c, lastA[c])
            nref += 1
        picks.append(c)
        pdelta.append(cache[c])
        sel[c] = True
        A.append(c)
        cache[c] = 0.0
        if t == k - 1:
            break
        for y in op._window(c, shape, cutoff):
            if sel[y]:
                cache[y] = 0.0
                continue
            cache[y] = score(y, len(A))
            lastA[y] = len(A)
    return picks, pdelta, nref


@pytest.mark.parametrize("shape,k,cutoff,K", [((6, 6, 6), 8, 3, 8), ((7, 5, 6), 10, 2, 2),
                                              ((5, 6, 7), 12, 3, 1)])
def test_bounded_lazy_matches_oracle(shape, k, cutoff, K):
    """Picks and pick deltas equal the oracle's algorithm 3, also with brackets so wide (K = 1, 2)
    that most arg-maxes need a refinement and stale window entries get refined (lastA)."""
    C, Ce = _problem(shape, seed=sum(shape))
    offs, _ = taper_support(4.0)
    lo, hi = _gershgorin(Ce)
    Kb, scale, _ = bound_steps(offs, lo, hi, kmax=K)
    qhi = _cg_bounds(Ce, shape, offs, Kb, scale)
    picks, pdelta, nref = bounded_lazy_alg3(C, Ce, shape, k, cutoff, qhi)
    rA, _, rdci = op.placement_window_precision(C, k, shape, cutoff)
    assert picks == rA
    np.testing.assert_allclose(pdelta, [rdci[a, i] for i, a in enumerate(rA)], rtol=1e-12)
    assert nref >= k
    if K >= 8:
        assert nref <= 2 * k


def test_bound_steps_refuses_indefinite_bounds():
    offs, _ = taper_support(4.0)
    assert bound_steps(offs, -0.1, 2.0) is None
    K, scale, width = bound_steps(offs, 0.6, 1.41)
    assert K == 5 and width < 1e-6 and math.isclose(scale, (1 + 1e-12) / (1 - width))

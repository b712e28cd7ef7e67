"""Oracle (TEST INFRASTRUCTURE ONLY): numpy restatement of the reference's greedy MI placement.

Follows ``/root/reference/placement_algorithm2.py`` line by line in behaviour:

* ``placement_algorithm_2``  <- ``placement_algorithm2.py:151-219`` (lazy greedy, Krause Alg. 2)
* ``placement_algorithm_1``  <- ``placement_algorithm2.py:128-145`` (full greedy) with
  ``argmax_`` <- ``:105-125``
* ``argmax_cache_linear``    <- ``:53-67`` (strict ``<`` from -1: lowest index wins ties)
* ``nominator``              <- ``:371-388``;  ``denominator`` <- ``:408-413``
* ``call_pinv``              <- ``:399-405`` (1x1 inverted as ``1/a``, else ``np.linalg.pinv``)
* ``make_slice``             <- ``:391-396`` restated with ``np.ix_`` (same values, same dtype
  and shapes, so every downstream ``np.dot`` / ``pinv`` sees identical operands; only the
  O(N^2) Python copy loop is gone).

The pinv restatement is pinned bit-for-bit against golden traces produced by the reference itself
(``tests/golden/make_golden.py``).  ``placement_lazy_precision`` is an O(N^3 + k N^2) restatement
of the same lazy policy using Cholesky / precision-matrix algebra (the maths the HIP path uses);
it is pinned against the pinv restatement in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import numpy as np

DELTA_EPS = 1e-8  # placement_algorithm2.py:116, :198  (absolute thresholds on |nom|, |denom|)


def make_slice(cov_vv, y, A):
    """placement_algorithm2.py:391-396 — copy cov_vv[y_i, A_j] into a fresh float64 [len(y), len(A)]."""
    out = np.zeros(shape=[len(y), len(A)])
    if len(y) and len(A):
        out[...] = cov_vv[np.ix_(np.asarray(y, dtype=np.int64), np.asarray(A, dtype=np.int64))]
    return out


def call_pinv(a):
    """placement_algorithm2.py:399-405."""
    assert a.shape[0] == a.shape[1]
    if a.shape[0] == 1:
        return 1 / a
    return np.linalg.pinv(a)


def nominator(y, A, cov_vv):
    """placement_algorithm2.py:371-388 — sigma_yy - Sigma_yA pinv(Sigma_AA) Sigma_Ay (a 1x1 array)."""
    A_ = list(A)
    sigm_yy = make_slice(cov_vv, [y], [y])
    if len(A_) == 0:
        return sigm_yy
    cov_yA = make_slice(cov_vv, [y], A_)
    cov_AA = make_slice(cov_vv, A_, A_)
    cov_Ay = make_slice(cov_vv, A_, [y])
    inv_cov_AA = call_pinv(cov_AA)
    dot_yA_iAA = np.dot(cov_yA, inv_cov_AA)
    dot_yAiAA_Ay = np.dot(dot_yA_iAA, cov_Ay)
    return sigm_yy - dot_yAiAA_Ay


def denominator(y, A_hat, cov_vv):
    """placement_algorithm2.py:408-413 — nominator over A_hat without y."""
    A_hat_ = list(A_hat)
    if y in A_hat_:
        A_hat_.remove(int(y))
    return nominator(y, A_hat_, cov_vv)


def _delta(nom, denom):
    """placement_algorithm2.py:193-203 / :116-119."""
    if np.abs(denom) < DELTA_EPS or np.abs(nom) < DELTA_EPS:
        return 0
    return nom / denom


def argmax_cache_linear(cache, A, V):
    """placement_algorithm2.py:53-67."""
    y_st = -1
    delta_st = -1
    Aset = set(int(a) for a in A)
    for y in V:
        if int(y) in Aset:
            continue
        delta_y = cache[y]
        if delta_st < delta_y:
            delta_st = delta_y
            y_st = y
    return y_st


def placement_algorithm_2(cov_vv, k, trace=None):
    """placement_algorithm2.py:151-219 — lazy greedy.  ``trace`` (list) receives one
    ``(y, delta)`` tuple per delta evaluation (the reference prints these at :205) and
    ``('select', y)`` per selection (:188)."""
    cov_vv = np.asarray(cov_vv, dtype=np.float64)
    A = []
    V = np.linspace(0, cov_vv.shape[0] - 1, cov_vv.shape[0], dtype=np.int64)
    A_bar = list(V)
    INF = float("inf")
    delta_cached = [INF] * len(V)
    uptodate = [False] * len(V)
    while len(A) < k:
        for i in range(len(uptodate)):
            uptodate[i] = False
        while True:
            y_st = argmax_cache_linear(delta_cached, A, V)
            if uptodate[y_st]:
                if trace is not None:
                    trace.append(("select", int(y_st)))
                break
            nom = nominator(y_st, A, cov_vv)
            denom = denominator(y_st, A_bar, cov_vv)
            delta_y = _delta(nom, denom)
            if trace is not None:
                trace.append((int(y_st), float(np.asarray(delta_y).reshape(-1)[0])))
            delta_cached[y_st] = delta_y
            uptodate[y_st] = True
        A.append(y_st)
        A_bar.remove(y_st)
    return A


def placement_algorithm_1(cov_vv, k):
    """placement_algorithm2.py:128-145 (with argmax_ :105-125) — full greedy."""
    cov_vv = np.asarray(cov_vv, dtype=np.float64)
    A = []
    V = np.linspace(0, cov_vv.shape[0] - 1, cov_vv.shape[0], dtype=np.int64)
    A_bar = list(V)
    while len(A) < k:
        y_st, delta_st = -1, -1
        Aset = set(int(a) for a in A)
        for y in V:
            if int(y) in Aset:
                continue
            delta_y = _delta(nominator(y, A, cov_vv), denominator(y, A_bar, cov_vv))
            if delta_st < delta_y:
                delta_st = delta_y
                y_st = y
        A.append(y_st)
        A_bar.remove(y_st)
    return A


# ---------------------------------------------------------------------------------------------
# Precision-matrix restatement (same decisions, O(N^3) once + O(kN^2)): pinned against the above.
# ---------------------------------------------------------------------------------------------
def all_deltas(cov_vv, A):
    """delta_y(A) for every y (selected entries -> nan), via
    nom_y   = sigma_yy - Sigma_yA Sigma_AA^-1 Sigma_Ay
    denom_y = 1 / [(Sigma_SS)^-1]_yy,   S = V \\ A  (conditional variance given S \\ {y})."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    A = [int(a) for a in A]
    S = np.setdiff1d(np.arange(N), np.asarray(A, dtype=np.int64))
    nom = np.full(N, np.nan)
    den = np.full(N, np.nan)
    diag = np.diag(cov)
    if A:
        LA = np.linalg.cholesky(cov[np.ix_(A, A)])
        W = np.linalg.solve(LA, cov[A, :])
        nom[S] = diag[S] - np.sum(W[:, S] ** 2, axis=0)
    else:
        nom[S] = diag[S]
    if len(S) == 1:
        den[S] = diag[S]
    elif len(S) > 1:
        P = np.linalg.inv(cov[np.ix_(S, S)])
        den[S] = 1.0 / np.diag(P)
    delta = np.full(N, np.nan)
    ok = (np.abs(nom[S]) >= DELTA_EPS) & (np.abs(den[S]) >= DELTA_EPS)
    d = np.zeros(len(S))
    d[ok] = nom[S][ok] / den[S][ok]
    delta[S] = d
    return delta, nom, den


def lazy_select(cache, fresh_delta, selected):
    """Emulate one round of the reference's lazy loop (placement_algorithm2.py:173-214) given the
    stale cache and the fresh deltas of this round.  Returns (y*, evaluated indices in order);
    updates ``cache`` in place."""
    N = len(cache)
    uptodate = np.zeros(N, dtype=bool)
    evaluated = []
    while True:
        y_st, d_st = -1, -1.0
        for y in range(N):
            if selected[y]:
                continue
            if d_st < cache[y]:
                d_st, y_st = cache[y], y
        if uptodate[y_st]:
            return y_st, evaluated
        cache[y_st] = fresh_delta[y_st]
        uptodate[y_st] = True
        evaluated.append(y_st)


def placement_lazy_precision(cov_vv, k, lazy=True):
    """Same selections as placement_algorithm_2 (lazy=True) / _1 (lazy=False) up to rounding."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    cache = np.full(N, np.inf)
    selected = np.zeros(N, dtype=bool)
    A = []
    for _ in range(k):
        delta, _, _ = all_deltas(cov, A)
        if lazy:
            y, _ = lazy_select(cache, delta, selected)
        else:
            d = np.where(selected, -np.inf, delta)
            y = int(np.argmax(d))
        A.append(int(y))
        selected[y] = True
    return A

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
def all_deltas(cov_vv, A, jitter=0.0, thr=DELTA_EPS):
    """delta_y(A) for every y (selected entries -> nan), via
    nom_y   = sigma_yy - Sigma_yA (Sigma_AA + eps I)^-1 Sigma_Ay
    denom_y = 1 / [(Sigma_SS + eps I)^-1]_yy - eps,   S = V \\ A
    (the conditional variance of y given S \\ {y} with eps on that block's diagonal; eps = 0 for
    placement_algorithm2, 1e-6 for the TF variant)."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    A = [int(a) for a in A]
    S = np.setdiff1d(np.arange(N), np.asarray(A, dtype=np.int64))
    nom = np.full(N, np.nan)
    den = np.full(N, np.nan)
    diag = np.diag(cov)
    if A:
        LA = np.linalg.cholesky(cov[np.ix_(A, A)] + jitter * np.eye(len(A)))
        W = np.linalg.solve(LA, cov[A, :])
        nom[S] = diag[S] - np.sum(W[:, S] ** 2, axis=0)
    else:
        nom[S] = diag[S]
    if len(S) == 1:
        den[S] = diag[S]
    elif len(S) > 1:
        P = np.linalg.inv(cov[np.ix_(S, S)] + jitter * np.eye(len(S)))
        den[S] = 1.0 / np.diag(P) - jitter
    delta = np.full(N, np.nan)
    ok = (np.abs(nom[S]) >= thr) & (np.abs(den[S]) >= thr)
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


def placement_lazy_precision(cov_vv, k, lazy=True, jitter=0.0, thr=DELTA_EPS, cache_init=np.inf,
                             snapshots=None):
    """Same selections as placement_algorithm_2 (lazy=True) / _1 (lazy=False) up to rounding;
    with (jitter, thr, cache_init) = (1e-6, 1e-7, 1e8) and ``snapshots`` (a list receiving the
    cache after each round, the selected entry then zeroed) it restates the TF variant
    ``sparse_placement_algorithm_2`` below."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    cache = np.full(N, float(cache_init))
    selected = np.zeros(N, dtype=bool)
    A = []
    for _ in range(k):
        delta, _, _ = all_deltas(cov, A, jitter, thr)
        if lazy:
            y, _ = lazy_select(cache, delta, selected)
        else:
            d = np.where(selected, -np.inf, delta)
            y = int(np.argmax(d))
        A.append(int(y))
        selected[y] = True
        if snapshots is not None:
            snapshots.append(cache.copy())
            cache[y] = 0.0
    return A


def _lazy_select_np(cache, fresh_delta, selected):
    """lazy_select with numpy scans (same decisions: the first maximum of the non-selected cache
    is the lowest index among ties, placement_algorithm2.py:53-67; NaN never wins)."""
    uptodate = np.zeros(len(cache), dtype=bool)
    evaluated = []
    while True:
        c = np.where(selected | np.isnan(cache), -np.inf, cache)
        y = int(np.argmax(c))
        if uptodate[y]:
            return y, evaluated
        cache[y] = fresh_delta[y]
        uptodate[y] = True
        evaluated.append(y)


def placement_lazy_incremental(cov_vv, k, lazy=True, jitter=0.0, thr=DELTA_EPS, cache_init=np.inf,
                               deltas_out=None, timings=None):
    """placement_lazy_precision with O(N^3) once + O(N^2) per round, for N ~ 16k (the GPU test of a
    full k = 50 sequence).  Same deltas, rank-1 updated instead of re-factored:
      nom_y  = sigma_yy - |W[:, y]|^2,  W[t] = (Sigma_{a_t,:} - W^T W[:, a_t]) / sqrt(pivot_t)
               (pivot_t = sigma_{a_t a_t} + eps - |W[:, a_t]|^2: Cholesky of Sigma_AA + eps I);
      P_yy   = Q_yy - |V[:, y]|^2,  Q = (Sigma + eps I)^-1,  V[t] = (Q e_{a_t} - V^T V[:, a_t]) /
               sqrt(P_{a_t a_t}): removing a_t from S = V \\ A downdates (Sigma_SS + eps I)^-1;
      denom_y = 1 / P_yy - eps.
    Pinned against placement_lazy_precision and the reference goldens in tests/test_oracle.py."""
    import time

    from scipy.linalg import lapack
    t0 = time.perf_counter()
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    Mj = cov.copy()
    Mj[np.diag_indices(N)] += jitter
    c, info = lapack.dpotrf(Mj, lower=1, clean=0, overwrite_a=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dpotrf info {info}")
    Q, info = lapack.dpotri(c, lower=1, overwrite_c=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dpotri info {info}")
    del c, Mj
    Q = np.tril(Q) + np.tril(Q, -1).T
    t1 = time.perf_counter()
    A = placement_lazy_columns(np.diag(cov).copy(), lambda y: cov[y], np.diag(Q).copy(),
                               lambda y: Q[y], k, lazy=lazy, jitter=jitter, thr=thr,
                               cache_init=cache_init, deltas_out=deltas_out)
    if timings is not None:  # the O(N^3) factor + inverse and the O(k N^2) rounds, in seconds
        timings.update(factor_inverse=t1 - t0, rounds=time.perf_counter() - t1)
    return A


def placement_lazy_columns(sigma_diag, sigma_row, q_diag, q_col, k, lazy=True, jitter=0.0,
                           thr=DELTA_EPS, cache_init=np.inf, deltas_out=None, margins_out=None,
                           log=None):
    """The rounds of placement_lazy_incremental from callbacks, so a caller can hold Sigma and
    Q = (Sigma + eps I)^-1 however it likes (tests/golden/make_golden_65k.py keeps only the
    in-place dpotri buffer of N = 65,536 and rebuilds Sigma's rows from the points):
    ``sigma_diag`` [N], ``sigma_row(y)`` -> Sigma e_y, ``q_diag`` [N] = diag(Q),
    ``q_col(y)`` -> Q e_y.  Same arithmetic, same decisions (placement_algorithm2.py:151-219).
    ``margins_out`` receives each round's margin: the pick's value minus the best other
    non-selected entry it was chosen over (the cache when lazy, the fresh deltas otherwise)."""
    N = len(sigma_diag)
    diag = np.asarray(sigma_diag, dtype=np.float64)
    nom = diag.copy()
    prec = np.asarray(q_diag, dtype=np.float64).copy()
    W = np.zeros((k, N))
    V = np.zeros((k, N))
    cache = np.full(N, float(cache_init))
    selected = np.zeros(N, dtype=bool)
    A = []
    for r in range(k):
        with np.errstate(divide="ignore", invalid="ignore"):
            den = 1.0 / prec - jitter
            ok = (np.abs(nom) >= thr) & (np.abs(den) >= thr)
            delta = np.where(ok, nom / den, 0.0)
        delta[selected] = np.nan
        if lazy:
            y, _ = _lazy_select_np(cache, delta, selected)
        else:
            d = np.where(selected | np.isnan(delta), -np.inf, delta)
            y = int(np.argmax(d))
        if deltas_out is not None:
            deltas_out.append(float(delta[y]))
        if margins_out is not None:
            other = np.where(selected | np.isnan(cache if lazy else delta), -np.inf,
                             cache if lazy else delta)
            other[y] = -np.inf
            margins_out.append(float(delta[y] - other.max()) if N > 1 else float("inf"))
        A.append(y)
        selected[y] = True
        if log is not None:
            log(r, y, float(delta[y]))
        w = (sigma_row(y) - W[:r].T @ W[:r, y]) / np.sqrt(diag[y] + jitter - W[:r, y] @ W[:r, y])
        W[r] = w
        nom = nom - w * w
        v = (q_col(y) - V[:r].T @ V[:r, y]) / np.sqrt(prec[y])
        V[r] = v
        prec = prec - v * v
    return A


# ---------------------------------------------------------------------------------------------
# The TF-graph variant: snippets_a2.sparse_placement_algorithm_2 (snippets_a2.py:679-822).
# TensorFlow is absent, so this is a restatement from the source (parity unpinned by execution);
# with TF_JITTER = 0, TF_SMALL = 1e-8 and TF_INF = inf it reduces to placement_algorithm_2 above,
# which IS pinned by the reference's own outputs.
# ---------------------------------------------------------------------------------------------
TF_JITTER = 1e-6   # snippets_a2.py:161-163  (diag of cov_AA += 1e-6 before pinv)
TF_SMALL = 1e-7    # snippets_a2.py:480  (if_denom_is_near_zero)
TF_INF = 1e8       # snippets_a2.py:690


def tf_pinv(a):
    """tfp.math.pinv with its default rcond = 10 * max(rows, cols) * eps(float64)."""
    return np.linalg.pinv(a, rcond=10.0 * max(a.shape) * np.finfo(np.float64).eps)


def tf_nominator(y, A, cov_vv, jitter=TF_JITTER):
    """snippets_a2.py:138-213 — sigma_yy - Sigma_yA pinv(Sigma_AA + eps I) Sigma_Ay, A \\ {y}."""
    A_ = sorted(int(a) for a in set(A) - {int(y)})   # tf.sets keep their values sorted
    sigm_yy = cov_vv[y, y]
    if not A_:
        return sigm_yy
    cov_yA = cov_vv[y, A_]
    cov_AA = cov_vv[np.ix_(A_, A_)].copy()
    cov_AA[np.diag_indices(len(A_))] += jitter
    cov_Ay = cov_vv[A_, y]
    mul1 = np.tensordot(cov_yA, tf_pinv(cov_AA), [[0], [0]])
    return sigm_yy - np.tensordot(mul1, cov_Ay, [[0], [0]])


def tf_denominator(y, A_hat, cov_vv, jitter=TF_JITTER):
    """snippets_a2.py:215-217."""
    return tf_nominator(y, set(A_hat) - {int(y)}, cov_vv, jitter)


def sparse_argmax_cache_linear(cache, A, N):
    """placement_algorithm2.py:24-50 — max over V \\ A (ascending), first (lowest) index of ties."""
    Aset = set(A)
    cand = np.array([v for v in range(N) if v not in Aset], dtype=np.int64)
    vals = cache[cand]
    return int(cand[np.flatnonzero(vals == vals.max())[0]])


def sparse_placement_algorithm_2(cov_vv, k, COVER_spatial, trace=None, jitter=TF_JITTER,
                                 small=TF_SMALL, inf=TF_INF):
    """snippets_a2.py:679-822.  Returns (A sorted as the tf.sets SparseTensor values, len(A),
    delta_cached_iters [N, k], A_selection_and_delta [k, 2]).  The keyword constants exist so
    tests can set them to placement_algorithm_2's (0, 1e-8, inf) and pin against its goldens."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    if N != int(np.prod(COVER_spatial[:3])):                       # :692 tf.Assert
        raise ValueError(f"N = {N} != prod(COVER_spatial) = {int(np.prod(COVER_spatial[:3]))}")
    A, A_bar = [], list(range(N))
    cache = np.full(N, float(inf))                                     # :708
    dci = np.zeros((N, k))
    sel = np.zeros((k, 2))
    for r in range(k):                                             # body_A :717-802
        uptodate = np.zeros(N, dtype=bool)                         # :722
        while True:                                                # while_true_outside / _inside
            y = sparse_argmax_cache_linear(cache, A, N)
            if uptodate[y]:
                break
            nom = tf_nominator(y, A, cov, jitter)
            denom = tf_denominator(y, A_bar, cov, jitter)
            near = abs(denom) < small or abs(nom) < small
            cache[y] = 0.0 if near else nom / denom                 # then_update_delta_y
            uptodate[y] = True
            if trace is not None:
                trace.append((y, float(cache[y])))
        A.append(y)                                                # append_to_A_remove_from_A_bar
        A_bar.remove(y)
        sel[r] = (y, cache[y])                                     # :767-768
        dci[:, r] = cache                                          # :778
        cache[y] = 0.0                                             # :796
    return sorted(A), len(A), dci, sel


# ---------------------------------------------------------------------------------------------
# Placement algorithm 3, the local-kernel greedy: snippets_a3.sparse_placement_algorithm_3
# (snippets_a3.py:43-330).  TensorFlow is absent: restated from the source (parity unpinned by
# execution).  Deltas are the TF variant's (tf_nominator / tf_denominator, jitter 1e-6,
# threshold 1e-7, INF 1e8); after each pick only the index window around it is re-scored.
# ---------------------------------------------------------------------------------------------
def _window(y, cover, cutoff):
    I0, I1, I2 = (int(c) for c in cover[:3])
    i0, r = divmod(int(y), I1 * I2)
    i1, i2 = divmod(r, I2)
    for j0 in range(max(i0 - cutoff, 0), min(i0 + cutoff, I0)):      # :300-305 (upper exclusive)
        for j1 in range(max(i1 - cutoff, 0), min(i1 + cutoff, I1)):  # :284-289
            for j2 in range(max(i2 - cutoff, 0), min(i2 + cutoff, I2)):  # :268-273
                yield j0 * I1 * I2 + j1 * I2 + j2


def sparse_placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff, order=None, jitter=TF_JITTER,
                                 small=TF_SMALL):
    """snippets_a3.py:43-330 -> (A sorted, final cache [N], delta_cached_iters [N, k]).
    ``order`` (list) receives the picks in selection order."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    if N != int(np.prod(COVER_spatial[:3])):                        # :51 tf.Assert
        raise ValueError("N != prod(COVER_spatial)")
    A, A_bar = [], list(range(N))

    def delta(y):                                                   # body_D :72-112
        nom = tf_nominator(y, A, cov, jitter)
        denom = tf_denominator(y, A_bar, cov, jitter)
        return 0.0 if (abs(denom) < small or abs(nom) < small) else nom / denom

    cache = np.full(N, TF_INF)
    dci = np.zeros((N, k))
    for y in range(N):                                              # :116-119 (loop_D)
        cache[y] = delta(y)
    dci[:, 0] = cache                                               # :121-124
    for i in range(k - 1):                                          # body_A :127-322
        y = sparse_argmax_cache_linear(cache, A, N)
        A.append(y)
        A_bar.remove(y)
        cache[y] = 0.0                                              # :151-156
        for yj in _window(y, COVER_spatial, cutoff):                # :196-308
            cache[yj] = 0.0 if yj in A else delta(yj)
        cache[y] = 0.0                                              # :309-314
        dci[:, i + 1] = cache                                       # :315-320
    y = sparse_argmax_cache_linear(cache, A, N)                     # :326-328
    A.append(y)
    if order is not None:
        order.extend(A)
    return sorted(A), cache, dci


def placement_window_precision(cov_vv, k, COVER_spatial, cutoff, jitter=TF_JITTER, thr=TF_SMALL):
    """Algorithm 3 with the precision-matrix deltas (the HIP path's algebra): (order, cache, dci)."""
    cov = np.asarray(cov_vv, dtype=np.float64)
    N = cov.shape[0]
    A = []
    delta, _, _ = all_deltas(cov, A, jitter, thr)
    cache = delta.copy()
    dci = np.zeros((N, k))
    dci[:, 0] = cache
    sel = np.zeros(N, dtype=bool)
    for i in range(k - 1):
        y = int(np.flatnonzero(~sel)[np.argmax(cache[~sel])])
        A.append(y)
        sel[y] = True
        delta, _, _ = all_deltas(cov, A, jitter, thr)
        cache[y] = 0.0
        for yj in _window(y, COVER_spatial, cutoff):
            cache[yj] = 0.0 if sel[yj] else delta[yj]
        dci[:, i + 1] = cache
    y = int(np.flatnonzero(~sel)[np.argmax(cache[~sel])])
    A.append(y)
    return A, cache, dci

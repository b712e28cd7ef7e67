"""Oracle (TEST INFRASTRUCTURE ONLY): numpy restatement of the local-kernel greedy of config C4.

Config C4 (128^3 = 2,097,152 candidates, k = 50) cannot form the dense cov_vv (35 TB), so it runs
the reference's own locality idea, the epsilon-local algorithm 3:

* **The local kernel** is the beta-decay taper of
  ``main_architecture_2_sampledistribution.py:355-421``: cov(u, v) is multiplied by
  ``exp(-(beta * delta)^2 / (2 pi))`` (delta = Euclidean distance of the C-order grid indices,
  ``:375-378``, ``:390-393``) and set to 0 where that decay is < 0.01 (``:417-420``).  With the
  reference's ``BETA_val = 4`` (``:779``, ``:973``) only the 6 face neighbours survive.
* **The local deltas** are Krause's ``H(y) - Hhat_epsilon(y | V \\ y)`` that
  ``snippets_a3.py:63`` and ``:182-186`` name ("VI. foreach y E N(y*; epsilon) ... O(epsilon N2)"):
  conditioning is restricted to the taper support N(y) = {u != y : decay(u, y) >= 0.01}:
      nom_y   = s_yy - s_yB (S_BB + eps I)^-1 s_By,   B = A ∩ N(y)
      denom_y = s_yy - s_yB (S_BB + eps I)^-1 s_By,   B = N(y) \\ A
  with the TF variant's constants (eps = 1e-6 on the conditioning block, snippets_a2.py:161-163;
  delta = 0 when |nom| or |denom| < 1e-7, snippets_a2.py:480).  The reference's executable
  snippets_a3 evaluates these over the FULL sets A and V \\ A of a dense matrix; restricted to
  N(y) they depend on A only through A ∩ N(y), so a pick y* changes only the deltas of N(y*) and
  the reference's window re-score (``snippets_a3.py:190-303``) keeps the cache exact whenever the
  window covers the taper support.  That restriction is the approximation this config makes;
  against the reference's dense algorithm 3 it is parity UNPINNED (TF is absent and no
  reference test covers it) — the GPU path is pinned to THIS restatement, indices bit-exact.
* **The cache policy** is ``snippets_a3.py:43-364`` exactly: every candidate scored once
  (``:77-124``), then per round arg-max over V \\ A with the lowest index winning ties
  (``placement_algorithm2.py:24-50``), cache[y*] = 0 (``:162-168``), re-score the index window
  ``[i_d - cutoff, i_d + cutoff)`` per axis (selected entries -> 0, ``:252-254``), snapshot into
  ``delta_cached_iters`` (``:318-332``); after k - 1 rounds a last arg-max adds the k-th pick
  (``:360-362``).

The covariance itself is s(u, v) = decay(u, v) * (K(x_u, x_v) + diag_shift [u == v]) with K the
PSD kernel of ``oracle.gp`` (TFP's ``exp(2 log amp + log k(r / ls))``) on the grid points X.
"""
from __future__ import annotations

import numpy as np

from .gp import _log_k

TAPER_FLOOR = 0.01   # main_architecture_2_sampledistribution.py:392, :417
TF_JITTER = 1e-6     # snippets_a2.py:161-163
TF_SMALL = 1e-7      # snippets_a2.py:480
TF_INF = 1e8         # snippets_a3.py:49


def decay(beta, d2):
    """main_architecture_2_sampledistribution.py:375-393 for integer squared index distances d2."""
    delta = np.abs(np.sqrt(np.asarray(d2, dtype=np.float64)))
    g = np.exp(-np.square(beta * delta) / (2 * np.pi))
    return np.where(g < TAPER_FLOOR, 0.0, g)


def taper_support(beta):
    """(offsets [m-1, 3] int64 in lexicographic = C-order, tau[d2] table) of the taper support
    N(0) \\ {0}: every index offset whose decay is >= 0.01."""
    beta = float(beta)
    r = 0
    while decay(beta, (r + 1) ** 2) > 0:
        r += 1
    rng = np.arange(-r, r + 1)
    o = np.stack(np.meshgrid(rng, rng, rng, indexing="ij"), -1).reshape(-1, 3)
    d2 = (o ** 2).sum(1)
    keep = (decay(beta, d2) > 0) & (d2 > 0)
    offs = o[keep].astype(np.int64)
    tau = decay(beta, np.arange(4 * 3 * r * r + 1))
    return offs, tau


def _kern(kind, d2, amp, ls):
    return np.exp(2.0 * np.log(amp) + _log_k(kind, d2, ls))


def local_deltas(X, shape, cand, selected, beta, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
                 jitter=TF_JITTER, thr=TF_SMALL, chunk=1 << 17):
    """delta_y for the candidates ``cand`` (flat indices) given the selected mask: the local nom /
    denom above, each the last Schur complement of an (m x m) matrix with y ordered last and the
    excluded neighbours (outside the grid, or on the other side of the A split) replaced by
    identity rows (they then contribute exactly nothing)."""
    X = np.asarray(X, dtype=np.float64)
    I0, I1, I2 = (int(s) for s in shape)
    offs, tau = taper_support(beta)
    m = len(offs) + 1
    cand = np.asarray(cand, dtype=np.int64)
    out = np.empty(len(cand))
    do = offs[:, None, :] - offs[None, :, :]
    tau_pair = tau[(do ** 2).sum(-1)]                               # [m-1, m-1]
    tau_y = tau[(offs ** 2).sum(-1)]                                # [m-1]
    kdiag = _kern(kind, 0.0, amp, ls)
    for s in range(0, len(cand), chunk):
        y = cand[s:s + chunk]
        n = len(y)
        iy = np.stack([y // (I1 * I2), (y // I2) % I1, y % I2], 1)
        iu = iy[:, None, :] + offs[None, :, :]                      # [n, m-1, 3]
        valid = np.all((iu >= 0) & (iu < np.array([I0, I1, I2])), axis=-1)
        u = np.where(valid, (iu[..., 0] * I1 + iu[..., 1]) * I2 + iu[..., 2], 0)
        xu = X[u]                                                   # [n, m-1, d]
        xy = X[y]
        Kuu = _kern(kind, ((xu[:, :, None, :] - xu[:, None, :, :]) ** 2).sum(-1), amp, ls)
        Kuy = _kern(kind, ((xu - xy[:, None, :]) ** 2).sum(-1), amp, ls)
        G = np.zeros((n, m, m))
        G[:, :m - 1, :m - 1] = tau_pair * Kuu
        G[:, :m - 1, m - 1] = tau_y * Kuy
        G[:, m - 1, :m - 1] = tau_y * Kuy
        idx = np.arange(m - 1)
        G[:, idx, idx] = kdiag + diag_shift + jitter
        G[:, m - 1, m - 1] = kdiag + diag_shift
        insel = selected[u] & valid
        res = []
        for keep in (insel, valid & ~insel):                       # nominator, denominator
            H = G.copy()
            drop = ~keep
            H[:, :m - 1, :][drop] = 0.0
            H[:, :, :m - 1] = np.where(drop[:, None, :], 0.0, H[:, :, :m - 1])
            dd = np.where(drop, 1.0, H[:, idx, idx])
            H[:, idx, idx] = dd
            L = np.linalg.cholesky(H)
            res.append(L[:, m - 1, m - 1] ** 2)
        nom, den = res
        ok = (np.abs(nom) >= thr) & (np.abs(den) >= thr)
        d = np.where(ok, nom / np.where(ok, den, 1.0), 0.0)
        d[selected[y]] = 0.0
        out[s:s + n] = d
    return out


def window(y, shape, cutoff):
    """snippets_a3.py:190-303: flat indices of [i_d - cutoff, i_d + cutoff) per axis, C order."""
    I0, I1, I2 = (int(s) for s in shape)
    i0, r = divmod(int(y), I1 * I2)
    i1, i2 = divmod(r, I2)
    j0 = np.arange(max(i0 - cutoff, 0), min(i0 + cutoff, I0))
    j1 = np.arange(max(i1 - cutoff, 0), min(i1 + cutoff, I1))
    j2 = np.arange(max(i2 - cutoff, 0), min(i2 + cutoff, I2))
    return ((j0[:, None, None] * I1 + j1[None, :, None]) * I2 + j2[None, None, :]).reshape(-1)


def _argmax(cache, selected):
    """placement_algorithm2.py:24-50: max over V \\ A, the lowest index among ties."""
    c = np.where(selected, -np.inf, cache)
    return int(np.argmax(c))


def local_placement_algorithm_3(X, shape, k, cutoff, beta, kind="eq", amp=1.0, ls=1.0,
                                diag_shift=0.0, snapshots=False, deltas=None):
    """snippets_a3.sparse_placement_algorithm_3 with the local deltas above.
    -> (picks in selection order, final cache [N], delta_cached_iters [N, k] or None).
    ``deltas`` (list) receives the cache value of each pick when it was selected."""
    I0, I1, I2 = (int(s) for s in shape)
    N = I0 * I1 * I2
    if len(X) != N:                                                 # snippets_a3.py:51
        raise ValueError(f"N = {len(X)} != prod(COVER_spatial) = {N}")
    selected = np.zeros(N, dtype=bool)
    kw = dict(kind=kind, amp=amp, ls=ls, diag_shift=diag_shift)
    cache = local_deltas(X, shape, np.arange(N), selected, beta, **kw)   # :77-124
    dci = np.zeros((N, k)) if snapshots else None
    if snapshots:
        dci[:, 0] = cache
    A = []
    for i in range(k - 1):                                          # body_A :137-350
        y = _argmax(cache, selected)
        if deltas is not None:
            deltas.append(float(cache[y]))
        A.append(y)
        selected[y] = True
        cache[y] = 0.0                                              # :162-168
        w = window(y, shape, cutoff)
        cache[w] = local_deltas(X, shape, w, selected, beta, **kw)  # :205-303 (A -> 0)
        cache[y] = 0.0                                              # :318-325
        if snapshots:
            dci[:, i + 1] = cache
    y = _argmax(cache, selected)                                    # :360-362
    if deltas is not None:
        deltas.append(float(cache[y]))
    A.append(y)
    return A, cache, dci


def tapered_cov(X, shape, beta, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0):
    """The dense tapered covariance (small grids only): what the reference's arch2 filter builds
    and its dense algorithm 3 consumes."""
    from .covariance import index_taper
    from .gp import kernel_matrix
    K = kernel_matrix(kind, X, X, amp, ls)[0]
    K[np.diag_indices(len(X))] += diag_shift
    return index_taper(K, shape, beta)

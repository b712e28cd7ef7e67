"""Greedy mutual-information sensor placement on MI355X — drop-in for the reference's
``placement_algorithm2`` module (``/root/reference/placement_algorithm2.py``).

Same names, argument meaning and results:

* ``placement_algorithm_2(cov_vv, k)``  lazy greedy, Krause Alg. 2    (reference :151-219)
* ``placement_algorithm_1(cov_vv, k)``  full greedy                   (reference :128-145)
* ``cov_vv_4x4()``                      the reference's 4x4 fixture    (reference :473-479)
* ``dg_create_random_cov(n)``           U U^T test covariance          (reference :441-444)

``cov_vv`` is an [N, N] float64 covariance (numpy array or device tensor); the result is a Python
list of ``np.int64`` indices in selection order.  The computation runs entirely in libvgposp
(``vgposp_greedy_init`` / ``vgposp_greedy_step``): one in-place Cholesky + inverse of Sigma, then
per selection one HBM-bound triangular mat-vec and a handful of O(N) kernels; the lazy-cache
decisions of the reference are reproduced exactly on device (see csrc/greedy.hip).

``GreedyPlacement`` is the device-resident form used by ``bench.py`` (inputs already in HBM, no
host round trip between selections).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import linalg
from ._lib import CholeskyError, call, query
from .linalg import _p, _stream


class GreedyPlacement:
    """Device-resident greedy placement on an [N, N] covariance held in HBM.

    ``Sigma`` (float64, contiguous, lda = N) is FACTORED IN PLACE by ``init()``: its lower triangle
    becomes L^-1, the strictly upper triangle (Sigma itself) and the saved diagonal are what the
    nominators read.  Pass ``copy=True`` to work on a private copy.
    """

    def __init__(self, Sigma, kmax, copy=False, jitter=0.0, threshold=1e-8,
                 cache_init=float("inf"), pad_odd=False):
        S = linalg.as_device(Sigma)
        if S.dim() != 2 or S.shape[0] != S.shape[1]:
            raise ValueError("cov_vv must be a square matrix")
        self.N = int(S.shape[0])                     # candidates
        if not (1 <= kmax <= self.N):
            raise ValueError(f"k must be in [1, {self.N}], got {kmax}")
        # pad_odd (with copy): an odd order is factored as [Sigma 0; 0 s] at N + 1, so every
        # recursion level runs on the fast (even-leading-dimension) GEMM; the padding candidate is
        # excluded on device after init (vgposp_greedy_exclude) and couples to nothing
        self.padded = bool(pad_odd and copy and self.N % 2 == 1 and self.N > 1)
        if self.padded:
            n = self.N
            P = torch.zeros((n + 1, n + 1), dtype=torch.float64, device=S.device)
            P[:n, :n].copy_(S)
            P[n, n] = torch.diagonal(S).mean()
            self.S = P
        else:
            self.S = S.clone() if copy else S
        self.n = int(self.S.shape[0])                # the library's order
        self.kmax = int(kmax)
        dev = self.S.device
        self.ws = linalg.workspace(query("vgposp_greedy_workspace_bytes", self.n, self.kmax))
        self.info = torch.zeros(1, dtype=torch.int32, device=dev)
        self.selected = torch.full((self.kmax,), -1, dtype=torch.int64, device=dev)
        self.sel_delta = torch.zeros(self.kmax, dtype=torch.float64, device=dev)
        self.evals = torch.zeros(self.kmax, dtype=torch.int64, device=dev)
        self.rounds = 0
        # (jitter, |nom|/|denom| threshold, initial cache): (0, 1e-8, inf) is placement_algorithm2;
        # (1e-6, 1e-7, 1e8) is the TF variant snippets_a2.sparse_placement_algorithm_2
        self.params = (float(jitter), float(threshold), float(cache_init))

    def init(self):
        call("vgposp_greedy_init_ex", _p(self.S), self.n, self.S.stride(0), self.kmax,
             *self.params, _p(self.info), _p(self.ws), self.ws.numel(), _stream())
        if self.padded:
            call("vgposp_greedy_exclude", _p(self.ws), self.n, self.kmax, self.N, _stream())
        self.rounds = 0
        return self

    def cache(self):
        """Device view of the lazy cache (delta_cached) [n] inside the workspace."""
        c = ctypes.c_void_p()
        call("vgposp_greedy_cache", _p(self.ws), self.n, self.kmax, ctypes.byref(c))
        off = c.value - self.ws.data_ptr()
        return self.ws[off:off + 8 * self.N].view(torch.float64)

    def check(self):
        linalg.check_info(self.info)

    def step(self, lazy=True):
        if self.rounds >= self.kmax:
            raise RuntimeError("all k sensors already placed")
        call("vgposp_greedy_step", _p(self.S), self.n, self.S.stride(0), self.kmax, self.rounds,
             int(lazy), _p(self.selected), _p(self.sel_delta), _p(self.evals), _p(self.ws),
             self.ws.numel(), _stream())
        self.rounds += 1

    def run(self, k=None, lazy=True):
        k = self.kmax if k is None else k
        self.init()
        for _ in range(k):
            self.step(lazy)
        return self

    def step_traced(self, trace):
        """A lazy step() that also appends the reference's per-evaluation records to ``trace``: one
        ``(y, delta_y)`` per delta evaluated this round, in the reference's order, then
        ``('select', y*)`` — what placement_algorithm2.py:205 and :188 print.

        The lazy loop (:183-208) evaluates the stale cache entries in descending key order (value,
        then lower index) and stops at the first fresh arg-max, so the evaluated entries are the
        first ``evals[r]`` of the pre-round cache sorted by key, and their deltas are the
        post-round cache values.  The device makes every decision; this only reads back the two
        cache states and the evaluation count."""
        r = self.rounds
        cache = self.cache()
        key = torch.nan_to_num(cache.clone(), nan=-float("inf"))
        if r:
            key[self.selected[:r]] = -float("inf")
        self.step(lazy=True)
        order = torch.sort(key, descending=True, stable=True).indices[: int(self.evals[r])]
        for c, d in zip(order.cpu().numpy(), cache[order].cpu().numpy()):
            trace.append((int(c), float(d)))
        trace.append(("select", int(self.selected[r])))

    def result(self):
        """Selections (host list of np.int64), their deltas, and per-round evaluation counts."""
        self.check()
        sel = self.selected[: self.rounds].cpu().numpy()
        if (sel < 0).any():
            raise RuntimeError("greedy placement found no candidate (all deltas NaN?)")
        return ([np.int64(s) for s in sel], self.sel_delta[: self.rounds].cpu().numpy(),
                self.evals[: self.rounds].cpu().numpy())


# A singular (PSD, not PD) cov_vv, e.g. an empirical covariance with fewer samples than locations
# (main.py:125-350): the reference's pinv still defines every delta.  The device path then factors
# Sigma + eps I with a relative eps and takes denom = 1 / P_yy - eps (vgposp_greedy_init_ex's
# jitter), so a candidate in the span of the others gets denom ~ 0 -> delta 0 at the 1e-8
# threshold, as with pinv, and every other delta moves by O(eps).
# A factorization can also "succeed" on a singular cov_vv: a zero pivot that rounds to a tiny
# positive value.  L^-1 then turns rounding noise into large deltas where pinv gives 0, so a pivot
# ratio L_ii^2 / sigma_ii below PIVOT_RTOL * n (rounding level) is treated like a failed pivot.
SINGULAR_EPS = (1e-12, 1e-10, 1e-8)
PIVOT_RTOL = 100 * np.finfo(np.float64).eps


def _check_pivots(g, sdiag):
    """After init(): raise CholeskyError if a pivot of Sigma = L L^T is at rounding level.  The
    factored buffer holds M = L^-1, so L_ii^2 / sigma_ii = 1 / (M_ii^2 sigma_ii)."""
    g.check()
    m = torch.diagonal(g.S)
    ratio = 1.0 / (m * m * sdiag)
    i = int(torch.argmin(ratio))
    if not float(ratio[i]) >= PIVOT_RTOL * g.n:
        raise CholeskyError(i + 1)


def _rounds(g, k, lazy, trace):
    for _ in range(k):
        if trace is not None:
            g.step_traced(trace)
        else:
            g.step(lazy)
    return g.result()[0]


def _place(cov_vv, k, lazy, verbose, trace=None):
    if k < 1:
        return []
    if verbose and trace is None:
        trace = []
    tr = None if trace is None else []
    try:
        g = GreedyPlacement(cov_vv, k, copy=True, pad_odd=True)
        sdiag = torch.diagonal(g.S).clone()
        g.init()
        _check_pivots(g, sdiag)
        A = _rounds(g, k, lazy, tr)
    except CholeskyError as err:
        S = linalg.as_device(cov_vv)
        scale = float(torch.mean(torch.diagonal(S)).abs()) or 1.0
        for rel in SINGULAR_EPS:
            try:
                tr = None if trace is None else []
                g = GreedyPlacement(S, k, copy=True, jitter=rel * scale, pad_odd=True).init()
                A = _rounds(g, k, lazy, tr)
                break
            except CholeskyError:
                continue
        else:
            raise err
    if trace is not None:
        trace.extend(tr)
    if verbose:  # the reference's lines, placement_algorithm2.py:205 and :188
        for t in trace:
            if t[0] == "select":
                print("y*=", t[1])
            else:
                print("delta_y=", t[1], "y_st=", t[0])
    return A


def placement_algorithm_2(cov_vv, k, verbose=False, trace=None):
    """Lazy greedy MI placement (placement_algorithm2.py:151-219).  Returns k indices.

    ``verbose=True`` prints the reference's per-evaluation lines (``delta_y= … y_st= …`` for every
    delta evaluated, ``y*= …`` per selection, :205 / :188); ``trace`` (a list) receives the same
    records as ``(y, delta)`` / ``('select', y)`` tuples without printing."""
    return _place(cov_vv, k, True, verbose, trace)


def placement_algorithm_1(cov_vv, k, verbose=False):
    """Full greedy MI placement (placement_algorithm2.py:128-145).  Returns k indices."""
    return _place(cov_vv, k, False, verbose)


def cov_vv_4x4():
    """The reference's fixture (placement_algorithm2.py:473-479)."""
    return np.array([[1.10, 0.31, 0.33, 0.27],
                     [0.31, 1.01, 0.30, 0.27],
                     [0.33, 0.30, 0.97, 0.33],
                     [0.27, 0.27, 0.33, 1.2]])


def dg_create_random_cov(n, rng=None):
    """placement_algorithm2.py:441-444."""
    r = np.random if rng is None else rng
    m = r.uniform(0, 1, n ** 2).reshape(-1, n)
    return np.dot(m, m.T)


def placement_from_points(X, k, kind="eq", amp=1.0, ls=1.0, noise=1e-2, jitter=1e-6, lazy=True):
    """Assemble Sigma = K(X, X) + (noise + jitter) I on device and place k sensors."""
    K = linalg.kernel_matrix(kind, X, None, amp, ls, diag_shift=noise + jitter)[0]
    g = GreedyPlacement(K, k).run(k, lazy=lazy)
    return g.result()[0]

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
                 cache_init=float("inf")):
        S = linalg.as_device(Sigma)
        if S.dim() != 2 or S.shape[0] != S.shape[1]:
            raise ValueError("cov_vv must be a square matrix")
        self.n = int(S.shape[0])
        if not (1 <= kmax <= self.n):
            raise ValueError(f"k must be in [1, {self.n}], got {kmax}")
        self.S = S.clone() if copy else S
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
        self.rounds = 0
        return self

    def cache(self):
        """Device view of the lazy cache (delta_cached) [n] inside the workspace."""
        c = ctypes.c_void_p()
        call("vgposp_greedy_cache", _p(self.ws), self.n, self.kmax, ctypes.byref(c))
        off = c.value - self.ws.data_ptr()
        return self.ws[off:off + 8 * self.n].view(torch.float64)

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
SINGULAR_EPS = (1e-12, 1e-10, 1e-8)


def _place(cov_vv, k, lazy, verbose):
    if k < 1:
        return []
    try:
        g = GreedyPlacement(cov_vv, k, copy=True).run(k, lazy=lazy)
        A, deltas, _ = g.result()
    except CholeskyError as err:
        S = linalg.as_device(cov_vv)
        scale = float(torch.mean(torch.diagonal(S)).abs()) or 1.0
        for rel in SINGULAR_EPS:
            try:
                g = GreedyPlacement(S, k, copy=True, jitter=rel * scale).run(k, lazy=lazy)
                A, deltas, _ = g.result()
                break
            except CholeskyError:
                continue
        else:
            raise err
    if verbose:
        for y, d in zip(A, deltas):
            print("y*=", y, "delta=", d)
    return A


def placement_algorithm_2(cov_vv, k, verbose=False):
    """Lazy greedy MI placement (placement_algorithm2.py:151-219).  Returns k indices."""
    return _place(cov_vv, k, True, verbose)


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

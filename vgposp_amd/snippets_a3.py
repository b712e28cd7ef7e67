"""Placement algorithm 3, the local-kernel greedy, on MI355X: the reference's
``snippets_a3.sparse_placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff)``
(``snippets_a3.py:43-330``).

The greedy of ``sparse_placement_algorithm_2`` (TF constants: jitter 1e-6 on the conditioning
blocks, threshold 1e-7, cache initialised to 1e8) with one change.  Every candidate is scored once
(round 0); after each pick y* only the candidates whose grid indices lie in
``[i_d - cutoff, i_d + cutoff)`` around y* (per axis, clipped) are re-scored.  Everything else keeps
its stale cache value.  The reference returns the set A, the final cache and the per-round cache
snapshots ``delta_cached_iters [N, k]``; so does this.

Device work per round is the dense-exact engine of ``placement_algorithm2`` (the HBM-bound
triangular mat-vec plus O(N) updates) followed by ``vgposp_greedy_select_window``.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call
from .linalg import _p, _stream
from .placement_algorithm2 import GreedyPlacement
from .snippets_a2 import TF_INF, TF_JITTER, TF_SMALL, SparseSet


def _cover(COVER_spatial, N):
    I = [int(c) for c in COVER_spatial[:3]]
    if N != I[0] * I[1] * I[2]:
        raise ValueError(f"assertion failed: N = {N} != prod(COVER_spatial) = {I[0] * I[1] * I[2]}")
    return I


class WindowGreedy(GreedyPlacement):
    """Device-resident algorithm 3 (round-by-round, like GreedyPlacement)."""

    def __init__(self, Sigma, kmax, COVER_spatial, cutoff, copy=False, jitter=TF_JITTER,
                 threshold=TF_SMALL, cache_init=TF_INF):
        super().__init__(Sigma, kmax, copy=copy, jitter=jitter, threshold=threshold,
                         cache_init=cache_init)
        self.I = _cover(COVER_spatial, self.n)
        self.cutoff = int(cutoff)
        if self.cutoff < 0:
            raise ValueError("cutoff must be >= 0")

    def step(self, lazy=None):
        if self.rounds >= self.kmax:
            raise RuntimeError("all k sensors already placed")
        call("vgposp_greedy_update", _p(self.S), self.n, self.S.stride(0), self.kmax, self.rounds,
             0, self.n, _p(self.selected), _p(self.ws), self.ws.numel(), _stream())
        call("vgposp_greedy_select_window", self.n, self.kmax, self.rounds, *self.I, self.cutoff,
             0, self.n, _p(self.selected), _p(self.sel_delta), _p(self.evals), _p(self.ws),
             self.ws.numel(), _stream())
        self.rounds += 1


def sparse_placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff):
    """-> (A as a SparseSet, final delta_cached [N, 1], delta_cached_iters [N, k]) like
    snippets_a3.py:330; ``A.order`` is not part of the reference (its A is a set) — the ordered
    picks are returned by ``placement_algorithm_3``."""
    A, cache, dci = _run(cov_vv, k, COVER_spatial, cutoff)
    vals = np.sort(np.asarray(A, dtype=np.int64))
    Aset = SparseSet(np.stack([vals, np.zeros_like(vals)], axis=1), vals, (len(cache), 1))
    return Aset, cache.reshape(-1, 1), dci


def placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff):
    """The ordered picks of algorithm 3 (list of np.int64)."""
    return _run(cov_vv, k, COVER_spatial, cutoff)[0]


def _run(cov_vv, k, COVER_spatial, cutoff):
    N = int(cov_vv.shape[0])
    _cover(COVER_spatial, N)
    g = WindowGreedy(cov_vv, k, COVER_spatial, cutoff, copy=True)
    g.init()
    cache = g.cache()
    dci = torch.empty((k, N), dtype=torch.float64, device=cache.device)
    for r in range(k):
        g.step()
        dci[r].copy_(cache)  # round 0: every score; round r: after the refresh around pick r-1
    A, _, _ = g.result()
    return A, cache.cpu().numpy(), dci.t().cpu().numpy()


__all__ = ["sparse_placement_algorithm_3", "placement_algorithm_3", "WindowGreedy"]

"""The TF-graph greedy placement ``snippets_a2.sparse_placement_algorithm_2`` on MI355X
(reference ``snippets_a2.py:679-822``, with ``tf_nominator`` :138-213, ``tf_denominator`` :215-217,
``if_denom_is_near_zero`` :467-487 and ``placement_algorithm2.sparse_argmax_cache_linear`` :24-50).

It is the lazy greedy of ``placement_algorithm2.placement_algorithm_2`` with three different
constants, all handled inside libvgposp (``vgposp_greedy_init_ex``):

* ``1e-6`` added to the diagonal of Sigma_AA and Sigma_AbarAbar before ``pinv`` (:161-163);
* ``|nom|`` or ``|denom| < 1e-7`` -> delta = 0 (:480);
* the cache starts at ``INF = 1e8`` (:690);

plus two outputs: the per-round cache snapshot ``delta_cached_iters[N, k]`` (:778, taken before
the selected entry's cache is zeroed at :796) and the ordered ``A_selection_and_delta[k, 2]``
(:767-768).  ``A`` itself is a set in the reference (a ``tf.SparseTensor`` built with
``tf.sets.union``, so sorted and order-free); it is returned here as a ``SparseSet`` with the same
``indices / values / dense_shape`` fields.
"""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch

from .placement_algorithm2 import GreedyPlacement

TF_JITTER = 1e-6   # snippets_a2.py:161-163
TF_SMALL = 1e-7    # snippets_a2.py:480
TF_INF = 1e8       # snippets_a2.py:690


class SparseSet(NamedTuple):
    """Host mirror of the reference's tf.SparseTensor set A (dense_shape [N, 1])."""
    indices: np.ndarray      # [len, 2] int64: (value, 0)
    values: np.ndarray       # [len] int64, ascending
    dense_shape: tuple


def sparse_placement_algorithm_2(cov_vv, k, COVER_spatial, jitter=TF_JITTER, threshold=TF_SMALL,
                                 cache_init=TF_INF):
    """Returns ``(A, len_A, delta_cached_iters [N, k] f64, A_selection_and_delta [k, 2] f64)``
    like snippets_a2.py:822.  ``cov_vv``: [N, N] float64 (numpy or device tensor), N must equal
    COVER_spatial[0] * COVER_spatial[1] * COVER_spatial[2] (the tf.Assert at :692)."""
    N = int(cov_vv.shape[0])
    cover = int(np.prod([int(c) for c in COVER_spatial[:3]]))
    if N != cover:
        raise ValueError(f"assertion failed: N = {N} != prod(COVER_spatial) = {cover}")
    g = GreedyPlacement(cov_vv, k, copy=True, jitter=jitter, threshold=threshold,
                        cache_init=cache_init, pad_odd=True)
    g.init()
    cache = g.cache()
    dci = torch.empty((k, N), dtype=torch.float64, device=cache.device)
    for r in range(k):
        g.step(lazy=True)
        dci[r].copy_(cache)                                   # :778 (before the zeroing)
        cache.index_fill_(0, g.selected[r:r + 1], 0.0)        # :796 delta_cached[y_st] = 0
    A, deltas, _ = g.result()
    sel = np.stack([np.asarray(A, dtype=np.float64), deltas], axis=1)
    vals = np.sort(np.asarray(A, dtype=np.int64))
    Aset = SparseSet(np.stack([vals, np.zeros_like(vals)], axis=1), vals, (N, 1))
    return Aset, len(vals), dci.t().cpu().numpy(), sel


__all__ = ["sparse_placement_algorithm_2", "SparseSet", "TF_JITTER", "TF_SMALL", "TF_INF"]

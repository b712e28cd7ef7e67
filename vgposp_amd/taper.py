"""The beta-decay taper of config C4 and the TF variant's constants (shared by the exact C4 path,
``sparse_placement``).

The reference's scaling answer is its algorithm 3 (``snippets_a3.sparse_placement_algorithm_3``,
``snippets_a3.py:43-364``) on the beta-decay local kernel of
``main_architecture_2_sampledistribution.py:355-421``: covariances are multiplied by
``exp(-(beta d)^2 / (2 pi))`` of the index distance d and zeroed where that decay is < 0.01
(``decay_fn``, ``:390-393``; ``BETA_val = 4`` there, with ``cutoff = 3``, ``:973``).  That is the
filter the reference intends, not the one its code computes: the ``tf.cond`` at ``:416-420`` has
its branches inverted (``zero_ij`` where the decay is >= 0.01, ``calc_ij`` — multiplying by a decay
of 0 — elsewhere), so as written it leaves the ``tf.zeros`` ``cov_vv`` (``:337``) all zero.
DESIGN.md §3 records the divergence.  ``taper_support`` is the non-zero
pattern of one row of that covariance, from which the C4 kernels build Sigma's entries on the fly.
"""
from __future__ import annotations

import numpy as np

TAPER_FLOOR = 0.01   # main_architecture_2_sampledistribution.py:392 (decay_fn's floor)
TF_JITTER = 1e-6     # snippets_a2.py:161-163 (diagonal of the conditioning block)
TF_SMALL = 1e-7      # snippets_a2.py:480 (|nom| or |denom| below -> delta = 0)


def decay(beta, d2):
    """The reference's decay_fn (main_architecture_2_sampledistribution.py:375-393) of integer
    squared index distances, with its 0.01 floor."""
    delta = np.abs(np.sqrt(np.asarray(d2, dtype=np.float64)))
    g = np.exp(-np.square(float(beta) * delta) / (2 * np.pi))
    return np.where(g < TAPER_FLOOR, 0.0, g)


def taper_support(beta):
    """(offsets int32 [m-1, 3] in C order, tau[d2]) — the non-zero pattern of the tapered
    covariance around a grid point, without the point itself."""
    r = 0
    while decay(beta, (r + 1) ** 2) > 0:
        r += 1
    ax = np.arange(-r, r + 1)
    o = np.stack(np.meshgrid(ax, ax, ax, indexing="ij"), -1).reshape(-1, 3)
    d2 = (o ** 2).sum(1)
    offs = o[(decay(beta, d2) > 0) & (d2 > 0)].astype(np.int32)
    tau = decay(beta, np.arange(12 * r * r + 1))
    if len(offs) + 1 > 64:
        raise ValueError(f"beta = {beta}: taper support of {len(offs) + 1} points > 64")
    return offs, tau


__all__ = ["TAPER_FLOOR", "TF_JITTER", "TF_SMALL", "decay", "taper_support"]

"""An APPROXIMATION of config C4 (the epsilon-local form): greedy MI placement on grids too large
for a dense cov_vv (128^3 = 2,097,152 candidates, k = 50), candidates sharded over the GPUs of one
node.  Its deltas condition only on each candidate's taper support, not on the full sets the
reference's algorithm 3 uses, and its picks diverge from that algorithm within a few rounds
(round-2 verdict).  The exact C4 path is ``sparse_placement.tapered_placement_algorithm_3``;
this module is kept as the documented approximation (and for the taper tables the exact path
shares: ``taper_support``, ``decay``, the TF constants).

The reference's scaling answer is its algorithm 3 (``snippets_a3.sparse_placement_algorithm_3``,
``snippets_a3.py:43-364``) on the beta-decay local kernel of
``main_architecture_2_sampledistribution.py:355-421``: covariances are multiplied by
``exp(-(beta d)^2 / (2 pi))`` of the index distance d and zeroed where that decay is < 0.01
(``BETA_val = 4`` there, with ``cutoff = 3``, ``:973``).  Here each delta conditions only on the
taper support N(y) of its candidate — the ``Hhat_epsilon(y | V \\ y)`` that ``snippets_a3.py:63``
and ``:182-186`` name — so nothing N x N is ever formed and a pick y* changes only the deltas
inside its window.  The cache policy is the reference's: score everything once, then per round
arg-max (lowest index on ties), zero the pick, re-score the index window ``[i_d - cutoff,
i_d + cutoff)`` around it.

Multi-GPU: every rank holds the grid points X (50 MB at 128^3) and the selected
mask, and owns a slab of whole i0-planes of candidates with their cache.  Per round the only
exchange is the arg-max: each rank reduces its slab to one 16-byte (delta, index) key, the keys
are all-gathered (RCCL over xGMI with the ``nccl`` backend) and every rank applies the same pick.
The window re-score touches at most the two slabs the window straddles.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ._lib import KERNEL_KINDS, call, query
from .linalg import _p, _stream

TAPER_FLOOR = 0.01   # main_architecture_2_sampledistribution.py:392, :417
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


def plane_slabs(shape, world):
    """Contiguous candidate slabs [c0, c1) of whole i0-planes per rank."""
    I0, I1, I2 = (int(s) for s in shape)
    e = [round(I0 * r / world) for r in range(world + 1)]
    return [(e[r] * I1 * I2, e[r + 1] * I1 * I2) for r in range(world)]


class HipLocalBackend:
    """Device state of one rank: X, the taper tables, the selected mask, this slab's cache and the
    arg-max keys.  Every call only enqueues work on the current stream."""

    def __init__(self, X, shape, kmax, cutoff, beta, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
                 jitter=TF_JITTER, threshold=TF_SMALL, c0=0, c1=None, device=None):
        self.shape = tuple(int(s) for s in shape)
        I0, I1, I2 = self.shape
        self.n = I0 * I1 * I2
        dev = torch.device(device) if device is not None else torch.device("cuda")
        X = torch.as_tensor(X, dtype=torch.float64, device=dev)
        if X.shape != (self.n, 3):
            raise ValueError(f"X must be [{self.n}, 3] grid points in C order, got {tuple(X.shape)}")
        self.X = X.contiguous()
        offs, tau = taper_support(beta)
        self.m = len(offs) + 1
        self.offs = torch.as_tensor(offs.reshape(-1) if len(offs) else np.zeros(3, np.int32),
                                    device=dev)
        self.tau = torch.as_tensor(tau, device=dev)
        self.kind = KERNEL_KINDS[kind]
        self.amp, self.ls, self.shift = float(amp), float(ls), float(diag_shift)
        self.jitter, self.thr = float(jitter), float(threshold)
        self.kmax, self.cutoff = int(kmax), int(cutoff)
        self.c0 = int(c0)
        self.c1 = self.n if c1 is None else int(c1)
        nloc = self.c1 - self.c0
        self.selected = torch.zeros(self.n, dtype=torch.uint8, device=dev)
        self.picks = torch.full((self.kmax,), -1, dtype=torch.int64, device=dev)
        self.pick_delta = torch.zeros(self.kmax, dtype=torch.float64, device=dev)
        self.cache = torch.zeros(max(nloc, 1), dtype=torch.float64, device=dev)
        self.info = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ws = torch.empty(query("vgposp_local_workspace_bytes", nloc), dtype=torch.uint8,
                              device=dev)
        self.key = torch.zeros(2, dtype=torch.int64, device=dev)

    def reset(self):
        self.selected.zero_()
        self.picks.fill_(-1)
        self.info.zero_()

    def _args(self):
        return (self.kind, _p(self.X), *self.shape, self.amp, self.ls, self.shift, self.jitter,
                self.thr, _p(self.offs), self.m, _p(self.tau), self.tau.numel(),
                _p(self.selected), self.c0, self.c1, self.cutoff, _p(self.cache), _p(self.info),
                _p(self.ws), self.ws.numel())

    def score_all(self):
        """Round 0: every candidate of the slab (snippets_a3.py:77-124)."""
        call("vgposp_local_score", *self._args(), _stream())

    def argmax(self, rnd):
        """This slab's (delta, index) key after round rnd - 1's pick and window."""
        call("vgposp_local_select", *self._args(), _p(self.picks), rnd, _p(self.key), _stream())
        return self.key

    def pick(self, keys, nkeys, rnd, window=True):
        """Apply the best of the gathered keys as pick rnd, then re-score its window."""
        call("vgposp_local_pick", *self._args(), _p(keys), nkeys, rnd, int(window),
             _p(self.picks), _p(self.pick_delta), _stream())

    def run_all(self, k):
        """Single rank: the full pass and all k rounds in two launches (m <= 16)."""
        call("vgposp_local_run", *self._args(), k, _p(self.picks), _p(self.pick_delta),
             _p(self.key), _stream())

    def local_cache(self):
        return self.cache[: self.c1 - self.c0]

    def check(self):
        if int(self.info.item()):
            raise np.linalg.LinAlgError("a local conditioning block was not positive definite "
                                        "(taper / jitter too small for this kernel)")


class LocalGreedyPlacement:
    """Algorithm 3 with local deltas over the ranks of ``group`` (or one GPU).  ``run`` returns
    the picks in selection order (identical on every rank)."""

    def __init__(self, backend, group=None):
        self.b = backend
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        dev = backend.key.device
        self.staging = (self.world > 1 and dist.get_backend(group) == "gloo"
                        and dev.type != "cpu")
        cdev = torch.device("cpu") if self.staging else dev
        self.keys = torch.zeros(2 * self.world, dtype=torch.int64, device=dev)
        self._send = torch.zeros(2, dtype=torch.int64, device=cdev)
        self._recv = torch.zeros(2 * self.world, dtype=torch.int64, device=cdev)

    def _gather_keys(self, key):
        if self.staging:
            self._send.copy_(key)
            dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
            self.keys.copy_(self._recv)
        else:
            dist.all_gather_into_tensor(self.keys, key, group=self.group)

    def round(self, rnd, last):
        b = self.b
        key = b.argmax(rnd)
        if self.world == 1:
            b.pick(key, 1, rnd, window=not last)
        else:
            self._gather_keys(key)
            b.pick(self.keys, self.world, rnd, window=not last)

    def run(self, k, snapshots=None):
        """snippets_a3.py:43-364.  ``snapshots`` (list) receives a copy of this rank's cache slab
        after the full pass and after every window re-score (delta_cached_iters columns)."""
        b = self.b
        if k > b.kmax:
            raise ValueError(f"k = {k} > kmax = {b.kmax}")
        b.reset()
        if self.world == 1 and snapshots is None and hasattr(b, "run_all"):
            b.run_all(k)
            return b.picks[:k]
        b.score_all()
        if snapshots is not None:
            snapshots.append(b.local_cache().clone())
        for i in range(k):
            self.round(i, last=(i == k - 1))
            if snapshots is not None and i < k - 1:
                snapshots.append(b.local_cache().clone())
        return b.picks[:k]


def local_placement_algorithm_3(X, k, COVER_spatial, cutoff, beta=4.0, kernel="eq", amp=1.0,
                                ls=1.0, diag_shift=0.0, group=None, snapshots=False):
    """snippets_a3.sparse_placement_algorithm_3 for a grid given by its points X (C order, the
    reference's COVER_spatial = (I0, I1, I2) layout) instead of a dense cov_vv.
    -> (picks as a list of np.int64 in selection order, the pick deltas, delta_cached_iters
    [N_slab, k] of this rank's slab or None)."""
    shape = tuple(int(c) for c in COVER_spatial[:3])
    N = shape[0] * shape[1] * shape[2]
    if len(X) != N:                                        # snippets_a3.py:51 tf.Assert
        raise ValueError(f"assertion failed: N = {len(X)} != prod(COVER_spatial) = {N}")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    c0, c1 = plane_slabs(shape, world)[rank]
    b = HipLocalBackend(X, shape, k, cutoff, beta, kernel, amp, ls, diag_shift, c0=c0, c1=c1)
    snaps = [] if snapshots else None
    picks = LocalGreedyPlacement(b, group).run(k, snaps).cpu().numpy()
    b.check()
    dci = torch.stack(snaps, 1).cpu().numpy() if snapshots else None
    return [np.int64(a) for a in picks], b.pick_delta[:k].cpu().numpy(), dci


__all__ = ["local_placement_algorithm_3", "LocalGreedyPlacement", "HipLocalBackend",
           "taper_support", "plane_slabs", "decay"]

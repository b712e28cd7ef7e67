"""Cholesky of ONE covariance over R ranks (one process per GPU) that each hold it whole.

The candidate-sharded placement (``sharded_placement.py``) needs the lower factor L
of Sigma on every rank before each rank forms its slab's columns of L^-1.  The factorization is the
O(N^3) step behind the reference's pinv calls (placement_algorithm2.py:399-413); replicated, it
bounds the speed-up of one 65k problem on 8 GPUs at ~2x.  Here the ranks split it:

* the host walks ``vgposp_potrf_lower``'s own recursion (split points from ``vgposp_potrf_split``),
  so every diagonal block, leaf inverse and 512-block inverse is the single-GPU one and lands at
  its global column of the potrf workspace (where ``vgposp_greedy_finish_slab`` reads them);
* a node smaller than ``dist_min`` (or of at most 512 columns, whose inverse the recursion forms
  as a block) is factored whole on every rank (``vgposp_potrf_block``: the latency-bound chain of
  leaves, ~2 % of the flops);
* a larger node (col0, nsub), split at n1, n2 = nsub - n1, after its top-left child:
    1. panel TRSM L21 = A21 L11^-T: rank r solves an even share of L21's n2 rows
       (``vgposp_potrf_panel``); the shares are all-gathered (n2 x n1 doubles in total);
    2. SYRK A22 -= L21 L21^T (lower): rank r updates a band of A22's rows balanced by lower-triangle
       area (``vgposp_potrf_trailing``); the bands' lower trapezoids are all-gathered
       (n2 (n2 + 1) / 2 doubles in total);
  then its bottom-right child.

Every rank ends with the same L (the upper triangle of the buffer, Sigma, is never written).  The
all-gathers run on RCCL over device buffers ("nccl" backend), or through host staging on gloo (the
CPU tests and the 2-ranks-on-one-GPU test).  At N = 65,536 and R = 8 they move ~26 GB in total
(each rank receives 7/8 of it); the flops per rank drop ~7x.

Overlap: the trailing update of a node is done in two parts.  Rows [0, h) of A22 (h = the split of
the bottom-right child, the rows its top-left recursion factors first) are updated and
all-gathered before that recursion starts; rows [h, n2) are updated next and their all-gather is
issued asynchronously and only unpacked when an operation reads those rows (the child's panel), so
it runs beside the child's whole top-left recursion.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.distributed as dist

from ._lib import call, query
from .linalg import _p, _stream

DIST_MIN = 4096   # nodes at least this large are split over the ranks
BLOCK_INV = 512   # nodes up to this size are factored whole: the recursion inverts them as blocks
ALIGN = 128       # share boundaries on GEMM-tile rows


def even_rows(n, world, align=ALIGN):
    """[a, b) row shares of n rows, equal up to ``align``."""
    edges = [0]
    for r in range(1, world):
        e = int(round(n * r / world / align)) * align
        edges.append(min(max(e, edges[-1]), n))
    edges.append(n)
    return [(edges[r], edges[r + 1]) for r in range(world)]


def lower_bands(n, world, align=ALIGN, start=0):
    """[a, b) row bands of rows [start, n) of an n x n lower triangle with equal area (row i has
    i + 1 entries): edge r at sqrt(start^2 + (n^2 - start^2) r / world)."""
    edges = [start]
    for r in range(1, world):
        e = int(round(math.sqrt(start * start + (n * n - start * start) * r / world) / align)) * align
        edges.append(min(max(e, edges[-1]), n))
    edges.append(n)
    return [(edges[r], edges[r + 1]) for r in range(world)]


class HipCholeskyOps:
    """The device pieces (libvgposp) on an [n, n] fp64 tensor with a potrf workspace for n."""

    def __init__(self, A, fws_ptr, fws_bytes, info):
        self.A = A
        self.n = int(A.shape[0])
        self.lda = int(A.stride(0))
        self.fws = fws_ptr
        self.fws_bytes = int(fws_bytes)
        self.info = info
        self.device = A.device

    def split(self, n):
        return query("vgposp_potrf_split", n)

    def block(self, col0, nb):
        call("vgposp_potrf_block", _p(self.A), self.n, self.lda, col0, nb, _p(self.info),
             self.fws, self.fws_bytes, _stream())

    def panel(self, col0, nsub, r0, r1):
        call("vgposp_potrf_panel", _p(self.A), self.n, self.lda, col0, nsub, r0, r1, self.fws,
             self.fws_bytes, _stream())

    def trailing(self, col0, nsub, b0, b1):
        call("vgposp_potrf_trailing", _p(self.A), self.n, self.lda, col0, nsub, b0, b1, self.fws,
             self.fws_bytes, _stream())

    def pack_elems(self, r0, r1, c0, c1, lower):
        return query("vgposp_pack_elems", r0, r1, c0, c1, int(lower))

    def pack(self, r0, r1, c0, c1, lower, buf, unpack):
        call("vgposp_pack_rows", _p(self.A), self.lda, r0, r1, c0, c1, int(lower), _p(buf),
             int(unpack), _stream())


class DistCholesky:
    """Factor ``ops``'s matrix (lower, in place) with the work of every large recursion node split
    over the ranks of ``group``."""

    def __init__(self, ops, group=None, dist_min=DIST_MIN):
        self.ops = ops
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.dist_min = int(dist_min)
        dev = ops.device
        self.staging = (self.world > 1 and dist.get_backend(group) == "gloo"
                        and dev.type != "cpu")
        self._bufs = {}
        self.exchanged = 0  # doubles all-gathered (diagnostic)

    def factor(self):
        self._pending = []
        self._rec(0, self.ops.n)
        self._flush(0, self.ops.n)

    def _splits(self, nsub):
        return self.world > 1 and nsub >= self.dist_min and nsub > BLOCK_INV

    def _rec(self, col0, nsub, depth=0):
        ops = self.ops
        if not self._splits(nsub):
            self._flush(col0, col0 + nsub)
            ops.block(col0, nsub)
            return
        n1 = ops.split(nsub)
        n2 = nsub - n1
        base = col0 + n1
        self._rec(col0, n1, depth + 1)
        self._flush(col0, col0 + nsub)     # the panel reads rows [col0, col0 + nsub)
        shares = even_rows(n2, self.world)
        ops.panel(col0, nsub, *shares[self.rank])
        self._exchange([(base + a, base + b, col0, base, 0) for a, b in shares])
        # trailing update: first the rows the bottom-right child factors first, then the rest
        # with a deferred all-gather
        h = ops.split(n2) if self._splits(n2) else n2
        bands = lower_bands(h, self.world)
        ops.trailing(col0, nsub, *bands[self.rank])
        self._exchange([(base + a, base + b, base, base + b, 1) for a, b in bands])
        if h < n2:
            bands = lower_bands(n2, self.world, start=h)
            ops.trailing(col0, nsub, *bands[self.rank])
            self._exchange([(base + a, base + b, base, base + b, 1) for a, b in bands],
                           defer=(base + h, base + n2), depth=depth)
        self._rec(base, n2, depth + 1)

    def _buf(self, key, numel, device):
        b = self._bufs.get(key)
        if b is None or b.numel() < numel:
            b = torch.empty(numel, dtype=torch.float64, device=device)
            self._bufs[key] = b
        return b[:numel]

    def _exchange(self, pieces, defer=None, depth=0):
        """All-gather every rank's piece (r0, r1, c0, c1, lower) of the matrix.  ``defer`` = the
        row range the pieces cover: the all-gather is issued asynchronously and the received
        pieces are unpacked by the first _flush that touches those rows.

        A deferred exchange keeps its buffers until that unpack, i.e. through the whole top-left
        recursion of the node's bottom-right child (that is the overlap); at most one is pending
        per recursion depth (a node's is unpacked by its bottom-right child's first flush, before
        the child issues its own), so each depth reuses one buffer pair.  Peak device memory per
        rank: the synchronous pair plus one deferred pair per depth, about 2 (1 + 1/R) x the
        top node's deferred rows (at the 65k top node, rows [h, n2) of A22: ~3 GB per buffer)."""
        ops = self.ops
        sizes = [ops.pack_elems(*p) for p in pieces]
        S = max(sizes)
        if S == 0:
            return
        if defer is None:
            send = self._buf("send", S, ops.device)
            recv = self._buf("recv", self.world * S, ops.device)
        else:  # this depth's pair: it lives until the unpack
            send = self._buf(("dsend", depth), S, ops.device)
            recv = self._buf(("drecv", depth), self.world * S, ops.device)
        if sizes[self.rank]:
            ops.pack(*pieces[self.rank], send, False)
        host = None
        if self.staging:
            hs = send.cpu()
            host = torch.empty(self.world * S, dtype=torch.float64)
            work = dist.all_gather_into_tensor(host, hs, group=self.group,
                                               async_op=defer is not None)
        else:
            work = dist.all_gather_into_tensor(recv, send, group=self.group,
                                               async_op=defer is not None)
        entry = (defer, work, send, recv, host, pieces, sizes, S)
        self.exchanged += sum(sizes)
        if defer is None:
            self._unpack(entry)
        else:
            self._pending.append(entry)

    def _unpack(self, entry):
        _, work, _, recv, host, pieces, sizes, S = entry
        if work is not None:
            work.wait()
        if host is not None:
            recv.copy_(host)
        for r, p in enumerate(pieces):
            if r != self.rank and sizes[r]:
                self.ops.pack(*p, recv[r * S:r * S + sizes[r]], True)

    def _flush(self, r0, r1):
        """Unpack (in issue order) every deferred all-gather whose rows meet [r0, r1)."""
        keep = []
        for e in getattr(self, "_pending", []):
            a, b = e[0]
            if a < r1 and r0 < b:
                self._unpack(e)
            else:
                keep.append(e)
        self._pending = keep


def greedy_cholesky_ops(g):
    """HipCholeskyOps over a GreedyPlacement's Sigma and the potrf workspace inside its greedy
    workspace (so vgposp_greedy_finish_slab finds the leaf / block inverses)."""
    fws, fbytes = ctypes.c_void_p(), ctypes.c_size_t()
    call("vgposp_greedy_fact_ws", _p(g.ws), g.n, g.kmax, ctypes.byref(fws), ctypes.byref(fbytes))
    return HipCholeskyOps(g.S, fws.value, fbytes.value, g.info)

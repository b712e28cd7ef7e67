"""Candidate-sharded greedy MI placement across GPUs, one process per GPU.

The candidate set V is cut into R contiguous slabs.  With ``partition_inverse=True`` (what
bench.py runs) the ranks factor the covariance TOGETHER (``dist_cholesky.DistCholesky``: every large
node of the recursive Cholesky has its panel TRSM and trailing SYRK split over the ranks, the
shares all-gathered; ``dist_factor=False`` replicates the factorization instead) and each rank then
forms L^-1 only in its own slab's columns (vgposp_greedy_finish_slab: about 1/R of the inverse's
flops, slabs balanced by that work, 128-aligned).  With ``partition_inverse=False`` the fused
Cholesky + full inverse is replicated and the slabs balance the triangular mat-vec (column c of
L^-1 has n - c stored rows).  Per round:

  0. (partitioned inverse) the owner of the last pick's column of L^-1 writes it, the others zeros,
     and ONE sum-all-reduce of that column (N x 8 bytes) gives every rank the mat-vec's vector;
  1. ``vgposp_greedy_update`` on its slab: W / V rank-1 rows, nom, P_yy and fresh deltas for the
     slab's candidates only (the HBM-bound mat-vec reads only the slab's columns of L^-1);
  2. ONE all-gather of the delta slabs (N x 8 bytes) so every rank holds all fresh deltas;
  3. ``vgposp_greedy_select`` over ALL candidates — the reference's lazy-cache decisions
     (placement_algorithm2.py:173-214) are re-run identically on every rank, so every rank picks
     the same y* with no further exchange (the arg-max never needs a MAX-LOC collective);
  4. ONE sum-all-reduce of the pivot row of y* (2 + 2 kmax doubles) that only its owner wrote.

Nothing else crosses devices, and the selections are bit-identical to the single-GPU path (the
per-column sums do not depend on the partition).  Collectives run on RCCL ("nccl" backend) over
device tensors, or on gloo through host staging (the CPU tests).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ._lib import call
from .linalg import _p, _stream


def slab_bounds(n, world, balance=True):
    """Contiguous candidate slabs [c0, c1) per rank; balance=True equalises sum_c (n - c)."""
    if not balance:
        edges = [round(n * r / world) for r in range(world + 1)]
    else:
        total = n * (n + 1) / 2.0
        edges = [0]
        for r in range(1, world):
            # solve c n - c^2/2 + c/2 = r/world * total for c
            target = total * r / world
            b = n + 0.5
            c = b - np.sqrt(max(b * b - 2.0 * target, 0.0))
            edges.append(int(min(max(round(c), edges[-1]), n)))
        edges.append(n)
    return [(edges[r], edges[r + 1]) for r in range(world)]


def inverse_slabs(n, world, align=128):
    """Contiguous slabs whose columns of L^-1 cost the same to form: the work of columns [0, c) is
    about n^3 - (n - c)^3, so rank r's boundary is n (1 - (1 - r / world)^(1/3)), rounded to a
    multiple of ``align`` (vgposp_greedy_init_slab's block boundary)."""
    edges = [0]
    for r in range(1, world):
        c = n * (1.0 - (1.0 - r / world) ** (1.0 / 3.0))
        c = int(round(c / align)) * align
        edges.append(int(min(max(c, edges[-1]), n)))
    edges.append(n)
    return [(edges[r], edges[r + 1]) for r in range(world)]


class HipGreedyBackend:
    """The per-rank device state: a GreedyPlacement plus tensor views of its delta / pivot."""

    def __init__(self, Sigma, kmax, copy=False, jitter=0.0):
        from .placement_algorithm2 import GreedyPlacement
        self._src = Sigma if copy else None
        self.g = GreedyPlacement(Sigma, kmax, copy=copy, jitter=jitter)
        # diag(Sigma) for the pivot-ratio check, taken right before each factorization
        # (snapshot_diag): Sigma may still be unassembled here (bench.py fills it per step)
        self.sdiag = None
        self.n = self.g.n
        self.kmax = self.g.kmax
        d, p, plen = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        call("vgposp_greedy_buffers", _p(self.g.ws), self.n, self.kmax, ctypes.byref(d),
             ctypes.byref(p), ctypes.byref(plen))
        base = self.g.ws.data_ptr()
        self._delta = self.g.ws[d.value - base:d.value - base + 8 * self.n].view(torch.float64)
        self._piv = self.g.ws[p.value - base:p.value - base + 8 * plen.value].view(torch.float64)

        x = ctypes.c_void_p()
        call("vgposp_greedy_xcol", _p(self.g.ws), self.n, self.kmax, ctypes.byref(x))
        self._xcol = self.g.ws[x.value - base:x.value - base + 8 * self.n].view(torch.float64)
        self._tmp = None

    def snapshot_diag(self):
        """diag(Sigma) as the factorization will see it (a device copy, no host sync)."""
        d = torch.diagonal(self.g.S)
        if self.sdiag is None or self.sdiag.shape != d.shape:
            self.sdiag = d.clone()
        else:
            self.sdiag.copy_(d)

    def init(self):
        self.g.init()

    # singular cov_vv (placement_algorithm2._place's rules, decided identically on every rank:
    # each holds the same factor)
    def factor_ok(self, c0, c1, partitioned, check_pivots):
        """No failed pivot, and (check_pivots) no pivot ratio L_ii^2 / sigma_ii at rounding level.
        The factored buffer holds L^-1 in the columns this rank inverted (all of them unless
        partitioned) and L elsewhere."""
        from .placement_algorithm2 import PIVOT_RTOL
        g = self.g
        ok = g.info.reshape(-1)[0] == 0
        if check_pivots:
            if self.sdiag is None:
                raise RuntimeError("factor_ok(check_pivots=True) needs snapshot_diag() before "
                                   "the factorization")
            d = torch.diagonal(g.S)
            inv = torch.ones_like(d, dtype=torch.bool)
            if partitioned:
                inv.zero_()
                inv[c0:c1] = True
            lii = torch.where(inv, 1.0 / d, d)
            ok = ok & (torch.min(lii * lii / self.sdiag) >= PIVOT_RTOL * g.n)
        return bool(ok.item())  # the status and the pivot ratio in ONE host read

    def diag_scale(self):
        return float(torch.mean(self.sdiag).abs()) or 1.0

    def rejitter(self, eps):
        """Start over on Sigma + eps I with denom = 1 / P_yy - eps (vgposp_greedy_init_ex)."""
        if self._src is None:
            raise RuntimeError("the jitter retry needs the backend to own a copy of Sigma")
        self.__init__(self._src, self.kmax, copy=True, jitter=eps)

    def init_slab(self, c0, c1):
        """Factor Sigma, form L^-1 only in columns [c0, c1) (vgposp_greedy_init_slab)."""
        from ._lib import query
        g = self.g
        need = query("vgposp_greedy_slab_tmp_bytes", g.n, c0, c1)
        if self._tmp is None or self._tmp.numel() < need:
            self._tmp = torch.empty(max(need, 8), dtype=torch.uint8, device=g.S.device)
        call("vgposp_greedy_init_slab", _p(g.S), g.n, g.S.stride(0), g.kmax, *g.params, c0, c1,
             _p(self._tmp), self._tmp.numel(), _p(g.info), _p(g.ws), g.ws.numel(), _stream())
        g.rounds = 0

    def prepare(self):
        """vgposp_greedy_prepare: the init kernel only (the caller factors Sigma)."""
        g = self.g
        call("vgposp_greedy_prepare", _p(g.S), g.n, g.S.stride(0), g.kmax, *g.params, _p(g.info),
             _p(g.ws), g.ws.numel(), _stream())
        g.rounds = 0

    def chol_ops(self):
        from .dist_cholesky import greedy_cholesky_ops
        return greedy_cholesky_ops(self.g)

    def finish_slab(self, c0, c1):
        """After the factorization: L^-1 in columns [c0, c1) and their column norms."""
        from ._lib import query
        g = self.g
        need = query("vgposp_greedy_slab_tmp_bytes", g.n, c0, c1)
        if self._tmp is None or self._tmp.numel() < need:
            self._tmp = torch.empty(max(need, 8), dtype=torch.uint8, device=g.S.device)
        call("vgposp_greedy_finish_slab", _p(g.S), g.n, g.S.stride(0), g.kmax, c0, c1,
             _p(self._tmp), self._tmp.numel(), _p(g.ws), g.ws.numel(), _stream())

    def extract(self, rnd, own0, own1):
        g = self.g
        call("vgposp_greedy_extract", _p(g.S), g.n, g.S.stride(0), g.kmax, rnd, own0, own1,
             _p(g.selected), _p(g.ws), g.ws.numel(), _stream())

    def xcol(self):
        return self._xcol

    def update(self, rnd, c0, c1, extract=True):
        g = self.g
        call("vgposp_greedy_update_ex", _p(g.S), g.n, g.S.stride(0), g.kmax, rnd, c0, c1,
             _p(g.selected), int(extract), _p(g.ws), g.ws.numel(), _stream())

    def select(self, rnd, lazy, c0, c1):
        g = self.g
        call("vgposp_greedy_select", g.n, g.kmax, rnd, int(lazy), c0, c1, _p(g.selected),
             _p(g.sel_delta), _p(g.evals), _p(g.ws), g.ws.numel(), _stream())
        g.rounds = rnd + 1

    def delta(self):
        return self._delta

    def piv(self):
        return self._piv

    def result(self):
        return self.g.result()


class ShardedGreedyPlacement:
    def __init__(self, backend, group=None, balance=True, partition_inverse=False, align=128,
                 dist_factor=True, dist_min=None):
        self.b = backend
        self.dist_factor = bool(dist_factor)
        self.dist_min = dist_min
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.partition = bool(partition_inverse)
        self.slabs = (inverse_slabs(backend.n, self.world, align) if self.partition else
                      slab_bounds(backend.n, self.world, balance))
        self.c0, self.c1 = self.slabs[self.rank]
        self.S = max(c1 - c0 for c0, c1 in self.slabs)
        dev = backend.delta().device
        self.staging = (dist.is_initialized() and dist.get_backend(group) == "gloo"
                        and dev.type != "cpu")
        cdev = torch.device("cpu") if self.staging else dev
        self.send = torch.zeros(self.S, dtype=torch.float64, device=cdev)
        self.recv = torch.zeros(self.world * self.S, dtype=torch.float64, device=cdev)

    def _allgather_delta(self):
        d = self.b.delta()
        self.send.zero_()
        self.send[: self.c1 - self.c0].copy_(d[self.c0:self.c1])
        if self.world > 1:
            dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        else:
            self.recv.copy_(self.send)
        for r, (a, e) in enumerate(self.slabs):
            if r != self.rank and e > a:
                d[a:e].copy_(self.recv[r * self.S:r * self.S + (e - a)])

    def _allreduce_piv(self, rnd):
        """Sum the pivot data of round ``rnd`` (nom, P_yy, W[0..rnd)[y], V[0..rnd)[y]: the
        2 + 2 rnd entries greedy_select_kernel rewrites; only the owner of y writes non-zeros)."""
        if self.world == 1:
            return
        p = self.b.piv()[: 2 + 2 * rnd]
        if self.staging:
            h = p.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            p.copy_(h)
        else:
            dist.all_reduce(p, op=dist.ReduceOp.SUM, group=self.group)

    def _allreduce_xcol(self):
        """The last pick's column of L^-1: only its owner wrote non-zeros."""
        if self.world == 1:
            return
        x = self.b.xcol()
        if self.staging:
            h = x.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            x.copy_(h)
        else:
            dist.all_reduce(x, op=dist.ReduceOp.SUM, group=self.group)

    def _factor(self):
        self.b.snapshot_diag()
        if self.partition and self.world > 1 and self.dist_factor:
            from .dist_cholesky import DIST_MIN, DistCholesky
            self.b.prepare()
            dc = DistCholesky(self.b.chol_ops(), self.group,
                              DIST_MIN if self.dist_min is None else self.dist_min)
            dc.factor()
            self.b.finish_slab(self.c0, self.c1)
        elif self.partition:
            self.b.init_slab(self.c0, self.c1)
        else:
            self.b.init()

    def run(self, k, lazy=True):
        """snippets of placement_algorithm2.py:151-219 over the ranks.  A singular cov_vv takes
        the single-GPU path's jitter retry (SINGULAR_EPS relative to the mean diagonal), decided
        identically on every rank."""
        from ._lib import CholeskyError
        from .placement_algorithm2 import SINGULAR_EPS
        self._factor()
        if not self.b.factor_ok(self.c0, self.c1, self.partition, check_pivots=True):
            scale = self.b.diag_scale()
            for rel in SINGULAR_EPS:
                self.b.rejitter(rel * scale)
                self._factor()
                if self.b.factor_ok(self.c0, self.c1, self.partition, check_pivots=False):
                    break
            else:
                raise CholeskyError(1)
        for rnd in range(k):
            if self.partition and rnd > 0:
                self.b.extract(rnd, self.c0, self.c1)
                self._allreduce_xcol()
                self.b.update(rnd, self.c0, self.c1, extract=False)
            else:
                self.b.update(rnd, self.c0, self.c1)
            self._allgather_delta()
            self.b.select(rnd, lazy, self.c0, self.c1)
            self._allreduce_piv(rnd)
        return self.b.result()


def placement_algorithm_2_sharded(cov_vv, k, group=None, lazy=True, partition_inverse=True,
                                  dist_factor=True, dist_min=None):
    """placement_algorithm_2 with candidates sharded over the ranks of ``group`` (every rank
    passes the same cov_vv and gets the same list)."""
    sh = ShardedGreedyPlacement(HipGreedyBackend(cov_vv, k, copy=True), group,
                                partition_inverse=partition_inverse, dist_factor=dist_factor,
                                dist_min=dist_min)
    return sh.run(k, lazy)[0]

"""Config C4, exact: the reference's algorithm 3 on the beta-decay tapered covariance at grid sizes
where cov_vv cannot be dense (128^3 = 2,097,152 candidates: 35 TB dense).

Reference semantics (``snippets_a3.sparse_placement_algorithm_3``, ``snippets_a3.py:43-364``, on
the covariance ``main_architecture_2_sampledistribution.py:355-421`` builds): every candidate is
scored once; then per round the arg-max of the cache over V \\ A (lowest index on ties,
``placement_algorithm2.py:24-50``) is picked, its cache entry zeroed, and the candidates of the
index window ``[i_d - cutoff, i_d + cutoff)`` around it are re-scored with ``tf_nominator`` /
``tf_denominator`` (``snippets_a2.py:138-218``) over the FULL sets A and V \\ (A u {y}) — the
conditioning block gets ``+1e-6`` on its diagonal (``:161-163``), and a delta is 0 when ``|nom|``
or ``|denom|`` is below 1e-7 (``:480``).  After k - 1 rounds a last arg-max adds the k-th pick
(``:360-362``).  This module computes exactly those quantities without forming anything N x N:

* ``denom_y = 1 / Q_yy - eps`` in round 0 and ``1 / (Q_yy - Q_yA Q_AA^-1 Q_Ay) - eps`` later, with
  ``Q = (Sigma + eps I)^-1`` (block inverse of ``(Sigma + eps I)_{V \\ A}``).  diag(Q) comes from a
  nested-dissection multifrontal Cholesky and its selected inverse (``nested_dissection.py`` plans
  it; ``csrc/frontal.hip`` runs it: batched fp64 MFMA GEMMs and Cholesky per tree level).  Each pick
  a adds the column ``Q e_a`` (conjugate gradients on the stencil matrix, ``csrc/exact_greedy.hip``).
* ``nom_y = s_yy - s_yA (Sigma_AA + eps I)^-1 s_Ay`` from the |A| x |A| block.

So the selections are the reference's dense algorithm 3 on the tapered covariance, up to rounding:
``tests/test_gpu_exact.py`` compares them with the dense algorithm-3 engine
(``snippets_a3.placement_algorithm_3``) on every grid where the dense matrix fits.
"""
from __future__ import annotations

import ctypes
import math
import time

import numpy as np
import torch

from ._lib import KERNEL_KINDS, CholeskyError, call, query
from .linalg import _p, _stream
from .local_placement import TF_JITTER, TF_SMALL, taper_support
from .nested_dissection import frontal_tree

I32 = torch.int32


def _dev(a, dev, dtype=I32):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=dev)


class TaperProblem:
    """The tapered covariance of a C-order grid: points X [N, 3], kernel (kind, amp, ls),
    diag_shift (noise + jitter of the kernel matrix), beta-decay taper; the TF jitter of the
    conditioning blocks."""

    def __init__(self, X, shape, beta=4.0, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
                 jitter=TF_JITTER, threshold=TF_SMALL, device=None):
        self.shape = tuple(int(s) for s in shape)
        I0, I1, I2 = self.shape
        self.n = I0 * I1 * I2
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.device = dev
        X = torch.as_tensor(X, dtype=torch.float64, device=dev)
        if X.shape != (self.n, 3):
            raise ValueError(f"X must be [{self.n}, 3] grid points in C order, got {tuple(X.shape)}")
        self.X = X.contiguous()
        self.beta = float(beta)
        offs, tau = taper_support(beta)
        self.offs_np = np.asarray(offs, dtype=np.int64).reshape(-1, 3)
        self.m = len(self.offs_np) + 1
        self.offs = _dev(self.offs_np.reshape(-1) if len(self.offs_np) else np.zeros(3), dev)
        self.tau_np = np.asarray(tau, dtype=np.float64)
        self.tau = torch.as_tensor(self.tau_np, device=dev)
        self.kind_name = kind
        self.kind = KERNEL_KINDS[kind]
        self.amp, self.ls, self.shift = float(amp), float(ls), float(diag_shift)
        self.jitter, self.thr = float(jitter), float(threshold)

    def taper_args(self):
        return (self.kind, _p(self.X), *self.shape, self.amp, self.ls, self.shift, self.jitter)

    def cg_iterations(self, tol=1e-16):
        """CG iterations for a relative residual of ``tol`` from a Gershgorin bound on the spectrum
        of Sigma + eps I (the kernel is <= amp^2 off the diagonal); 400 without a positive bound."""
        a2 = self.amp ** 2
        d = self.tau_np[0] * (a2 + self.shift) + self.jitter
        s = sum(self.tau_np[int((o ** 2).sum())] for o in self.offs_np) * a2
        if d - s <= 0:
            return 400
        kappa = (d + s) / (d - s)
        rho = (math.sqrt(kappa) - 1) / (math.sqrt(kappa) + 1)
        if rho <= 0:
            return 1
        return int(min(400, math.ceil(math.log(tol / 2) / math.log(rho)) + 4))


class FrontalSelectedInverse:
    """diag((Sigma + eps I)^-1) of a TaperProblem through the nested-dissection plan: bottom-up
    multifrontal Cholesky (assembly, extend-add, batched partial factorization per tree level),
    then the top-down selected inverse.  Every call only enqueues work on the current stream."""

    def __init__(self, prob: TaperProblem, leaf=512):
        self.p = prob
        t0 = time.perf_counter()
        self.tree = frontal_tree(prob.shape, prob.offs_np, leaf)
        self.plan_s = time.perf_counter() - t0
        dev = prob.device
        T = self.tree
        self.owner_ord = _dev(T.owner, dev)
        self.owner_pos = _dev(T.owner_pos, dev)
        self.g = []
        for g in T.groups:
            self.g.append({
                "piv": _dev(g.piv, dev), "U": _dev(g.U, dev), "ulen": _dev(g.ulen, dev),
                "pmap": _dev(g.pmap, dev), "par_off": _dev(g.par_off, dev, torch.int64),
                "par_dim": _dev(g.par_dim, dev), "sib": _dev(g.sibling, dev),
                "order": _dev(g.order, dev)})
        self.infos = []

    def flops(self):
        return self.tree.flops(padded=True)

    def run(self, out=None, timer=None):
        """-> qdiag [N] (device).  Cholesky status per group in ``self.infos`` (device).
        ``timer`` (callable(tag)) is called between phases (e.g. to record events).

        Storage is per tree level: three flat buffers (PP, UP, UU) holding the level's groups at
        their plan offsets; a child's parent is addressed by its static offsets into the parent
        level's buffers (nested_dissection.Group.par_off)."""
        prob, T = self.p, self.tree
        tick = timer if timer is not None else (lambda tag: None)
        dev = prob.device
        f64 = torch.float64
        G = T.groups
        L = T.levels
        store = [None] * len(L)
        uu_prev = None
        self.infos = []
        tick(("start", -1))
        for li, lvl in enumerate(L):
            s0, s1, s2 = lvl["size"]
            PP = torch.zeros(max(s0, 1), dtype=f64, device=dev)
            UP = torch.zeros(max(s1, 1), dtype=f64, device=dev)
            UU = torch.zeros(max(s2, 1), dtype=f64, device=dev)
            for gi in lvl["groups"]:
                g, d = G[gi], self.g[gi]
                call("vgposp_front_assemble", *prob.taper_args(), _p(prob.offs), prob.m,
                     _p(prob.tau), prob.tau.numel(), _p(self.owner_ord), _p(self.owner_pos),
                     _p(d["piv"]), g.p, _p(d["U"]), g.u, _p(d["ulen"]), _p(d["order"]), g.nf,
                     _p(PP[g.off[0]:]), _p(UP[g.off[1]:]), _stream())
            if li > 0:
                for ci in L[li - 1]["groups"]:
                    c, cd = G[ci], self.g[ci]
                    if not c.u:
                        continue
                    for sib in (0, 1):
                        call("vgposp_front_extend_add", _p(uu_prev[c.off[2]:]), c.u, c.nf,
                             _p(cd["pmap"]), _p(cd["par_off"]), _p(cd["par_dim"]), _p(cd["sib"]),
                             sib, _p(PP), _p(UP), _p(UU), _stream())
            uu_prev = None
            for gi in lvl["groups"]:
                g = G[gi]
                info = torch.empty(g.nf, dtype=I32, device=dev)
                ws = torch.empty(query("vgposp_front_factor_workspace_bytes", g.p, g.u, g.nf),
                                 dtype=torch.uint8, device=dev)
                call("vgposp_front_factor", _p(PP[g.off[0]:]), _p(UP[g.off[1]:] if g.u else None),
                     _p(UU[g.off[2]:] if g.u else None), g.p, g.u, g.nf, _p(info), _p(ws),
                     ws.numel(), _stream())
                del ws
                self.infos.append(info)
            tick(("factor", li))
            store[li] = (PP, UP)
            uu_prev = UU
        del uu_prev
        qdiag = out if out is not None else torch.empty(prob.n, dtype=f64, device=dev)
        Qpar = None
        for li in range(len(L) - 1, -1, -1):
            lvl = L[li]
            s0, s1, s2 = lvl["size"]
            M, W = store[li]
            QPP = torch.empty(max(s0, 1), dtype=f64, device=dev)
            QUP = torch.empty(max(s1, 1), dtype=f64, device=dev)
            QUU = torch.empty(max(s2, 1), dtype=f64, device=dev)
            for gi in lvl["groups"]:
                g, d = G[gi], self.g[gi]
                if g.u:
                    call("vgposp_front_gather", _p(Qpar[0]), _p(Qpar[1]), _p(Qpar[2]),
                         _p(d["pmap"]), _p(d["par_off"]), _p(d["par_dim"]), g.nf, g.u,
                         _p(QUU[g.off[2]:]), _stream())
                call("vgposp_front_selinv", _p(M[g.off[0]:]), _p(W[g.off[1]:] if g.u else None),
                     _p(QUU[g.off[2]:] if g.u else None), g.p, g.u, g.nf, _p(QPP[g.off[0]:]),
                     _p(QUP[g.off[1]:] if g.u else None), _stream())
                call("vgposp_front_diag", _p(QPP[g.off[0]:]), g.p, g.nf, _p(d["piv"]), _p(qdiag),
                     _stream())
            store[li] = None
            del M, W
            Qpar = (QPP, QUP, QUU)
            tick(("selinv", li))
        return qdiag

    def check(self):
        for gi, info in enumerate(self.infos):
            bad = torch.nonzero(info).flatten()
            if len(bad):
                b = int(bad[0])
                raise CholeskyError(int(info[b]), b)


class ExactWindowGreedy:
    """The rounds of algorithm 3 on a TaperProblem, given diag(Q)."""

    def __init__(self, prob: TaperProblem, kmax, cutoff, cg_tol=1e-16, cg_iters=None):
        if kmax > 128:
            raise ValueError("the exact path places at most 128 sensors per run")
        self.p = prob
        self.kmax, self.cutoff = int(kmax), int(cutoff)
        dev = prob.device
        n = prob.n
        self.radius = max(int(np.abs(prob.offs_np).max()) if len(prob.offs_np) else 1, 1)
        self.cache = torch.zeros(n, dtype=torch.float64, device=dev)
        self.selected = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.picks = torch.full((self.kmax,), -1, dtype=torch.int64, device=dev)
        self.pick_delta = torch.zeros(self.kmax, dtype=torch.float64, device=dev)
        self.cg_tol = float(cg_tol)
        self.cg_iters = int(cg_iters) if cg_iters else prob.cg_iterations(cg_tol)
        self.box = [min(2 * self.radius * self.cg_iters + 1, s) for s in prob.shape]
        self.ws = torch.empty(query("vgposp_exact_workspace_bytes", *prob.shape, prob.m, self.kmax,
                                    self.radius, self.cg_iters), dtype=torch.uint8, device=dev)

    def _args(self, qdiag):
        pr = self.p
        return (*pr.taper_args(), pr.thr, _p(pr.offs), pr.m, _p(pr.tau), pr.tau.numel(),
                self.kmax, self.cutoff, self.radius, self.cg_iters, _p(qdiag), _p(self.cache),
                _p(self.selected), _p(self.ws), self.ws.numel())

    def run(self, qdiag, k, snapshots=None):
        """snippets_a3.py:43-364 -> picks [k] (device).  ``snapshots`` (list) receives the cache
        after round 0 and after every window re-score (delta_cached_iters columns)."""
        if k > self.kmax:
            raise ValueError(f"k = {k} > kmax = {self.kmax}")
        self.picks.fill_(-1)
        call("vgposp_exact_prepare", *self._args(qdiag), _stream())
        if snapshots is not None:
            snapshots.append(self.cache.clone())
        for t in range(k):
            last = t == k - 1
            call("vgposp_exact_round", *self._args(qdiag), t, int(last), _p(self.picks),
                 _p(self.pick_delta), self.cg_tol, _stream())
            if snapshots is not None and not last:
                snapshots.append(self.cache.clone())
        return self.picks[:k]

    def _buffers(self):
        q, b, c = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        call("vgposp_exact_buffers", _p(self.ws), *self.p.shape, self.p.m, self.kmax, self.radius,
             self.cg_iters, ctypes.byref(q), ctypes.byref(b), ctypes.byref(c))
        base = self.ws.data_ptr()
        return q.value - base, b.value - base, c.value - base

    def q_columns(self):
        """The CG columns Q e_{a_t} expanded to the grid: [kmax, N] (zero outside each box)."""
        qo, bo, _ = self._buffers()
        b0, b1, b2 = self.box
        bv = b0 * b1 * b2
        cols = self.ws[qo: qo + 8 * self.kmax * bv].view(torch.float64).view(self.kmax, b0, b1, b2)
        lo = self.ws[bo: bo + 8 * 3 * self.kmax].view(torch.int64).view(self.kmax, 3).cpu()
        full = torch.zeros((self.kmax,) + self.p.shape, dtype=torch.float64, device=self.ws.device)
        for t in range(self.kmax):
            l0, l1, l2 = (int(v) for v in lo[t])
            full[t, l0:l0 + b0, l1:l1 + b1, l2:l2 + b2] = cols[t]
        return full.view(self.kmax, -1)

    def cg_iterations_used(self):
        """Iterations the last CG solve took (the full budget if it did not stop early)."""
        _, _, co = self._buffers()
        st = self.ws[co: co + 8].view(torch.int32)
        return int(st[1]) if int(st[0]) else self.cg_iters


class ExactTaperPlacement:
    """One C4 problem end to end: selected inverse + rounds (device-resident)."""

    def __init__(self, X, shape, k, cutoff, beta=4.0, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
                 jitter=TF_JITTER, threshold=TF_SMALL, leaf=512, device=None):
        self.prob = TaperProblem(X, shape, beta, kind, amp, ls, diag_shift, jitter, threshold,
                                 device)
        self.sel = FrontalSelectedInverse(self.prob, leaf)
        self.greedy = ExactWindowGreedy(self.prob, k, cutoff)
        self.k = int(k)
        self.qdiag = torch.empty(self.prob.n, dtype=torch.float64, device=self.prob.device)

    def run(self, snapshots=None):
        self.sel.run(out=self.qdiag)
        return self.greedy.run(self.qdiag, self.k, snapshots)

    def check(self):
        self.sel.check()


def tapered_placement_algorithm_3(X, k, COVER_spatial, cutoff, beta=4.0, kernel="eq", amp=1.0,
                                  ls=1.0, diag_shift=0.0, snapshots=False, leaf=512):
    """snippets_a3.sparse_placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff) for the tapered
    covariance of the grid points X (C order, COVER_spatial = (I0, I1, I2)), exact, without the
    dense cov_vv.  -> (picks as a list of np.int64 in selection order, the pick deltas,
    delta_cached_iters [N, k] or None)."""
    shape = tuple(int(c) for c in COVER_spatial[:3])
    N = shape[0] * shape[1] * shape[2]
    if len(X) != N:                                         # snippets_a3.py:51 tf.Assert
        raise ValueError(f"assertion failed: N = {len(X)} != prod(COVER_spatial) = {N}")
    run = ExactTaperPlacement(X, shape, k, cutoff, beta, kernel, amp, ls, diag_shift, leaf=leaf)
    snaps = [] if snapshots else None
    picks = run.run(snaps).cpu().numpy()
    run.check()
    dci = torch.stack(snaps, 1).cpu().numpy() if snapshots else None
    return [np.int64(a) for a in picks], run.greedy.pick_delta[:k].cpu().numpy(), dci


__all__ = ["TaperProblem", "FrontalSelectedInverse", "ExactWindowGreedy", "ExactTaperPlacement",
           "tapered_placement_algorithm_3"]

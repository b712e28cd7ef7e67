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
from .taper import TF_JITTER, TF_SMALL, taper_support
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


class HipFrontalOps:
    """The device operations of the multifrontal selected inverse on libvgposp (frontal.hip):
    flat fp64 level buffers are torch tensors, every call enqueues on the current stream."""

    def __init__(self, prob: TaperProblem):
        self.p = prob
        self.dev = prob.device

    # buffers
    def zeros(self, n):
        return torch.zeros(max(int(n), 1), dtype=torch.float64, device=self.dev)

    def empty(self, n):
        return torch.empty(max(int(n), 1), dtype=torch.float64, device=self.dev)

    @staticmethod
    def at(buf, off):
        return None if buf is None else buf[int(off):]

    def ints(self, a, dtype=np.int32):
        return _dev(np.asarray(a, dtype=dtype), self.dev,
                    torch.int64 if dtype == np.int64 else torch.int32)

    @staticmethod
    def block(buf, off, rows, ld, cols):
        """[rows, cols] view of a row-major block with leading dimension ld at offset off."""
        return buf[int(off): int(off) + rows * ld].view(rows, ld)[:, :cols]

    # dense / sparse front steps
    def assemble(self, tree, g, d, PP, UP):
        pr = self.p
        call("vgposp_front_assemble", *pr.taper_args(), _p(pr.offs), pr.m, _p(pr.tau),
             pr.tau.numel(), _p(d["owner_ord"]), _p(d["owner_pos"]), _p(d["piv"]), g.p,
             _p(d["U"]), g.u, _p(d["ulen"]), _p(d["order"]), g.nf, _p(PP), _p(UP), _stream())

    def extend_add(self, UUc, uc, nfc, pmap, par_off, par_dim, sibl, sib, PP, UP, UU):
        call("vgposp_front_extend_add", _p(UUc), uc, nfc, _p(pmap), _p(par_off), _p(par_dim),
             _p(sibl), sib, _p(PP), _p(UP), _p(UU), _stream())

    def factor(self, PP, UP, UU, p, u, nf):
        info = torch.empty(nf, dtype=I32, device=self.dev)
        ws = torch.empty(query("vgposp_front_factor_workspace_bytes", p, u, nf),
                         dtype=torch.uint8, device=self.dev)
        call("vgposp_front_factor", _p(PP), _p(UP), _p(UU), p, u, nf, _p(info), _p(ws), ws.numel(),
             _stream())
        return info

    def gather(self, QPP, QUP, QUU, pmap, par_off, par_dim, nfc, uc, out):
        call("vgposp_front_gather", _p(QPP), _p(QUP), _p(QUU), _p(pmap), _p(par_off),
             _p(par_dim), nfc, uc, _p(out), _stream())

    def selinv(self, M, W, QUU, p, u, nf, QPP, QUP):
        call("vgposp_front_selinv", _p(M), _p(W), _p(QUU), p, u, nf, _p(QPP), _p(QUP), _stream())

    def diag(self, QPP, p, nf, piv, out):
        call("vgposp_front_diag", _p(QPP), p, nf, _p(piv), _p(out), _stream())

    @staticmethod
    def nonzero_info(info):
        bad = torch.nonzero(info).flatten()
        return (int(bad[0]), int(info[int(bad[0])])) if len(bad) else None

    # transfers carry the lower triangle only (row-packed, n (n + 1) / 2 doubles)
    def pack_lower(self, buf, off, ld, n):
        out = torch.empty(max(n * (n + 1) // 2, 1), dtype=torch.float64, device=self.dev)
        call("vgposp_pack_rows", _p(buf[int(off):]), ld, 0, n, 0, n, 1, _p(out), 0, _stream())
        return out[:n * (n + 1) // 2]

    def unpack_lower(self, packed, buf, off, ld, n, symmetric):
        call("vgposp_pack_rows", _p(buf[int(off):]), ld, 0, n, 0, n, 1, _p(packed), 1, _stream())
        if symmetric:
            call("vgposp_sym_from_lower", _p(buf[int(off):]), n, ld, _stream())

    def empty_packed(self, n):
        return torch.empty(max(n * (n + 1) // 2, 1), dtype=torch.float64,
                           device=self.dev)[:n * (n + 1) // 2]


class FrontComm:
    """Point-to-point transfers of [ulen, ulen] blocks between the ranks of the subcube mapping
    and the final sum of the diag(Q) slabs: RCCL over xGMI for device tensors with the ``nccl``
    backend, host-staged with gloo."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.bytes = 0

    def _staged(self, t):
        return self.dist.get_backend(self.group) == "gloo" and t.device.type != "cpu"

    def send(self, t, dst):
        t = t.contiguous()
        self.bytes += t.numel() * t.element_size()
        if self._staged(t):
            self.dist.send(t.cpu(), dst, group=self.group)
        else:
            self.dist.send(t, dst, group=self.group)

    def recv(self, t, src):
        if self._staged(t):
            h = torch.empty(t.shape, dtype=t.dtype)
            self.dist.recv(h, src, group=self.group)
            t.copy_(h)
        else:
            self.dist.recv(t, src, group=self.group)

    def allreduce(self, t):
        if self._staged(t):
            h = t.cpu()
            self.dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            self.dist.all_reduce(t, group=self.group)


class FrontalSelectedInverse:
    """diag((Sigma + eps I)^-1) of a TaperProblem through the nested-dissection plan: bottom-up
    multifrontal Cholesky (assembly, extend-add, batched partial factorization per tree level),
    then the top-down selected inverse.  Every call only enqueues work on the current stream.

    Over R ranks (``comm`` with world R): subtree-to-subcube mapping (nested_dissection.
    FrontalLayout) — each rank factors its own subtrees, a front whose parent lives on another
    rank sends its [u, u] update there and receives its Q_UU back, and the diag(Q) slabs are
    summed at the end (each node belongs to exactly one rank)."""

    def __init__(self, prob: TaperProblem, leaf=512, comm=None, ops=None):
        self.p = prob
        t0 = time.perf_counter()
        self.tree = frontal_tree(prob.shape, prob.offs_np, leaf)
        self.comm = comm
        world = comm.world if comm is not None else 1
        rank = comm.rank if comm is not None else 0
        self.lay = self.tree.layout(world, rank) if world > 1 else self.tree.layout(1, 0)
        self.plan_s = time.perf_counter() - t0
        self.ops = ops if ops is not None else HipFrontalOps(prob)
        o = self.ops
        T = self.tree
        self.owner_ord = o.ints(T.owner)
        self.owner_pos = o.ints(T.owner_pos)
        self.g = []
        for g in self.lay.groups:
            self.g.append({
                "piv": o.ints(g.piv), "U": o.ints(g.U), "ulen": o.ints(g.ulen),
                "pmap": o.ints(g.pmap), "par_off": o.ints(g.par_off, np.int64),
                "par_dim": o.ints(g.par_dim), "sib": o.ints(g.sibling), "order": o.ints(g.order),
                "owner_ord": self.owner_ord, "owner_pos": self.owner_pos})
        self.remote = {}
        for li in range(len(self.lay.levels)):
            for rc in self.lay.recv_update[li]:
                self.remote[rc.front] = {
                    "pmap": o.ints(rc.pmap[None, :]), "par_off": o.ints(rc.par_off[None, :],
                                                                          np.int64),
                    "par_dim": o.ints(rc.par_dim[None, :]), "sib": o.ints([rc.sibling])}
        self.infos = []

    def flops(self):
        """Padded flops of this rank's fronts."""
        return self.lay.flops()

    def run(self, out=None, timer=None):
        """-> qdiag [N] (device).  Cholesky status per group in ``self.infos`` (device).
        ``timer`` (callable(tag)) is called between phases (e.g. to record events).

        Storage is per tree level: three flat buffers (PP, UP, UU) holding the level's groups at
        their plan offsets; a child's parent is addressed by its static offsets into the parent
        level's buffers (nested_dissection.Group.par_off)."""
        o, T, lay, comm = self.ops, self.tree, self.lay, self.comm
        tick = timer if timer is not None else (lambda tag: None)
        G, L = lay.groups, lay.levels
        store = [None] * len(L)
        uu_prev = None
        self.infos = []
        tick(("start", -1))
        for li, lvl in enumerate(L):
            s0, s1, s2 = lvl["size"]
            PP, UP, UU = o.zeros(s0), o.zeros(s1), o.zeros(s2)
            for gi in lvl["groups"]:
                g = G[gi]
                o.assemble(T, g, self.g[gi], o.at(PP, g.off[0]), o.at(UP, g.off[1]))
            if li > 0:
                for ci in L[li - 1]["groups"]:
                    c, cd = G[ci], self.g[ci]
                    if not c.u:
                        continue
                    for sib in (0, 1):
                        o.extend_add(o.at(uu_prev, c.off[2]), c.u, c.nf, cd["pmap"],
                                     cd["par_off"], cd["par_dim"], cd["sib"], sib, PP, UP, UU)
            for rc in lay.recv_update[li]:          # updates of children on other ranks
                n = rc.ulen
                pk = o.empty_packed(n)
                comm.recv(pk, rc.src)
                buf = o.zeros(n * n)
                o.unpack_lower(pk, buf, 0, n, n, False)
                del pk
                r = self.remote[rc.front]
                o.extend_add(buf, rc.ulen, 1, r["pmap"], r["par_off"], r["par_dim"], r["sib"],
                             rc.sibling, PP, UP, UU)
                del buf
            uu_prev = None
            for gi in lvl["groups"]:
                g = G[gi]
                self.infos.append(o.factor(o.at(PP, g.off[0]), o.at(UP, g.off[1]) if g.u else None,
                                           o.at(UU, g.off[2]) if g.u else None, g.p, g.u, g.nf))
            for gi, s, fi, dst in lay.send_update[li]:
                g = G[gi]
                n = T.fronts[fi].U.size
                comm.send(o.pack_lower(UU, g.off[2] + s * g.u * g.u, g.u, n), dst)
            tick(("factor", li))
            store[li] = (PP, UP)
            uu_prev = UU
        del uu_prev
        qdiag = out if out is not None else o.empty(T.n)
        if comm is not None and comm.world > 1:
            qdiag.zero_()
        Qpar = None
        for li in range(len(L) - 1, -1, -1):
            lvl = L[li]
            s0, s1, s2 = lvl["size"]
            M, W = store[li]
            QPP, QUP = o.empty(s0), o.empty(s1)
            QUU = o.zeros(s2) if lay.recv_q[li] else o.empty(s2)
            for gi in lvl["groups"]:
                g, d = G[gi], self.g[gi]
                if g.u and Qpar is not None:
                    o.gather(Qpar[0], Qpar[1], Qpar[2], d["pmap"], d["par_off"], d["par_dim"],
                             g.nf, g.u, o.at(QUU, g.off[2]))
            # Q_UU of fronts whose parent is on another rank (after the gathers, which leave
            # those slots zero)
            for gi, s, fi, src in lay.recv_q[li]:
                g = G[gi]
                n = T.fronts[fi].U.size
                pk = o.empty_packed(n)
                comm.recv(pk, src)
                o.unpack_lower(pk, QUU, g.off[2] + s * g.u * g.u, g.u, n, True)
                del pk
            for gi in lvl["groups"]:
                g, d = G[gi], self.g[gi]
                o.selinv(o.at(M, g.off[0]), o.at(W, g.off[1]) if g.u else None,
                         o.at(QUU, g.off[2]) if g.u else None, g.p, g.u, g.nf,
                         o.at(QPP, g.off[0]), o.at(QUP, g.off[1]) if g.u else None)
                o.diag(o.at(QPP, g.off[0]), g.p, g.nf, d["piv"], qdiag)
            for rc in lay.send_q[li]:               # Q_UU for children on other ranks
                r = self.remote[rc.front]
                buf = o.empty(rc.ulen * rc.ulen)
                o.gather(QPP, QUP, QUU, r["pmap"], r["par_off"], r["par_dim"], 1, rc.ulen, buf)
                comm.send(o.pack_lower(buf, 0, rc.ulen, rc.ulen), rc.src)
                del buf
            store[li] = None
            del M, W
            Qpar = (QPP, QUP, QUU)
            tick(("selinv", li))
        if comm is not None and comm.world > 1:
            comm.allreduce(qdiag)
        return qdiag

    def check(self):
        for info in self.infos:
            bad = self.ops.nonzero_info(info)
            if bad is not None:
                raise CholeskyError(bad[1], bad[0])


_REACH = {}


def reach_table(offsets, K):
    """The grid offsets within K stencil steps of a node (breadth-first over the stencil
    ``offsets`` [m-1, 3]), sorted by step count, then C order: (tab [T, 3] int32 with the node
    itself first, cnt [K + 1] int32 = offsets within d steps, nb [T, m-1] int32 = row of
    tab[i] + offsets[o] in the table or -1).  The K-step Krylov space of e_y lives on exactly these
    nodes (around y, clipped to the grid).  Depends on the stencil only (not on the data), so it
    is built once per (stencil, K)."""
    key = (np.asarray(offsets, dtype=np.int64).tobytes(), int(K))
    if key not in _REACH:
        _REACH[key] = _reach_table(offsets, K)
    return _REACH[key]


def _reach_table(offsets, K):
    offs = [tuple(int(v) for v in o) for o in np.asarray(offsets, dtype=np.int64).reshape(-1, 3)]
    dist = {(0, 0, 0): 0}
    frontier = [(0, 0, 0)]
    for d in range(1, int(K) + 1):
        nxt = []
        for v in frontier:
            for o in offs:
                w = (v[0] + o[0], v[1] + o[1], v[2] + o[2])
                if w not in dist:
                    dist[w] = d
                    nxt.append(w)
        frontier = nxt
    items = sorted(dist.items(), key=lambda kv: (kv[1], kv[0]))
    tab = np.array([k for k, _ in items], dtype=np.int32).reshape(-1, 3)
    dd = np.array([v for _, v in items], dtype=np.int64)
    cnt = np.array([(dd <= d).sum() for d in range(int(K) + 1)], dtype=np.int32)
    pos = {k: i for i, (k, _) in enumerate(items)}
    nb = np.full((len(tab), max(len(offs), 1)), -1, dtype=np.int32)
    for i, (k, _) in enumerate(items):
        for j, o in enumerate(offs):
            nb[i, j] = pos.get((k[0] + o[0], k[1] + o[1], k[2] + o[2]), -1)
    return tab, cnt, nb[:, :len(offs)]


def cg_iterations_for(lam_min, lam_max, tol=1e-16):
    """CG iterations for a relative residual of ``tol`` on a spectrum inside [lam_min, lam_max]
    (the Chebyshev bound 2 rho^it, plus 4 for rounding)."""
    kappa = lam_max / lam_min
    rho = (math.sqrt(kappa) - 1) / (math.sqrt(kappa) + 1)
    if rho <= 0:
        return 1
    return int(min(400, math.ceil(math.log(tol / 2) / math.log(rho)) + 4))


BOUND_TMAX, BOUND_NBMAX = 14 * 64, 8192
REFINE_BATCH = 32       # candidates refined together by one batched CG (vgposp_exact_refine_pending);
#                         measured at 128^3: batch 8 14.3 ms, 16 13.4, 32 12.4 (profiles/r4_c4_batch_*)
REFINE_BATCH_MAX = 32   # the library's CG_B
BOUND_MARGIN = 1e-12                       # relative rounding margin on the upper bounds
# Two-level bounds: every candidate gets the K_lo-step bound (bracket width <= BOUND_LO_TARGET:
# K = 4 at the reference's beta = 4), the few that reach a refinement batch the K_hi-step one
# (width <= BOUND_HI_TARGET, K = 6) before any of them is given a CG column.  One K = 5 level for
# all (round 3's) cost the 2M-candidate bounds pass 4.8 ms at 128^3.
BOUND_LO_TARGET = 3e-5
PRETIGHTEN = 2048      # two levels: candidates tightened before the rounds (at most 32,768)
BOUND_HI_TARGET = 1e-7


def bound_steps(offsets, lam_min, lam_max, target=1e-6, kmax=12):
    """(K, hi_scale, width) for vgposp_exact_bounds: the fewest CG steps whose bracket width
    4 rho^2K is <= target, else the most whose reach table fits the kernel (at most kmax);
    rho = (sqrt(kappa) - 1) / (sqrt(kappa) + 1) from the Gershgorin bounds.  The bracket only
    decides how often the rounds refine (a CG column each): at 128^3, beta = 4 a width of 1e-6
    (K = 5) refines 51 times for k = 50, 2e-5 (K = 4) 111 times, 4e-8 (K = 6) 50 times at twice
    the bounds cost.  None when the bounds cannot bracket Q_yy (lambda_min <= 0, or no K with
    4 rho^2K < 1/2)."""
    if not (lam_min > 0.0 and lam_max >= lam_min):
        return None
    kappa = lam_max / lam_min
    rho = (math.sqrt(kappa) - 1.0) / (math.sqrt(kappa) + 1.0)
    m1 = len(np.asarray(offsets).reshape(-1, 3))
    best = None
    for K in range(1, kmax + 1):
        tab, _, _ = reach_table(offsets, K)
        if len(tab) > BOUND_TMAX or len(tab) * m1 > BOUND_NBMAX:
            break
        width = 4.0 * rho ** (2 * K)
        if width < 0.5:
            best = (K, (1.0 + BOUND_MARGIN) / (1.0 - width), width)
            if width <= target:
                break
    return best


def radau_steps(b):
    """The Gauss-Radau form of a Chebyshev (K, hi_scale, width) triple: K - 1 steps (at least 1),
    hi_scale = the rounding margin only, width = the Chebyshev width of K steps (the Radau
    bracket after K - 1 steps measures about that on the beta = 4 taper; informational only —
    the bound is valid whatever its width)."""
    K, _, width = b
    return (max(1, K - 1), 1.0 + BOUND_MARGIN, width)


class ExactWindowGreedy:
    """The rounds of algorithm 3 on a TaperProblem: given diag(Q) (``run``, after the selected
    inverse), or with diag(Q) only bounded (``run_bounded``, after ``bound_qdiag``)."""

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
        self.nslots = 2 * self.kmax
        self.refinements = 0      # candidates refined (CG columns) in the last bounded run
        self.refine_batches = 0   # batched CG solves in the last bounded run
        self.bound = None
        self.tight = None
        # bound_qdiag's default: two bound levels (Gauss-Radau K = 3 for every candidate, K = 5
        # for the `pretighten` (2,048) best round-0 entries at once and for any other that reaches a
        # refinement batch): 6.3 ms per 128^3 k = 50 run against 6.75 for one level of K = 4.
        # Without the pre-tightening two levels lost (8.0 ms: 134 candidates tightened in 6
        # refinement events, each a host round trip; profiles/r4_c4_pretighten.jsonl)
        self.two_level = True
        self.radau = True         # Gauss-Radau upper bounds (mu = the Gershgorin lambda_min)
        self.bound_target = 1e-6  # one-level bracket target (Chebyshev width; Radau: one step less)
        self.lo_target = BOUND_LO_TARGET  # two levels: the first level's bracket target
        # two levels: the candidates with the largest round-0 entries tightened at once before
        # the rounds (vgposp_exact_pretighten); 0 = only on demand, by refinement events
        self.pretighten = PRETIGHTEN
        self.bound_mu = 0.0       # mu of the last bounds (0: the Chebyshev bound)
        self.tightened = 0        # candidates tightened to the K_hi bound in the last bounded run

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
        call("vgposp_exact_prepare", *self._args(qdiag), 0, _stream())
        if snapshots is not None:
            snapshots.append(self.cache.clone())
        for t in range(k):
            last = t == k - 1
            call("vgposp_exact_round", *self._args(qdiag), t, int(last), _p(self.picks),
                 _p(self.pick_delta), self.cg_tol, _stream())
            if snapshots is not None and not last:
                snapshots.append(self.cache.clone())
        return self.picks[:k]

    # ---------------------------------------------------------------- bounded-lazy form
    def gershgorin(self, qdiag):
        """Stencil coefficients + Gershgorin [lambda_min, lambda_max] of Sigma + eps I (one host
        read)."""
        call("vgposp_exact_coef", *self._args(qdiag), _stream())
        off = self._buffers()[5]
        g = self.ws[off: off + 16].view(torch.float64).cpu()
        return float(g[0]), float(g[1])

    def bound_qdiag(self, qdiag, c0=0, c1=None, steps=None, tighten=None, mu=0.0):
        """qdiag[c0:c1] <- upper bounds of Q_yy (vgposp_exact_bounds).  Returns the (K, hi_scale,
        width) used, or None when the spectrum bounds cannot bracket Q_yy (then the selected
        inverse is the only exact route).  ``steps``: an explicit (K, hi_scale, width) triple,
        with ``mu`` > 0 its Gauss-Radau form (default: the Chebyshev form); otherwise the steps
        are chosen here, in the Gauss-Radau form when ``self.radau``.  With ``tighten`` (7-point
        stencils) the bounds are
        the K_lo-step ones and run_bounded tightens candidates to K_hi steps before their CG
        column (``self.tight`` = the K_hi triple, None when there is no second level; default
        ``self.two_level``)."""
        tighten = self.two_level if tighten is None else tighten
        lo, hi = self.gershgorin(qdiag)
        offs = self.p.offs_np
        two = tighten and steps is None and len(offs.reshape(-1, 3)) == 6
        if steps is not None:
            b = steps
        else:
            b = bound_steps(offs, lo, hi, target=self.lo_target if two else self.bound_target)
        self.tight = None
        self.bound_mu = float(mu) if steps is not None else 0.0
        if b is None:
            self.bound = None
            return None
        if two:
            t = bound_steps(offs, lo, hi, target=BOUND_HI_TARGET)
            if t is not None and t[0] > b[0]:
                self.tight = t
        if self.radau and steps is None:
            # the Gauss-Radau bound brackets after K steps about as tightly as the Chebyshev one
            # after K + 1 (exact_greedy.hip, radau_step): one CG step fewer for the same width
            self.bound_mu = lo
            b = radau_steps(b)
            if self.tight is not None:
                self.tight = radau_steps(self.tight)
        self.bound = b
        # the measured spectrum bounds are tighter than the kernel-agnostic one the columns were
        # sized with: fewer CG iterations (and a smaller Krylov box) give the same tolerance
        its = cg_iterations_for(lo, hi, self.cg_tol)
        if its < self.cg_iters:
            self.cg_iters = its
            self.box = [min(2 * self.radius * its + 1, s) for s in self.p.shape]
        K, scale, _ = b
        tab, T = self._device_table(K)
        c1 = self.p.n if c1 is None else int(c1)
        call("vgposp_exact_bounds", *self._args(qdiag), *[_p(a) for a in tab], T, K, scale,
             self.bound_mu, int(c0), c1, _stream())
        return b

    def _device_table(self, K):
        """The reach table of K steps on the device (int32: offsets, neighbours, counts), uploaded
        once per K."""
        tabs = self.__dict__.setdefault("_tabs", {})
        if K not in tabs:
            tab, cnt, nb = reach_table(self.p.offs_np, K)
            dev = self.p.device
            tabs[K] = ([torch.as_tensor(np.ascontiguousarray(a).reshape(-1), dtype=torch.int32,
                                        device=dev)
                        for a in (tab, nb if nb.size else np.zeros(1), cnt)], len(tab))
        return tabs[K]

    def run_bounded(self, qdiag, k, batch=None):
        """The rounds with qdiag holding upper bounds of Q_yy: the cache holds upper bounds of the
        reference's cached deltas; an arg-max that lands on a candidate whose Q_yy is only bounded
        refines it (its CG column; its cache entry becomes the reference's value) and the arg-max
        is taken again, so every pick is the reference's arg-max.  The refinement takes the
        ``batch`` (<= 8) best entries without a column together — one batched CG costs the
        launches of one column, and the next rounds' picks are mostly among them.

        The refine-or-pick decision is made ON THE DEVICE (vgposp_exact_steps: one kernel per
        round takes the arg-max and either picks it or stalls the rounds and writes the
        refinement batch).  The host reads the 32-byte control block once per refinement event
        (about 7 per 128^3 run), refines the pending batch (vgposp_exact_refine_pending) and
        re-issues the rounds from the stalled one — as many as there are refined candidates not
        yet picked, plus the one that will stall next.  Round 3 read the device twice per
        arg-max instead (57 host reads per run)."""
        if k > self.kmax:
            raise ValueError(f"k = {k} > kmax = {self.kmax}")
        B = REFINE_BATCH if batch is None else int(batch)
        if not 1 <= B <= REFINE_BATCH_MAX:
            raise ValueError(f"batch must be in [1, {REFINE_BATCH_MAX}], got {B}")
        self.picks.fill_(-1)
        args = self._args(qdiag)
        st = _stream()
        tight = self.tight
        call("vgposp_exact_prepare", *args, 1 if tight is None else 3, st)
        call("vgposp_exact_steps_reset", *args, st)
        ctl = self._ctl()
        pk, pd = _p(self.picks), _p(self.pick_delta)
        if tight is not None:
            ttab, tT = self._device_table(tight[0])
            targs = (*[_p(a) for a in ttab], tT, tight[0], tight[1], self.bound_mu, pk)
        if tight is not None and self.pretighten > 0:
            call("vgposp_exact_pretighten", *args, *targs[:-1], int(self.pretighten), st)
        call("vgposp_exact_steps", *args, 0, 1, k, B, pk, pd, st)  # round 0 stalls: nothing refined
        issued, reads = 1, 0
        # every host read must show progress since the previous one: the stall moved to another
        # round, or candidates were refined (c[4]) or tightened (c[7]), or (no stall) more rounds
        # were issued.  A read that shows none of these would repeat forever.  (Counting reads
        # instead is wrong: recycled slots let a candidate be refined again, and stall events per
        # round are not bounded by the batch size.)
        prev = None
        while True:
            # stall round, CG batch, refined-unpicked, events, refined, age, tightening list, tightened
            c = ctl.cpu().tolist()
            reads += 1
            state = (c[0], c[4], c[7], issued)
            if state == prev:
                raise RuntimeError(f"run_bounded: control block {c} unchanged after the previous "
                                   f"read ({reads} reads, k = {k}): the device rounds are not "
                                   "progressing")
            prev = state
            stall = c[0]
            if stall >= 0:
                if c[1] == 0 and c[6] == 0:
                    raise RuntimeError(f"run_bounded: round {stall} stalled with neither a CG "
                                       f"batch nor a tightening list (control block {c})")
                if c[6] > 0:
                    if tight is None:
                        raise RuntimeError("tightening list without a K_hi table")
                    call("vgposp_exact_tighten_pending", *args, *targs, st)
                if c[1] > 0:
                    call("vgposp_exact_refine_pending", *args, B, pk, self.cg_tol, st)
                r0, r1 = stall, min(k, stall + c[2] + c[1] + 1)
            elif issued < k:
                r0, r1 = issued, min(k, issued + max(c[2], 0) + 1)
            else:
                break
            call("vgposp_exact_steps", *args, r0, r1, k, B, pk, pd, st)
            issued = r1
        self.refinements, self.refine_batches, self.host_reads = c[4], c[3], reads
        self.tightened = c[7]
        return self.picks[:k]

    def _ctl(self):
        """The device control block of the rounds (int32 [8], vgposp_exact_buffers)."""
        p = ctypes.c_void_p()
        call("vgposp_exact_ctl", _p(self.ws), *self.p.shape, self.p.m, self.kmax, self.radius,
             self.cg_iters, ctypes.byref(p))
        off = p.value - self.ws.data_ptr()
        return self.ws[off: off + 32].view(torch.int32)

    def _buffers(self):
        ptrs = [ctypes.c_void_p() for _ in range(6)]
        call("vgposp_exact_buffers", _p(self.ws), *self.p.shape, self.p.m, self.kmax, self.radius,
             self.cg_iters, *[ctypes.byref(q) for q in ptrs])
        base = self.ws.data_ptr()
        return [q.value - base for q in ptrs]

    def q_columns(self):
        """The CG columns Q e_{a_t} of the picks expanded to the grid: [kmax, N] (zero outside
        each box; rows of picks without a column are zero)."""
        qo, bo, _, so, _, _ = self._buffers()
        b0, b1, b2 = self.box
        bv = b0 * b1 * b2
        cols = self.ws[qo: qo + 8 * self.nslots * bv].view(torch.float64).view(self.nslots, b0, b1,
                                                                               b2)
        lo = self.ws[bo: bo + 8 * 3 * self.nslots].view(torch.int64).view(self.nslots, 3).cpu()
        slots = self.ws[so: so + 4 * self.kmax].view(torch.int32).cpu()
        picks = self.picks.cpu()
        full = torch.zeros((self.kmax,) + self.p.shape, dtype=torch.float64, device=self.ws.device)
        for t in range(self.kmax):
            s = int(slots[t])
            if int(picks[t]) < 0 or not 0 <= s < self.nslots:
                continue
            l0, l1, l2 = (int(v) for v in lo[s])
            if not all(0 <= l <= sh - b for l, sh, b in zip((l0, l1, l2), self.p.shape, self.box)):
                continue  # no column for this pick (the last one of the selected-inverse form)
            full[t, l0:l0 + b0, l1:l1 + b1, l2:l2 + b2] = cols[s]
        return full.view(self.kmax, -1)

    def cg_iterations_used(self):
        """Iterations the last CG solve took (the full budget if it did not stop early)."""
        co = self._buffers()[2]
        st = self.ws[co: co + 8].view(torch.int32)
        return int(st[1]) if int(st[0]) else self.cg_iters


def allgather_slabs(vec, group=None):
    """Every rank computed vec[r chunk: (r + 1) chunk] (chunk = ceil(n / world)); afterwards
    every rank holds all of it (one all-gather; gloo groups stage through the host)."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = vec.numel()
    chunk = -(-n // world)
    full = torch.zeros(chunk * world, dtype=vec.dtype, device=vec.device)
    mine = torch.zeros(chunk, dtype=vec.dtype, device=vec.device)
    lo, hi = min(rank * chunk, n), min((rank + 1) * chunk, n)
    mine[:hi - lo] = vec[lo:hi]
    if dist.get_backend(group) == "gloo" and vec.is_cuda:
        out = full.cpu()
        dist.all_gather_into_tensor(out, mine.cpu(), group=group)
        full.copy_(out)
    else:
        dist.all_gather_into_tensor(full, mine, group=group)
    vec.copy_(full[:n])
    return 8 * chunk * (world - 1)


def slab_of(n, world, rank):
    chunk = -(-n // world)
    return min(rank * chunk, n), min((rank + 1) * chunk, n)


class ExactTaperPlacement:
    """One C4 problem end to end (device-resident).  method:
      "bounds": upper bounds of diag(Q) from K-step CG per candidate (sharded over the ranks of
                `group`, one all-gather) and the bounded-lazy rounds (replicated on every rank);
      "selinv": diag(Q) from the multifrontal selected inverse (sharded subtree-to-subcube) and
                the plain rounds — the only form that also yields delta_cached_iters;
      "auto":   "bounds" unless snapshots are asked for or the spectrum bounds cannot bracket."""

    def __init__(self, X, shape, k, cutoff, beta=4.0, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
                 jitter=TF_JITTER, threshold=TF_SMALL, leaf=512, device=None, group=None,
                 method="auto"):
        if method not in ("auto", "bounds", "selinv"):
            raise ValueError(f"method must be auto / bounds / selinv, got {method!r}")
        self.prob = TaperProblem(X, shape, beta, kind, amp, ls, diag_shift, jitter, threshold,
                                 device)
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.comm = FrontComm(group) if self.world > 1 else None
        self.leaf = leaf
        self._sel = None
        self.greedy = ExactWindowGreedy(self.prob, k, cutoff)
        self.k = int(k)
        self.method = method
        self.used = None
        self.exchanged_bytes = 0
        self.qdiag = torch.empty(self.prob.n, dtype=torch.float64, device=self.prob.device)

    @property
    def sel(self):
        if self._sel is None:
            self._sel = FrontalSelectedInverse(self.prob, self.leaf, comm=self.comm)
        return self._sel

    def run(self, snapshots=None):
        if self.method != "selinv" and snapshots is None:
            c0, c1 = slab_of(self.prob.n, self.world, self.rank)
            b = self.greedy.bound_qdiag(self.qdiag, c0, c1)
            if b is not None:
                if self.world > 1:
                    self.exchanged_bytes = allgather_slabs(self.qdiag, self.group)
                self.used = "bounds"
                return self.greedy.run_bounded(self.qdiag, self.k)
            if self.method == "bounds":
                raise ValueError("the Gershgorin bounds of Sigma + eps I do not bracket Q_yy "
                                 "(not diagonally dominant): use method='selinv'")
        self.used = "selinv"
        self.sel.run(out=self.qdiag)
        return self.greedy.run(self.qdiag, self.k, snapshots)

    def check(self):
        if self.used == "selinv":
            self.sel.check()


def tapered_placement_algorithm_3(X, k, COVER_spatial, cutoff, beta=4.0, kernel="eq", amp=1.0,
                                  ls=1.0, diag_shift=0.0, snapshots=False, leaf=512, group=None,
                                  method="auto"):
    """snippets_a3.sparse_placement_algorithm_3(cov_vv, k, COVER_spatial, cutoff) for the tapered
    covariance of the grid points X (C order, COVER_spatial = (I0, I1, I2)), exact, without the
    dense cov_vv.  -> (picks as a list of np.int64 in selection order, the pick deltas,
    delta_cached_iters [N, k] or None)."""
    shape = tuple(int(c) for c in COVER_spatial[:3])
    N = shape[0] * shape[1] * shape[2]
    if len(X) != N:                                         # snippets_a3.py:51 tf.Assert
        raise ValueError(f"assertion failed: N = {len(X)} != prod(COVER_spatial) = {N}")
    run = ExactTaperPlacement(X, shape, k, cutoff, beta, kernel, amp, ls, diag_shift, leaf=leaf,
                              group=group, method=method)
    snaps = [] if snapshots else None
    picks = run.run(snaps).cpu().numpy()
    run.check()
    dci = torch.stack(snaps, 1).cpu().numpy() if snapshots else None
    return [np.int64(a) for a in picks], run.greedy.pick_delta[:k].cpu().numpy(), dci


__all__ = ["TaperProblem", "HipFrontalOps", "FrontComm", "FrontalSelectedInverse",
           "ExactWindowGreedy", "ExactTaperPlacement", "tapered_placement_algorithm_3",
           "reach_table", "bound_steps", "allgather_slabs", "slab_of"]

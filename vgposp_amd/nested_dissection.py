"""Symbolic analysis of the exact config-C4 path: geometric nested dissection of the tapered
covariance of an I0 x I1 x I2 grid.

The beta-decay taper of ``main_architecture_2_sampledistribution.py:355-421`` makes cov_vv zero
beyond a fixed index stencil (the 6 face neighbours at the reference's ``BETA_val = 4``), so the
covariance is a sparse SPD matrix with the sparsity of a 3-D stencil of radius r (the largest
offset component).  Algorithm 3 on it (``snippets_a3.py:43-364``) needs, exactly:

* diag((Sigma + eps I)^-1) for every candidate (the round-0 denominators, ``snippets_a3.py:77-124``
  with ``tf_denominator`` = ``tf_nominator`` over V \\ {y}, ``snippets_a2.py:138-218``);
* one column (Sigma + eps I)^-1 e_a per pick (the later rounds' denominators over V \\ A).

The first is a selected inversion.  This module plans it: the grid is cut recursively by slabs of
thickness r (a slab of that width disconnects the two sides for any stencil of radius r), giving an
elimination tree of *fronts*.  A front is one separator slab (or a leaf box) with

* P: its pivots (the slab's nodes, C order);
* U: the halo of the front's whole box, i.e. the nodes outside the box within the stencil of a
  node inside it.  Every such node lies in an ancestor's slab (checked), and after the box's
  interior is eliminated U is exactly the set of later nodes coupled to P, so the front is the
  dense (|P| + |U|)^2 matrix of a multifrontal Cholesky.

Fronts are grouped by tree depth (and leaf / separator) into *groups* that are processed as one
batch: every front of a group is padded to the group's (p, u) (padded pivots get an identity
diagonal, padded U rows are zero), so the dense work of a group is a handful of strided batched
fp64 GEMM / Cholesky launches.

Everything here is host-side numpy, computed once per (shape, offsets, leaf) and cached.
"""
from __future__ import annotations

import functools
from dataclasses import dataclass, field

import numpy as np


def _round_up(x, m):
    return ((int(x) + m - 1) // m) * m


@dataclass
class Front:
    lo: tuple            # the front's whole box [lo, hi) (its subtree's nodes)
    hi: tuple
    depth: int
    leaf: bool
    parent: int = -1     # index into FrontalTree.fronts (postorder), -1 for a root
    children: list = field(default_factory=list)
    piv: np.ndarray = None   # int64 global indices, C order
    U: np.ndarray = None     # int64 global indices, sorted
    group: int = -1
    slot: int = -1
    sibling: int = 0     # index among its parent's children (0 or 1)


@dataclass
class Group:
    depth: int
    leaf: bool
    fronts: list         # front indices (postorder ids)
    p: int = 0           # padded pivot count
    u: int = 0           # padded boundary count
    p_max: int = 0
    u_max: int = 0
    piv: np.ndarray = None    # int32 [nf, p], -1 padding
    U: np.ndarray = None      # int32 [nf, u], sorted; padded with the grid size n
    ulen: np.ndarray = None   # int32 [nf]
    pmap: np.ndarray = None   # int32 [nf, u]: position of U[f][k] in the parent's front, -1 pad
    parent_group: np.ndarray = None  # int32 [nf]
    parent_slot: np.ndarray = None   # int32 [nf]
    sibling: np.ndarray = None       # int32 [nf]
    order: np.ndarray = None         # int32 [nf] postorder id of each front
    level: int = 0                   # index into FrontalTree.levels
    off: tuple = (0, 0, 0)           # element offsets of this group's PP / UP / UU in its level
    # the parent front of every front, as offsets into the parent LEVEL's PP / UP / UU buffers and
    # its (p, u): int64 [nf, 3] and int32 [nf, 2] (-1 for a root)
    par_off: np.ndarray = None
    par_dim: np.ndarray = None

    @property
    def nf(self):
        return len(self.fronts)

    @property
    def F(self):
        return self.p + self.u


def stencil_radius(offsets):
    offsets = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
    return int(np.abs(offsets).max()) if len(offsets) else 0


class FrontalTree:
    """The nested-dissection elimination tree of a grid with stencil ``offsets`` ([m-1, 3], the
    taper support without 0; symmetric)."""

    def __init__(self, shape, offsets, leaf=512, pad=16):
        self.shape = tuple(int(s) for s in shape)
        I0, I1, I2 = self.shape
        self.n = I0 * I1 * I2
        self.offsets = np.asarray(offsets, dtype=np.int64).reshape(-1, 3)
        self.r = max(stencil_radius(self.offsets), 1)
        self.leaf_max = int(leaf)
        self.pad = int(pad)
        self.fronts: list[Front] = []
        self._build([0, 0, 0], list(self.shape), 0, -1)
        self._index()
        self._groups()

    # ------------------------------------------------------------------ tree
    def _nodes(self, lo, hi):
        I0, I1, I2 = self.shape
        a = [np.arange(l, h, dtype=np.int64) for l, h in zip(lo, hi)]
        return ((a[0][:, None, None] * I1 + a[1][None, :, None]) * I2 + a[2][None, None, :]).ravel()

    def _build(self, lo, hi, depth, parent):
        """Append the subtree of box [lo, hi) in postorder; returns its root's id."""
        ext = [h - l for l, h in zip(lo, hi)]
        vol = ext[0] * ext[1] * ext[2]
        r = self.r
        ax = int(np.argmax(ext))
        if vol <= self.leaf_max or ext[ax] < r + 2:
            f = Front(tuple(lo), tuple(hi), depth, True, parent)
            f.piv = self._nodes(lo, hi)
            self.fronts.append(f)
            return len(self.fronts) - 1
        mid = lo[ax] + (ext[ax] - r) // 2
        kids = []
        l2 = list(hi)
        l2[ax] = mid
        h2 = list(lo)
        h2[ax] = mid + r
        placeholder = len(self.fronts)  # children are appended first (postorder)
        for clo, chi in ((list(lo), l2), (h2, list(hi))):
            if all(h > l for l, h in zip(clo, chi)):
                kids.append(self._build(clo, chi, depth + 1, -2))
        slo, shi = list(lo), list(hi)
        slo[ax], shi[ax] = mid, mid + r
        f = Front(tuple(lo), tuple(hi), depth, False, parent, kids)
        f.piv = self._nodes(slo, shi)
        self.fronts.append(f)
        me = len(self.fronts) - 1
        for s, c in enumerate(kids):
            self.fronts[c].parent = me
            self.fronts[c].sibling = s
        del placeholder
        return me

    def _halo(self, f):
        lo = np.array(f.lo)
        hi = np.array(f.hi)
        r = self.r
        shp = np.array(self.shape)
        elo = np.maximum(lo - r, 0)
        ehi = np.minimum(hi + r, shp)
        a = [np.arange(l, h) for l, h in zip(elo, ehi)]
        g = np.stack(np.meshgrid(*a, indexing="ij"), -1).reshape(-1, 3)
        inside = np.all((g >= lo) & (g < hi), axis=1)
        g = g[~inside]
        if len(g) == 0 or len(self.offsets) == 0:
            return np.zeros(0, dtype=np.int64)
        adj = np.zeros(len(g), dtype=bool)
        for o in self.offsets:
            q = g + o
            adj |= np.all((q >= lo) & (q < hi), axis=1)
        g = g[adj]
        I0, I1, I2 = self.shape
        return np.sort((g[:, 0] * I1 + g[:, 1]) * I2 + g[:, 2])

    def _index(self):
        n = self.n
        self.owner = np.full(n, -1, dtype=np.int64)
        self.owner_pos = np.full(n, -1, dtype=np.int64)
        for i, f in enumerate(self.fronts):
            if np.any(self.owner[f.piv] >= 0):
                raise AssertionError("nested dissection assigned a node twice")
            self.owner[f.piv] = i
            self.owner_pos[f.piv] = np.arange(len(f.piv))
        if np.any(self.owner < 0):
            raise AssertionError("nested dissection missed nodes")
        for i, f in enumerate(self.fronts):
            f.U = self._halo(f)
            # every halo node must belong to an ancestor's separator (the property the
            # multifrontal assembly relies on)
            anc = set()
            a = f.parent
            while a >= 0:
                anc.add(a)
                a = self.fronts[a].parent
            own = np.unique(self.owner[f.U])
            if not set(own.tolist()) <= anc:
                raise AssertionError(f"front {i}: halo outside its ancestors")

    def _groups(self):
        """The single-rank layout (every front on this process): ``self.groups`` / ``levels``."""
        lay = FrontalLayout(self, world=1, rank=0)
        self.groups, self.levels = lay.groups, lay.levels
        for gi, g in enumerate(self.groups):
            for s, i in enumerate(g.fronts):
                self.fronts[i].group = gi
                self.fronts[i].slot = s

    def owners(self, world):
        """Subtree-to-subcube mapping of the fronts onto `world` ranks: a front owning ranks
        [lo, hi) gives its first child [lo, mid) and its second [mid, hi); the front itself runs on
        rank lo.  With world = 2^d every front of depth >= d is private to one rank and the top
        2^d - 1 fronts sit on the ranks that hold their first child's subtree."""
        own = np.zeros(len(self.fronts), dtype=np.int64)
        root = len(self.fronts) - 1

        def go(i, lo, hi):
            own[i] = lo
            kids = self.fronts[i].children
            if len(kids) == 2 and hi - lo > 1:
                mid = (lo + hi + 1) // 2
                go(kids[0], lo, mid)
                go(kids[1], mid, hi)
            else:
                for c in kids:
                    go(c, lo, hi)
        go(root, 0, int(world))
        return own

    def layout(self, world=1, rank=0):
        return FrontalLayout(self, world, rank)

    # ------------------------------------------------------------------ summaries
    def flops(self, padded=True):
        """Algorithmic fp64 flops of factor + selected inverse: per front p^3 + 3 p^2 u + 3 p u^2
        (potrf p^3/3, trtri p^3/3, L_UP and W products 2 p^2 u, SYRK p u^2; selected inverse:
        M^T M p^3/3, Q_UU W 2 p u^2, W^T T p^2 u)."""
        tot = 0.0
        for g in self.groups:
            if padded:
                p, u, nf = float(g.p), float(g.u), g.nf
                tot += nf * (p ** 3 + 3 * p * p * u + 3 * p * u * u)
            else:
                for i in g.fronts:
                    p, u = float(len(self.fronts[i].piv)), float(len(self.fronts[i].U))
                    tot += p ** 3 + 3 * p * p * u + 3 * p * u * u
        return tot

    def storage_bytes(self):
        """Factor storage (M_PP and W of every front, padded)."""
        return sum(8 * g.nf * (g.p * g.p + g.u * g.p) for g in self.groups)

    def summary(self):
        return [{"depth": g.depth, "leaf": g.leaf, "fronts": g.nf, "p": g.p, "u": g.u,
                 "p_max": g.p_max, "u_max": g.u_max} for g in self.groups]

    def level_bytes(self):
        """Bytes of the PP / UP / UU buffers of every level."""
        return [[8 * v for v in lvl["size"]] for lvl in self.levels]


@functools.lru_cache(maxsize=8)
def _cached(shape, offs_key, leaf, pad):
    offs = np.array(offs_key, dtype=np.int64).reshape(-1, 3)
    return FrontalTree(shape, offs, leaf, pad)


def frontal_tree(shape, offsets, leaf=512, pad=16):
    """Cached FrontalTree for (shape, offsets, leaf, pad)."""
    offs = tuple(int(v) for v in np.asarray(offsets, dtype=np.int64).reshape(-1))
    return _cached(tuple(int(s) for s in shape), offs, int(leaf), int(pad))




class FrontalLayout:
    """The fronts one rank factors, cut into levels (tree depths, deepest first) and groups of
    similar padded size, each level stored as three flat buffers (PP, UP, UU) holding its groups at
    static offsets.  A child whose parent is on the same rank addresses the parent front by its
    offsets into the parent level's buffers (Group.par_off / par_dim); a child whose parent is on
    another rank is a *transfer*: its update (factor phase) goes to the parent's rank as an
    [ulen, ulen] block, and the parent's rank sends back that child's Q_UU (selected inverse).

      send_update[li]  : (group, slot, front, dest) after level li is factored
      recv_update[li]  : RemoteChild records extend-added into level li before it is factored
      send_q[li]       : RemoteChild records gathered from level li's Q and sent after it
      recv_q[li]       : (group, slot, front, src) whose Q_UU arrives before level li's selinv
    """

    tol = 0.1

    def __init__(self, tree, world=1, rank=0):
        self.tree = tree
        self.world, self.rank = int(world), int(rank)
        T = tree
        self.owner = T.owners(world) if world > 1 else np.zeros(len(T.fronts), dtype=np.int64)
        mine = [i for i in range(len(T.fronts)) if self.owner[i] == rank]
        maxd = max(f.depth for f in T.fronts)
        bydepth = {d: [] for d in range(maxd, -1, -1)}
        for i in mine:
            bydepth[T.fronts[i].depth].append(i)
        self.groups: list[Group] = []
        self.levels = []
        self.where = {}          # front -> (group, slot)
        self.depth_level = {}
        for d in range(maxd, -1, -1):
            ids = sorted(bydepth[d], key=lambda i: (-_round_up(max(len(T.fronts[i].piv), 1),
                                                               T.pad), -len(T.fronts[i].U), i))
            lvl = {"depth": d, "groups": [], "size": [0, 0, 0]}
            self.depth_level[d] = len(self.levels)
            self._cut(ids, d, lvl)
            self.levels.append(lvl)
        L = len(self.levels)
        self.send_update = [[] for _ in range(L)]
        self.recv_update = [[] for _ in range(L)]
        self.send_q = [[] for _ in range(L)]
        self.recv_q = [[] for _ in range(L)]
        for gi, g in enumerate(self.groups):
            self._fill(gi, g)
        # children of this rank's fronts that live on other ranks
        for i in mine:
            for c in T.fronts[i].children:
                if self.owner[c] != rank:
                    rc = self._remote_child(c, i)
                    li = self.depth_level[T.fronts[i].depth]
                    self.recv_update[li].append(rc)
                    self.send_q[li].append(rc)
        for li in range(L):
            self.recv_update[li].sort(key=lambda r: r.front)
            self.send_q[li].sort(key=lambda r: r.front)
            self.send_update[li].sort(key=lambda t: t[2])
            self.recv_q[li].sort(key=lambda t: t[2])

    def _cut(self, ids, d, lvl):
        T = self.tree

        def fl(p, u):
            return p ** 3 + 3.0 * p * p * u + 3.0 * p * u * u

        def dims(i):
            f = T.fronts[i]
            return (_round_up(max(len(f.piv), 1), T.pad), _round_up(len(f.U), T.pad))
        cur = []
        P = U = 0
        worst = float("inf")
        for i in ids:
            pf, uf = dims(i)
            if cur:
                P2, U2, w2 = max(P, pf), max(U, uf), min(worst, fl(pf, uf))
                if fl(P2, U2) > (1 + self.tol) * w2:
                    self._new_group(d, cur, lvl)
                    cur = []
            if not cur:
                P, U, worst = pf, uf, fl(pf, uf)
            else:
                P, U, worst = max(P, pf), max(U, uf), min(worst, fl(pf, uf))
            cur.append(i)
        if cur:
            self._new_group(d, cur, lvl)

    def _new_group(self, depth, ids, lvl):
        T = self.tree
        gi = len(self.groups)
        g = Group(depth, all(T.fronts[i].leaf for i in ids), list(ids))
        g.p_max = max(len(T.fronts[i].piv) for i in ids)
        g.u_max = max(len(T.fronts[i].U) for i in ids)
        g.p = _round_up(max(g.p_max, 1), T.pad)
        g.u = _round_up(g.u_max, T.pad) if g.u_max else 0
        g.level = len(self.levels)
        sz = lvl["size"]
        g.off = (sz[0], sz[1], sz[2])
        sz[0] += g.nf * g.p * g.p
        sz[1] += g.nf * g.u * g.p
        sz[2] += g.nf * g.u * g.u
        for s, i in enumerate(ids):
            self.where[i] = (gi, s)
        self.groups.append(g)
        lvl["groups"].append(gi)

    def _pmap(self, c, parent):
        """Positions of child c's boundary in its parent's front (this rank's layout)."""
        T = self.tree
        f, par = T.fronts[c], T.fronts[parent]
        pg = self.groups[self.where[parent][0]]
        own = T.owner[f.U]
        pos = np.where(own == parent, T.owner_pos[f.U], -1)
        inU = own != parent
        k = np.searchsorted(par.U, f.U[inU])
        if np.any(k >= len(par.U)) or np.any(par.U[np.minimum(k, len(par.U) - 1)] != f.U[inU]):
            raise AssertionError("child boundary not inside the parent's front")
        pos[inU] = pg.p + k
        return pos

    def _par(self, parent):
        pgi, ps = self.where[parent]
        pg = self.groups[pgi]
        return ((pg.off[0] + ps * pg.p * pg.p, pg.off[1] + ps * pg.u * pg.p,
                 pg.off[2] + ps * pg.u * pg.u), (pg.p, pg.u))

    def _fill(self, gi, g):
        T = self.tree
        nf = g.nf
        g.piv = np.full((nf, g.p), -1, dtype=np.int32)
        g.U = np.full((nf, max(g.u, 1)), T.n, dtype=np.int32)
        g.ulen = np.zeros(nf, dtype=np.int32)
        g.pmap = np.full((nf, max(g.u, 1)), -1, dtype=np.int32)
        g.parent_group = np.full(nf, -1, dtype=np.int32)
        g.parent_slot = np.full(nf, -1, dtype=np.int32)
        g.sibling = np.zeros(nf, dtype=np.int32)
        g.order = np.asarray(g.fronts, dtype=np.int32)
        g.par_off = np.full((nf, 3), -1, dtype=np.int64)
        g.par_dim = np.full((nf, 2), -1, dtype=np.int32)
        li = g.level
        for s, i in enumerate(g.fronts):
            f = T.fronts[i]
            g.piv[s, :len(f.piv)] = f.piv
            g.U[s, :len(f.U)] = f.U
            g.ulen[s] = len(f.U)
            g.sibling[s] = f.sibling
            if f.parent < 0:
                continue
            if self.owner[f.parent] != self.rank:
                # the parent is elsewhere: sibling -1 keeps this front out of the local
                # extend-add launches; its update and Q_UU travel as [ulen, ulen] blocks
                g.sibling[s] = -1
                self.send_update[li].append((gi, s, i, int(self.owner[f.parent])))
                self.recv_q[li].append((gi, s, i, int(self.owner[f.parent])))
                continue
            pgi, ps = self.where[f.parent]
            g.parent_group[s] = pgi
            g.parent_slot[s] = ps
            off, dim = self._par(f.parent)
            g.par_off[s] = off
            g.par_dim[s] = dim
            g.pmap[s, :len(f.U)] = self._pmap(i, f.parent)

    def _remote_child(self, c, parent):
        T = self.tree
        f = T.fronts[c]
        off, dim = self._par(parent)
        return RemoteChild(front=c, parent=parent, src=int(self.owner[c]), ulen=len(f.U),
                           sibling=f.sibling, pmap=self._pmap(c, parent).astype(np.int32),
                           par_off=np.asarray(off, dtype=np.int64),
                           par_dim=np.asarray(dim, dtype=np.int32))

    def flops(self):
        return sum(g.nf * (float(g.p) ** 3 + 3.0 * g.p * g.p * g.u + 3.0 * g.p * g.u * g.u)
                   for g in self.groups)


@dataclass
class RemoteChild:
    front: int
    parent: int
    src: int
    ulen: int
    sibling: int
    pmap: np.ndarray
    par_off: np.ndarray
    par_dim: np.ndarray


__all__ = ["FrontalTree", "FrontalLayout", "RemoteChild", "Front", "Group", "frontal_tree",
           "stencil_radius"]

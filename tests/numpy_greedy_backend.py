"""TEST INFRASTRUCTURE: a numpy implementation of the libvgposp greedy phases
(vgposp_greedy_init / _update / _select semantics) so the multi-rank orchestration of
vgposp_amd.sharded_placement can be exercised with gloo on CPU.  Never used by the product."""
import numpy as np
import torch

EPS = 1e-8


def _keymax(vals, idx):
    """(value desc, index asc) arg-max over candidate indices idx."""
    if len(idx) == 0:
        return -1
    v = vals[idx]
    best = np.max(v)
    return int(idx[np.flatnonzero(v == best)[0]])


def split_point(n, nb=128):
    """vgposp_potrf_split: the recursion's split (potrf.hip split_point)."""
    return nb * (((n + nb - 1) // nb) // 2) if n > nb else 0


class NumpyCholeskyOps:
    """vgposp_potrf_block / _panel / _trailing / pack_rows on a numpy matrix (lower triangle
    factored in place, the strictly upper triangle never written), for DistCholesky on gloo."""

    def __init__(self, A):
        self.A = A
        self.n = A.shape[0]
        self.device = torch.device("cpu")
        self.failed = False  # a leading minor was not positive definite (device `info` != 0)

    def split(self, n):
        return split_point(n)

    def block(self, col0, nb):
        s = slice(col0, col0 + nb)
        B = np.tril(self.A[s, s])
        try:
            L = np.linalg.cholesky(B + np.tril(B, -1).T)
        except np.linalg.LinAlgError:
            self.failed = True
            L = np.eye(nb)
        low = np.tril(np.ones((nb, nb), dtype=bool))
        blk = self.A[s, s]
        blk[low] = L[low]

    def panel(self, col0, nsub, r0, r1):
        n1 = split_point(nsub)
        L11 = np.tril(self.A[col0:col0 + n1, col0:col0 + n1])
        rows = slice(col0 + n1 + r0, col0 + n1 + r1)
        cols = slice(col0, col0 + n1)
        self.A[rows, cols] = np.linalg.solve(L11, self.A[rows, cols].T).T

    def trailing(self, col0, nsub, b0, b1):
        n1 = split_point(nsub)
        base = col0 + n1
        L21 = self.A[base:col0 + nsub, col0:base]
        upd = L21[b0:b1] @ L21[:b1].T
        for i in range(b1 - b0):
            r = b0 + i
            self.A[base + r, base:base + r + 1] -= upd[i, :r + 1]

    def pack_elems(self, r0, r1, c0, c1, lower):
        m = r1 - r0
        if m <= 0:
            return 0
        return m * (r0 + 1 - c0) + m * (m - 1) // 2 if lower else m * (c1 - c0)

    def pack(self, r0, r1, c0, c1, lower, buf, unpack):
        b = buf.numpy()
        off = 0
        for r in range(r0, r1):
            e = r + 1 if lower else c1
            w = e - c0
            if unpack:
                self.A[r, c0:e] = b[off:off + w]
            else:
                b[off:off + w] = self.A[r, c0:e]
            off += w


class NumpyGreedyBackend:
    def __init__(self, Sigma, kmax, jitter=0.0):
        self.S = np.array(Sigma, dtype=np.float64)
        self.n = self.S.shape[0]
        self.kmax = kmax
        self.eps = float(jitter)
        self._delta = torch.zeros(self.n, dtype=torch.float64)
        self._piv = torch.zeros(2 + 2 * kmax, dtype=torch.float64)
        self.ok = True
        self.L = None

    def init(self):
        try:
            L = np.linalg.cholesky(self.S + self.eps * np.eye(self.n))
            self.ok = True
        except np.linalg.LinAlgError:
            L = np.eye(self.n)
            self.ok = False
        self.L = L
        self.M = np.linalg.inv(L)
        self.sdiag = np.diag(self.S).copy()
        self.colsq = np.sum(self.M ** 2, axis=0)
        n, k = self.n, self.kmax
        self.nom = np.zeros(n)
        self.prec = np.zeros(n)
        self.W = np.zeros((k, n))
        self.V = np.zeros((k, n))
        self._delta.zero_()
        self._piv.zero_()
        self.cache = np.full(n, np.inf)
        self.sel = np.zeros(n, dtype=bool)
        self.selected = []
        self.sel_delta = []

    def prepare(self):
        self.F = self.S + self.eps * np.eye(self.n)

    def chol_ops(self):
        self._ops = NumpyCholeskyOps(self.F)
        return self._ops

    def finish_slab(self, c0, c1):
        """After DistCholesky on chol_ops(): the partitioned state from the shared factor."""
        L = np.tril(self.F)
        self.init()
        self.ok = bool(not self._ops.failed and np.all(np.isfinite(L)) and np.all(np.diag(L) > 0))
        self.L = L
        self.M = np.linalg.inv(L) if self.ok else np.eye(self.n)
        self.colsq = np.sum(self.M ** 2, axis=0)
        self._mask_slab(c0, c1)

    def init_slab(self, c0, c1):
        """Partitioned inverse: only columns [c0, c1) of L^-1 exist on this rank (NaN elsewhere, so
        any use of another rank's column shows up)."""
        self.init()
        self._mask_slab(c0, c1)

    def _mask_slab(self, c0, c1):
        own = np.zeros(self.n, dtype=bool)
        own[c0:c1] = True
        self.M[:, ~own] = np.nan
        self.colsq = np.where(own, self.colsq, np.nan)
        self._xcol = torch.zeros(self.n, dtype=torch.float64)

    def extract(self, rnd, own0, own1):
        a = self.selected[rnd - 1]
        x = self._xcol.numpy()
        x[:] = self.M[:, a] if own0 <= a < own1 else 0.0

    def xcol(self):
        return self._xcol

    def update(self, rnd, c0, c1, extract=True):
        idx = np.arange(c0, c1)
        if rnd == 0:
            self.prec[idx] = self.colsq[idx]
            self.nom[idx] = self.sdiag[idx]
        else:
            a, t1 = self.selected[rnd - 1], rnd - 1
            piv = self._piv.numpy()
            xa = self.M[:, a] if extract else self._xcol.numpy()
            q = self.M[:, idx].T @ xa
            s = self.S[idx, a].copy()
            s -= piv[2:2 + t1] @ self.W[:t1][:, idx]
            q -= piv[2 + t1:2 + 2 * t1] @ self.V[:t1][:, idx]
            noma = piv[0] + self.eps
            w = s / np.sqrt(noma) if noma > 0 else 0 * s
            v = q / np.sqrt(piv[1]) if piv[1] > 0 else 0 * q
            self.W[t1, idx] = w
            self.V[t1, idx] = v
            self.nom[idx] -= w * w
            self.prec[idx] -= v * v
        d = self._delta.numpy()
        for i in idx:
            if self.sel[i]:
                continue
            den = 1.0 / self.prec[i] - self.eps
            d[i] = 0.0 if (abs(den) < EPS or abs(self.nom[i]) < EPS) else self.nom[i] / den

    def select(self, rnd, lazy, c0, c1):
        d = self._delta.numpy()
        cand = np.flatnonzero(~self.sel)
        fy = _keymax(d, cand)
        if not lazy:
            y = fy
        else:
            fresh = np.zeros(self.n, dtype=bool)
            for i in cand:
                c = self.cache[i]
                if c > d[fy] or (c == d[fy] and i < fy):
                    self.cache[i] = d[i]
                    fresh[i] = True
            while True:
                y = _keymax(self.cache, cand)
                if fresh[y]:
                    break
                self.cache[y] = d[y]
                fresh[y] = True
        self.selected.append(y)
        self.sel_delta.append(d[y])
        self.sel[y] = True
        p = self._piv.numpy()
        p[:] = 0.0
        if c0 <= y < c1:
            p[0], p[1] = self.nom[y], self.prec[y]
            p[2:2 + rnd] = self.W[:rnd, y]
            p[2 + rnd:2 + 2 * rnd] = self.V[:rnd, y]

    def delta(self):
        return self._delta

    def piv(self):
        return self._piv

    def result(self):
        return [np.int64(s) for s in self.selected], np.array(self.sel_delta), None

    def snapshot_diag(self):
        pass  # init() reads diag(S) itself

    # singular cov_vv (ShardedGreedyPlacement.run's jitter retry)
    def factor_ok(self, c0, c1, partitioned, check_pivots):
        if not self.ok:
            return False
        if not check_pivots:
            return True
        lii = np.diag(self.L)
        return bool(np.min(lii * lii / self.sdiag) >= 100 * np.finfo(np.float64).eps * self.n)

    def diag_scale(self):
        return abs(float(np.mean(np.diag(self.S)))) or 1.0

    def rejitter(self, eps):
        self.__init__(self.S, self.kmax, jitter=eps)

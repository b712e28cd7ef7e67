"""CPU (numpy) restatement of the multifrontal selected inversion that vgposp_amd.sparse_placement
runs on the GPU, group by group with the same padded batches and index maps.  Test
infrastructure: it checks the symbolic analysis (vgposp_amd.nested_dissection) and the batched
formulation on CPU against a dense inverse, without a GPU."""
from __future__ import annotations

import numpy as np


def tapered_entry_matrix(X, shape, offsets, tau, kern, shift, jitter):
    """Dense (Sigma + jitter I) of the taper on small grids: s(u, v) = tau[|i_u - i_v|^2]
    (K(x_u, x_v) + shift [u == v])."""
    I0, I1, I2 = shape
    n = I0 * I1 * I2
    idx = np.stack(np.unravel_index(np.arange(n), shape), 1)
    d2 = ((idx[:, None, :] - idx[None, :, :]) ** 2).sum(-1)
    t = np.where(d2 < len(tau), tau[np.minimum(d2, len(tau) - 1)], 0.0)
    r2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    S = t * (kern(r2) + shift * np.eye(n))
    return S + jitter * np.eye(n)


def selected_inverse_diag(tree, C):
    """diag(C^-1) through the frontal tree, mirroring the device algorithm:
    factor (bottom-up): F_PP = L L^T, M = L^-1, L_UP = F_UP M^T, F_UU -= L_UP L_UP^T, W = L_UP M;
    selected inverse (top-down): Q_UU gathered from the parent's Q front, T = -Q_UU W,
    Q_PP = M^T M - W^T T, Q_UP = T."""
    G = tree.groups
    PP, UP, UU = [], [], []
    for g in G:
        PP.append(np.zeros((g.nf, g.p, g.p)))
        UP.append(np.zeros((g.nf, g.u, g.p)))
        UU.append(np.zeros((g.nf, g.u, g.u)))

    def put(gi, s, a, b, v, add):
        """lower-triangle element (max, min) of front (gi, s) in [P | U] positions."""
        r, c = max(a, b), min(a, b)
        p = G[gi].p
        if r < p:
            tgt, i, j = PP[gi], r, c
        elif c < p:
            tgt, i, j = UP[gi], r - p, c
        else:
            tgt, i, j = UU[gi], r - p, c - p
        if add:
            tgt[s, i, j] += v
        else:
            tgt[s, i, j] = v

    def get(gi, s, a, b):
        r, c = max(a, b), min(a, b)
        p = G[gi].p
        if r < p:
            return PP[gi][s, r, c]
        if c < p:
            return UP[gi][s, r - p, c]
        return UU[gi][s, r - p, c - p]

    # ---- factor, deepest groups first
    for gi, g in enumerate(G):
        # assembly of the original entries: column j in P, rows in P (lower) or U
        for s in range(g.nf):
            piv = g.piv[s]
            U = g.U[s, :g.ulen[s]]
            pos = {int(v): k for k, v in enumerate(piv) if v >= 0}
            upos = {int(v): g.p + k for k, v in enumerate(U)}
            for pj, j in enumerate(piv):
                if j < 0:
                    PP[gi][s, pj, pj] = 1.0
                    continue
                nz = np.nonzero(C[:, j])[0]
                for i in nz:
                    if i in pos and pos[i] >= pj:
                        put(gi, s, pos[i], pj, C[i, j], False)
                    elif i in upos:
                        put(gi, s, upos[i], pj, C[i, j], False)
        # extend-add of the children's updates (children were factored before: deeper groups)
        for ci, cg in enumerate(G[:gi]):
            for s in range(cg.nf):
                if cg.parent_group[s] != gi:
                    continue
                ps = cg.parent_slot[s]
                m = cg.pmap[s]
                for a in range(cg.u):
                    if m[a] < 0:
                        continue
                    for b in range(a + 1):
                        if m[b] >= 0:
                            put(gi, ps, m[a], m[b], UU[ci][s, a, b], True)
        # dense partial factorization of every front of the group
        for s in range(g.nf):
            A = np.tril(PP[gi][s])
            L = np.linalg.cholesky(A + np.tril(A, -1).T)
            M = np.linalg.inv(L)
            Lup = UP[gi][s] @ M.T
            UU[gi][s] = np.tril(UU[gi][s] - Lup @ Lup.T)
            UP[gi][s] = Lup @ M
            PP[gi][s] = np.tril(M)
    # ---- selected inverse, root first
    diag = np.zeros(tree.n)
    for gi in range(len(G) - 1, -1, -1):
        g = G[gi]
        for s in range(g.nf):
            M = PP[gi][s]
            W = UP[gi][s]
            if g.u:
                pg, ps = g.parent_group[s], g.parent_slot[s]
                m = g.pmap[s]
                Q = np.zeros((g.u, g.u))
                for a in range(g.u):
                    for b in range(g.u):
                        if m[a] >= 0 and m[b] >= 0:
                            Q[a, b] = get(pg, ps, m[a], m[b])
                T = -Q @ W
                QPP = M.T @ M - W.T @ T
                UU[gi][s] = Q
                UP[gi][s] = T
            else:
                QPP = M.T @ M
            PP[gi][s] = np.tril(QPP)
            piv = g.piv[s]
            ok = piv >= 0
            diag[piv[ok]] = np.diag(QPP)[ok]
    return diag


__all__ = ["tapered_entry_matrix", "selected_inverse_diag"]

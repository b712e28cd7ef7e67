"""CPU restatement of the device operations of vgposp_amd.sparse_placement.HipFrontalOps (the
frontal.hip kernels), on torch CPU tensors with numpy arithmetic, so that the orchestration in
FrontalSelectedInverse — level buffers, extend-add / gather descriptors, and the multi-rank
transfers over gloo — runs and is checked on CPU.  Test infrastructure only."""
from __future__ import annotations

import numpy as np
import torch


def _lower_pos(r, c, p, u, off, PP, UP, UU):
    """(array, flat index) of lower-triangle element (max(r, c), min(r, c)) of a front."""
    a, b = max(r, c), min(r, c)
    if a < p:
        return PP, off[0] + a * p + b
    if b < p:
        return UP, off[1] + (a - p) * p + b
    return UU, off[2] + (a - p) * u + (b - p)


class TorchCpuFrontalOps:
    def __init__(self, C):
        """C: the dense (Sigma + jitter I) of a small grid (the entries the assembly reads)."""
        self.C = np.asarray(C, dtype=np.float64)

    def zeros(self, n):
        return torch.zeros(max(int(n), 1), dtype=torch.float64)

    def empty(self, n):
        return torch.zeros(max(int(n), 1), dtype=torch.float64)

    @staticmethod
    def at(buf, off):
        return None if buf is None else buf[int(off):]

    def ints(self, a, dtype=np.int32):
        return np.array(a, dtype=dtype)

    @staticmethod
    def block(buf, off, rows, ld, cols):
        return buf[int(off): int(off) + rows * ld].view(rows, ld)[:, :cols]

    def assemble(self, tree, g, d, PP, UP):
        pp, up = PP.numpy(), (UP.numpy() if UP is not None else None)
        owner = tree.owner
        for s in range(g.nf):
            ord_f = int(d["order"][s])
            U = d["U"][s, :d["ulen"][s]]
            for pj in range(g.p):
                j = int(d["piv"][s, pj])
                base = s * g.p * g.p
                if j < 0:
                    pp[base + pj * g.p + pj] = 1.0
                    continue
                for i in np.nonzero(self.C[:, j])[0]:
                    oi = owner[i]
                    if oi < ord_f:
                        continue
                    if oi == ord_f:
                        pi = tree.owner_pos[i]
                        if pi >= pj:
                            pp[base + pi * g.p + pj] = self.C[i, j]
                    else:
                        k = int(np.searchsorted(U, i))
                        up[s * g.u * g.p + k * g.p + pj] = self.C[i, j]

    def extend_add(self, UUc, uc, nfc, pmap, par_off, par_dim, sibl, sib, PP, UP, UU):
        src = UUc.numpy()
        arrs = (PP.numpy(), UP.numpy(), UU.numpy())
        for s in range(nfc):
            if sibl[s] != sib:
                continue
            p, u = int(par_dim[s][0]), int(par_dim[s][1])
            m = pmap[s]
            for a in range(uc):
                if m[a] < 0:
                    continue
                for b in range(a + 1):
                    if m[b] < 0:
                        continue
                    v = src[s * uc * uc + a * uc + b]
                    if v == 0.0:
                        continue
                    arr, idx = _lower_pos(int(m[a]), int(m[b]), p, u, par_off[s], *arrs)
                    arr[idx] += v

    def factor(self, PP, UP, UU, p, u, nf):
        pp = PP.numpy()
        up = UP.numpy() if UP is not None else None
        uu = UU.numpy() if UU is not None else None
        info = np.zeros(nf, dtype=np.int32)
        for s in range(nf):
            A = pp[s * p * p:(s + 1) * p * p].reshape(p, p)
            Al = np.tril(A)
            try:
                Lf = np.linalg.cholesky(Al + np.tril(Al, -1).T)
            except np.linalg.LinAlgError:
                info[s] = 1
                continue
            M = np.linalg.inv(Lf)
            A[:] = np.tril(M)
            if u:
                F = up[s * u * p:(s + 1) * u * p].reshape(u, p)
                Lup = F @ M.T
                B = uu[s * u * u:(s + 1) * u * u].reshape(u, u)
                B[:] = np.tril(B - Lup @ Lup.T)
                F[:] = Lup @ M
        return info

    def gather(self, QPP, QUP, QUU, pmap, par_off, par_dim, nfc, uc, out):
        arrs = (QPP.numpy(), QUP.numpy(), QUU.numpy())
        dst = out.numpy()
        for s in range(nfc):
            p, u = int(par_dim[s][0]), int(par_dim[s][1])
            m = pmap[s]
            for a in range(uc):
                for b in range(uc):
                    v = 0.0
                    if m[a] >= 0 and m[b] >= 0:
                        arr, idx = _lower_pos(int(m[a]), int(m[b]), p, u, par_off[s], *arrs)
                        v = arr[idx]
                    dst[s * uc * uc + a * uc + b] = v

    def selinv(self, M, W, QUU, p, u, nf, QPP, QUP):
        m, qpp = M.numpy(), QPP.numpy()
        for s in range(nf):
            Ms = np.tril(m[s * p * p:(s + 1) * p * p].reshape(p, p))
            Q = Ms.T @ Ms
            if u:
                Ws = W.numpy()[s * u * p:(s + 1) * u * p].reshape(u, p)
                Qu = QUU.numpy()[s * u * u:(s + 1) * u * u].reshape(u, u)
                T = -Qu @ Ws
                Q = Q - Ws.T @ T
                QUP.numpy()[s * u * p:(s + 1) * u * p] = T.reshape(-1)
            qpp[s * p * p:(s + 1) * p * p] = np.tril(Q).reshape(-1)

    def diag(self, QPP, p, nf, piv, out):
        q, o = QPP.numpy(), out.numpy()
        for s in range(nf):
            for k in range(p):
                j = piv[s, k]
                if j >= 0:
                    o[j] = q[s * p * p + k * p + k]

    def pack_lower(self, buf, off, ld, n):
        A = buf[int(off): int(off) + n * ld].view(n, ld)[:, :n].numpy()
        return torch.from_numpy(A[np.tril_indices(n)].copy())

    def unpack_lower(self, packed, buf, off, ld, n, symmetric):
        A = buf[int(off): int(off) + n * ld].view(n, ld)[:, :n].numpy()
        A[np.tril_indices(n)] = packed.numpy()
        if symmetric:
            iu = np.triu_indices(n, 1)
            A[iu] = A.T[iu]

    def empty_packed(self, n):
        return torch.zeros(n * (n + 1) // 2, dtype=torch.float64)

    @staticmethod
    def nonzero_info(info):
        bad = np.nonzero(info)[0]
        return (int(bad[0]), int(info[bad[0]])) if len(bad) else None

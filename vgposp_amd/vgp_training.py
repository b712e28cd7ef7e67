"""VGP training objective and its analytic gradient on MI355X.

The reference trains a variational GP (variational_Gaussian_process_example.py:51-102;
main_architecture_2_sampledistribution.py:223-265) with

    loc, scale = tfd.VariationalGaussianProcess.optimal_variational_posterior(
                     kernel, Z, X, y, noise)                           # full data, every step
    loss = vgp.variational_loss(y_batch, x_batch, kl_weight=B / N)     # minibatch
    tf.train.AdamOptimizer(0.01).minimize(loss)                        # amp, ls, noise, Z

and TF autodiff differentiates through both.  Here the forward pass and a hand-derived reverse
pass run as libvgposp kernels.  The derivation is restated in numpy in
``oracle/gp.py:vgp_training_loss_grads`` and checked there against finite differences.  The heavy
operations are:

* ``Kzx = K(Z, X)`` (M x N, HBM-write-bound assembly);
* ``P0 = Kzx Kzx^T`` (2 M^2 N flops, split-K fp64 MFMA GEMM);
* ``c = Kzx y`` (HBM-bound GEMV);
* the reverse ``Kzx_bar = (2 / noise) Sinv_bar Kzx + c_bar y^T`` (2 M^2 N flops);
* its kernel VJP (one HBM pass over Kzx_bar, ``vgposp_kernel_vjp``).

Everything else is M x M (Cholesky + inverse, triangular GEMMs) or M x batch.

Data parallel over the N observations: with a process group, every rank holds a
shard of (X, y).  Two all-reduces run per step: [P0 partial, c partial] (M^2 + M doubles) forward,
and [amp_bar, ls_bar, Z_bar] of the Kzx VJP (2 + M d doubles) backward.  The minibatch terms are
replicated and never reduced.
"""
from __future__ import annotations

import math

import torch

from . import linalg
from ._lib import call, query
from .linalg import F64, _p, _stream, kind_id

LOG_2PI = math.log(2.0 * math.pi)


def kernel_vjp(kind, X1, X2, amp, ls, Kbar, u=None, w=None, want_x1bar=True):
    """(grad[2] = (d/damp, d/dls), X1bar [n1, d] or None) of sum(Kbar * K(X1, X2))
    (+ the rank-1 term u w^T added to Kbar)."""
    X1, X2 = linalg.as_device(X1), linalg.as_device(X2)
    X1 = X1[:, None] if X1.dim() == 1 else X1
    X2 = X2[:, None] if X2.dim() == 1 else X2
    n1, d = X1.shape
    n2 = X2.shape[0]
    a, l = linalg._vec(amp), linalg._vec(ls)
    grad = torch.empty(2, dtype=F64, device=X1.device)
    X1bar = torch.empty((n1, d), dtype=F64, device=X1.device) if want_x1bar else None
    ws = linalg.workspace(query("vgposp_kernel_vjp_workspace_bytes", n1, n2, d))
    call("vgposp_kernel_vjp", kind_id(kind), _p(X1), n1, _p(X2), n2, d, _p(a), _p(l), _p(Kbar),
         Kbar.stride(0), _p(u), _p(w), _p(grad), _p(X1bar), _p(ws), ws.numel(), _stream())
    return grad, X1bar


def _chol_inv(A, infos=None, mixed=False):
    """(L^-1 with explicit zeros above the diagonal, sum log diag L) of an SPD [M, M] (copied).
    With ``infos`` (a list) the device status is appended for a later check instead of being
    synchronised on here.  mixed=True: fp32 factor + fp64 refinement (linalg.cholesky_inv_mixed,
    config C5); the refined factor is the fp64 one to rounding."""
    if mixed:
        Li, ld, info, _ = linalg.cholesky_inv_mixed(A, check=infos is None)
        if infos is not None:
            infos.append(info)
        return Li, torch.sum(torch.log(ld))
    Li, ld, info = linalg.cholesky_(A.clone(), invert=True, check=infos is None)
    if infos is not None:
        infos.append(info)
    return torch.tril(Li), torch.sum(torch.log(ld))


def _spd_inv(Li):
    """A^-1 = L^-T L^-1 (full) from L^-1."""
    return linalg.gemm(Li, Li, transa=True, tri_a=True, tri_b=True)


def _sym_from_lower(P):
    return torch.tril(P) + torch.tril(P, -1).t()


def _col(v):
    return v.reshape(-1, 1)


class VGPObjective:
    """Negative ELBO of the reference's VGP training graph and its gradient, for one kernel.

    ``Z`` [M, d], ``X`` [N, d] (this rank's shard), ``y`` [N]; ``amp``, ``ls``, ``noise`` are
    0-d / [1] device tensors (constrained values).  ``jitter`` is the VGP's jitter (Kzz factor,
    likelihood variance) and ``posterior_jitter`` that of optimal_variational_posterior.  The KL
    prior is N(0, Kzz + (noise + 1e-6) I): TFP's inducing-point GaussianProcess with its default
    jitter.
    """

    def __init__(self, kind, X, y, jitter=1e-6, posterior_jitter=1e-6, trace_adjoint=False,
                 group=None, precision="fp64"):
        if precision not in ("fp64", "mixed"):
            raise ValueError(f"precision must be 'fp64' or 'mixed', got {precision!r}")
        self.mixed = precision == "mixed"
        self.kind = kind
        self.X = linalg.as_device(X)
        self.X = self.X[:, None] if self.X.dim() == 1 else self.X
        self.y = linalg.as_device(y).reshape(-1)
        if self.y.numel() != self.X.shape[0]:
            raise ValueError("X and y sizes differ")
        self.j = float(jitter)
        self.pj = float(posterior_jitter)
        self.trace_adjoint = bool(trace_adjoint)
        self.group = group
        self._Kzx = None
        self._side = None

    def _allreduce(self, t):
        """Sum over the data-parallel group (host-staged for gloo, in place on device for RCCL)."""
        if self.group is None:
            return t
        dist = torch.distributed
        if dist.get_backend(self.group) == "gloo" and t.device.type != "cpu":
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def _kzx(self, Z, a, l):
        M, N = Z.shape[0], self.X.shape[0]
        if self._Kzx is None or self._Kzx.shape != (M, N):
            self._Kzx = torch.empty((1, M, N), dtype=F64, device=self.X.device)
        return linalg.kernel_matrix(self.kind, Z, self.X, a, l, out=self._Kzx)[0]

    def optimal_posterior(self, Z, amp, ls, noise):
        """(loc [M], scale [M, M]) of optimal_variational_posterior over all shards."""
        Z = linalg.as_device(Z)
        Z = Z[:, None] if Z.dim() == 1 else Z
        a, l, s = (linalg.as_device(v).reshape(()) for v in (amp, ls, noise))
        st = self._forward_posterior(Z, a, l, s)
        return st["m"], st["A"]

    def _kzz_factors(self, Kzz, s, infos):
        """The three Cholesky + inverse factorizations that need only Kzz (Kzz + jitter I for the
        VGP, Kzz + (noise + 1e-6) I for the KL prior, Kzz itself for log|det A|), enqueued on a
        side stream so that their latency-bound leaves overlap the Kzx assembly and the split-K
        Kzx Kzx^T on the main stream.  The caller waits on the returned stream before use."""
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream()
        side = self._side
        side.wait_stream(main)
        Kzz.record_stream(side)
        M = Kzz.shape[0]
        with torch.cuda.stream(side):
            I = torch.eye(M, dtype=F64, device=Kzz.device)
            Lzi, _ = _chol_inv(Kzz + self.j * I, infos, self.mixed)
            Lpi, logdetLp = _chol_inv(Kzz + (s + 1e-6) * I, infos, self.mixed)
            Lki, logdetLk = _chol_inv(Kzz, infos, self.mixed)
            out = dict(Lzi=Lzi, Kzj_inv=_spd_inv(Lzi), Lpi=Lpi, logdetLp=logdetLp,
                       Kp_inv=_spd_inv(Lpi), Kzz_inv=_spd_inv(Lki), logdetLk=logdetLk)
        for t in out.values():
            t.record_stream(main)
        for t in infos:
            t.record_stream(main)
        return out, side

    def _forward_posterior(self, Z, a, l, s, infos=None, side=False):
        M = Z.shape[0]
        Kzz = linalg.kernel_matrix(self.kind, Z, Z, a, l)[0]
        fac = self._kzz_factors(Kzz, s, infos) if side else None
        Kzx = self._kzx(Z, a, l)
        red = torch.empty(M * M + M, dtype=F64, device=Z.device)
        P0 = red[:M * M].view(M, M)
        c = red[M * M:].view(M, 1)
        linalg.gemm(Kzx, Kzx, P0, transb=True, lower_c=True, splitk=True)
        linalg.gemm(Kzx, _col(self.y), c)
        self._allreduce(red)
        P0 = _sym_from_lower(P0)
        c = c.reshape(-1)
        Sinv = Kzz + P0 / s
        Sinv.diagonal().add_(self.pj)
        Li, logdetL = _chol_inv(Sinv, infos, self.mixed)
        t = linalg.gemm(Li, linalg.gemm(Li, _col(c), tri_a=True), transa=True, tri_a=True)
        m = linalg.gemm(Kzz, t).reshape(-1) / s
        A = linalg.gemm(Li, Kzz, tri_a=True)
        st = dict(Kzz=Kzz, Kzx=Kzx, P0=P0, c=c, Li=Li, logdetL=logdetL, t=t.reshape(-1), m=m, A=A)
        if fac is not None:
            torch.cuda.current_stream().wait_stream(fac[1])
            st.update(fac[0])
        return st

    def loss_and_grads(self, Z, amp, ls, noise, Xb, yb, kl_weight, want_grads=True, infos=None):
        """-> (loss, d/damp, d/dls, d/dnoise, d/dZ [M, d]) as 0-d / [M, d] device tensors.

        No host synchronisation unless ``infos`` is None: with a list, the device Cholesky
        statuses are appended for the caller to check (the graph-captured training step)."""
        Z = linalg.as_device(Z)
        Z = Z[:, None] if Z.dim() == 1 else Z
        Xb = linalg.as_device(Xb)
        Xb = Xb[:, None] if Xb.dim() == 1 else Xb
        yb = linalg.as_device(yb).reshape(-1)
        a, l, s = (linalg.as_device(v).reshape(()) for v in (amp, ls, noise))
        j, w = self.j, float(kl_weight)
        M, nb = Z.shape[0], yb.numel()
        check = infos is None
        infos = [] if check else infos  # Cholesky statuses, checked once at the end
        # every 1 / s factor is applied on device to an M x M operand (no host copy of s)
        s_inv = 1.0 / s
        st = self._forward_posterior(Z, a, l, s, infos, side=True)
        Kzz, Kzx, P0, c, Li, logdetL, t, m, A = (st[k] for k in
                                                 ("Kzz", "Kzx", "P0", "c", "Li", "logdetL", "t",
                                                  "m", "A"))
        Kzb = linalg.kernel_matrix(self.kind, Z, Xb, a, l)[0]
        # ---- variational loss ----
        Lzi, Kzj_inv, Lpi, logdetLp, Kp_inv, Kzz_inv, logdetLk = (
            st[k] for k in ("Lzi", "Kzj_inv", "Lpi", "logdetLp", "Kp_inv", "Kzz_inv", "logdetLk"))
        v = linalg.gemm(Kzj_inv, _col(m))
        r = yb - linalg.gemm(Kzb, v, transa=True).reshape(-1)
        v = v.reshape(-1)
        s2 = s + j
        rr = torch.dot(r, r)
        obs = -0.5 * rr / s2 - 0.5 * nb * torch.log(2.0 * math.pi * s2)
        # Trace term with two M x B products instead of three: with H = Kzj^-1 Kzb (Kzj^-1 =
        # Lzi^T Lzi) and R = op(A) H,  tr(G^T G) = <Kzb, H> for G = Lzi Kzb, and
        # tr(R^T R) = <Q, H H^T> with Q = A^T A (A A^T for the trace_adjoint form).
        H = linalg.gemm(Kzj_inv, Kzb)
        HHt = _sym_from_lower(linalg.gemm(H, H, transb=True, lower_c=True))
        Q = linalg.gemm(A, A, transa=not self.trace_adjoint, transb=self.trace_adjoint)
        T = 0.5 * (nb * a * a - torch.dot(Kzb.reshape(-1), H.reshape(-1)) + torch.sum(Q * HHt)) / s
        logdetA = 2.0 * logdetLk - logdetL
        PA = linalg.gemm(Lpi, A, tri_a=True)
        qm = linalg.gemm(Lpi, _col(m), tri_a=True)
        KL = logdetLp - logdetA + 0.5 * (-M + torch.sum(PA * PA) + torch.sum(qm * qm))
        E = obs - T - w * KL
        if not want_grads:
            if check:
                for info in infos:
                    linalg.check_info(info)
            return -E, None, None, None, None
        # ---- reverse pass (d E) ----
        mu_b = r / s2
        s_b = 0.5 * rr / (s2 * s2) - 0.5 * nb / s2
        u = linalg.gemm(Kzj_inv, linalg.gemm(Kzb, _col(mu_b))).reshape(-1)
        m_b = u.clone()
        Kzz_b = -torch.outer(u, v)
        s_b = s_b + T / s
        a_b = -nb * a / s
        Kzz_b -= (0.5 * s_inv) * HHt
        # dE/dR = -R / s gives A_b = -(1/s) R H^T = -(1/s) A HHt (HHt A for trace_adjoint) and
        # H_b = -(1/s) Q H; through H = Kzj^-1 Kzb: Kzb_b += Kzj^-1 H_b, Kzz_b -= Kzj^-1 H_b H^T.
        # With P = Kzj^-1 Q all of it is M x M work plus one M x B product:
        #   Kzb_b = H / s + Kzj^-1 H_b = ((I - P) / s) H,   Kzz_b += (1/s) P HHt.
        A_b = (linalg.gemm(HHt, A) if self.trace_adjoint else linalg.gemm(A, HHt)) * (-s_inv)
        P = linalg.gemm(Kzj_inv, Q)
        Kzz_b += s_inv * linalg.gemm(P, HHt)
        W = -P
        W.diagonal().add_(1.0)
        Kzb_b = linalg.gemm(W * s_inv, H)
        QA = linalg.gemm(Kp_inv, A)
        qv = linalg.gemm(Kp_inv, _col(m)).reshape(-1)
        A_b -= w * QA
        m_b -= w * qv
        Kp_b = Kp_inv - torch.outer(qv, qv)
        linalg.gemm(QA, QA, Kp_b, alpha=-1.0, beta=1.0, transb=True)
        Kp_b *= -0.5 * w
        Kzz_b += Kp_b
        s_b = s_b + torch.trace(Kp_b)
        Kzz_b += w * Kzz_inv
        Sinv_b = (-0.5 * w) * _spd_inv(Li)
        Kzz_b += torch.outer(m_b, t) / s
        t_b = linalg.gemm(Kzz, _col(m_b)) / s
        s_b = s_b - torch.dot(m_b, m) / s
        c_b = linalg.gemm(Li, linalg.gemm(Li, t_b, tri_a=True), transa=True, tri_a=True).reshape(-1)
        ct = torch.outer(c_b, t)
        Sinv_b -= 0.5 * (ct + ct.t())
        linalg.gemm(Li, A_b, Kzz_b, beta=1.0, transa=True, tri_a=True)
        # Cholesky adjoint: L^T Lbar = -A_b A^T  ->  sym(L^-T Phi(-A_b A^T) L^-1)
        Pm = -torch.tril(linalg.gemm(A_b, A, transb=True))
        Pm.diagonal().mul_(0.5)
        Sc = linalg.gemm(Li, linalg.gemm(Pm, Li, tri_b=True), transa=True, tri_a=True)
        Sinv_b += 0.5 * (Sc + Sc.t())
        Kzz_b += Sinv_b
        s_b = s_b - torch.sum(Sinv_b * P0) / (s * s)
        # Kzx_bar = (2 / s) Sinv_b Kzx + c_b y^T  (rank-1 term fused into the VJP)
        Kzx_b = linalg.gemm(Sinv_b * (2.0 * s_inv), Kzx)
        g2, Zb2 = kernel_vjp(self.kind, Z, self.X, a, l, Kzx_b, c_b, self.y)
        red = torch.cat([g2, Zb2.reshape(-1)])
        self._allreduce(red)
        g2, Zb2 = red[:2], red[2:].view_as(Z)
        g1, Zb1 = kernel_vjp(self.kind, Z, Z, a, l, (Kzz_b + Kzz_b.t()).contiguous())
        g3, Zb3 = kernel_vjp(self.kind, Z, Xb, a, l, Kzb_b, v, mu_b)
        a_b = a_b + 0.5 * g1[0] + g2[0] + g3[0]
        l_b = 0.5 * g1[1] + g2[1] + g3[1]
        Z_b = Zb1 + Zb2 + Zb3
        if check:
            for info in infos:
                linalg.check_info(info)
        return -E, -a_b, -l_b, -s_b, -Z_b


__all__ = ["VGPObjective", "kernel_vjp"]

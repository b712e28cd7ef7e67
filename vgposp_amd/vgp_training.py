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

import ctypes

import torch

from . import linalg
from ._lib import call, query
from .linalg import F64, _p, _stream, kind_id

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


def _chol_inv(A, infos=None, mixed=False, inplace=False, mixed_iters=None):
    """(L^-1 in the lower triangle, diag L [M]) of an SPD [M, M].  The upper triangle of the
    result is NOT zeroed: every consumer reads it as a stored-lower-triangular GEMM operand
    (tri_a / tri_b).  ``inplace`` factors A itself instead of a copy.  With ``infos`` (a list) the
    device status is appended for a later check instead of being synchronised on here.
    mixed=True: fp32 factor + fp64 refinement (linalg.cholesky_inv_mixed, config C5); the refined
    factor is the fp64 one to rounding."""
    if mixed:
        Li, ld, info, _ = linalg.cholesky_inv_mixed(A, iters=mixed_iters, check=infos is None)
    else:
        Li, ld, info = linalg.cholesky_(A if inplace else A.clone(), invert=True,
                                        check=infos is None)
        ld = ld.reshape(-1)
    if infos is not None:
        infos.append(info)
    return Li, ld


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


def _lincomb(terms, s=None, shift=0.0, diag_scale=1.0, diag=(0.0, 0), out=None):
    """out = sum c (s + shift)^e X over terms [(X, c, e)] (same shape, contiguous), on the
    diagonal of a square out times diag_scale plus diag[0] (s + shift)^diag[1]
    (vgposp_lincomb: one launch, s read on device)."""
    X0 = terms[0][0]
    if out is None:
        out = torch.empty_like(X0)
    rows, cols = (X0.shape[0], X0.shape[1]) if X0.dim() == 2 else (1, X0.numel())
    xs = _ptrs([t[0] for t in terms])
    cs = (ctypes.c_double * len(terms))(*[float(t[1]) for t in terms])
    es = (ctypes.c_int * len(terms))(*[int(t[2]) for t in terms])
    call("vgposp_lincomb", rows, cols, cols, len(terms), xs, cs, es, float(diag_scale),
         float(diag[0]), int(diag[1]), _p(s), float(shift), _p(out), _stream())
    return out


def _dots(pairs, out):
    """out[p] = the p-th of [(x, incx, y or None, incy, n, op)] (vgposp_dots, op 1 = sum log)."""
    n = len(pairs)
    ws = linalg.workspace(query("vgposp_dots_workspace_bytes", n))
    call("vgposp_dots", n, _ptrs([q[0] for q in pairs]),
         (ctypes.c_int64 * n)(*[q[1] for q in pairs]), _ptrs([q[2] for q in pairs]),
         (ctypes.c_int64 * n)(*[q[3] for q in pairs]), (ctypes.c_int64 * n)(*[q[4] for q in pairs]),
         (ctypes.c_int * n)(*[q[5] for q in pairs]), _p(out), _p(ws), ws.numel(), _stream())
    return out


def _spd_inv(Li):
    """A^-1 = L^-T L^-1 (full) from L^-1."""
    return linalg.gemm(Li, Li, transa=True, tri_a=True, tri_b=True)


def _col(v):
    return v.reshape(-1, 1)


def _wait(a, b):
    """Stream a waits for the work enqueued so far on stream b (nothing when they are one)."""
    if a is not b:
        a.wait_stream(b)


class VGPObjective:
    """Negative ELBO of the reference's VGP training graph and its gradient, for one kernel.

    ``Z`` [M, d], ``X`` [N, d] (this rank's shard), ``y`` [N]; ``amp``, ``ls``, ``noise`` are
    0-d / [1] device tensors (constrained values).  ``jitter`` is the VGP's jitter (Kzz factor,
    likelihood variance) and ``posterior_jitter`` that of optimal_variational_posterior.  The KL
    prior is N(0, Kzz + (noise + 1e-6) I): TFP's inducing-point GaussianProcess with its default
    jitter.
    """

    def __init__(self, kind, X, y, jitter=1e-6, posterior_jitter=1e-6, trace_adjoint=False,
                 group=None, precision="fp64", streams=None, grouped=True):
        # "mixed" = fp32 factor + 3 fp64 refinement steps (fp64 to rounding); "mixed:2" = two
        # steps (|E| 1e-2 -> 1e-8: the ELBO within north_star's 1e-5 of fp64).
        # ``streams``: side-stream bitmask of the training step (1: Kzb beside the forward pass,
        # 2: the vector chain beside the M x M products, 4: VJPs and reductions beside G Kzx);
        # None = the measured default (0 for fp64, 7 for mixed, see loss_and_grads).
        # ``grouped``: the M x M products of one dependency level in one grouped launch.
        kind_, _, steps = str(precision).partition(":")
        if kind_ not in ("fp64", "mixed") or (steps and (kind_ != "mixed" or not steps.isdigit())):
            raise ValueError(f"precision must be 'fp64', 'mixed' or 'mixed:<steps>', "
                             f"got {precision!r}")
        self.mixed = kind_ == "mixed"
        self.mixed_iters = int(steps) if steps else None
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
        self._tail = None  # side stream of the step (Kzb, the vector chain, VJPs, reductions)
        self._capture_hook = None  # set by VGPTrainOp while capturing a data-parallel step
        self._streams = (7 if self.mixed else 0) if streams is None else int(streams)
        if not 0 <= self._streams <= 7:
            raise ValueError(f"streams must be a bitmask in [0, 7], got {streams!r}")
        self.grouped = bool(grouped)

    def _allreduce(self, t):
        """Sum over the data-parallel group (host-staged for gloo, in place on device for RCCL).
        While a segmented HIP graph of the step is being captured (VGPTrainOp with a group), the
        all-reduce is a segment boundary instead: the capture hook ends the current graph there
        and the replay runs the all-reduce between the segments."""
        if self.group is None:
            return t
        if self._capture_hook is not None:
            return self._capture_hook(t)
        return self.allreduce_now(t)

    def join_side_streams(self):
        """The current stream waits for every side stream of the step (a segment boundary)."""
        cur = torch.cuda.current_stream()
        for st in (self._side or []) + ([self._tail] if self._tail is not None else []):
            _wait(cur, st)

    def allreduce_now(self, t):
        dist = torch.distributed
        if dist.get_backend(self.group) == "gloo" and t.device.type != "cpu":
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def _kzx(self, Z, a, l, c):
        """Kzx = K(Z, X) [M, N] and c <- Kzx y in one pass over Kzx."""
        M, N = Z.shape[0], self.X.shape[0]
        if self._Kzx is None or self._Kzx.shape != (M, N):
            self._Kzx = torch.empty((M, N), dtype=F64, device=self.X.device)
        linalg.kernel_matrix_matvec(self.kind, Z, self.X, a, l, self.y, self._Kzx, c)
        return self._Kzx

    def optimal_posterior(self, Z, amp, ls, noise):
        """(loc [M], scale [M, M]) of optimal_variational_posterior over all shards."""
        Z = linalg.as_device(Z)
        Z = Z[:, None] if Z.dim() == 1 else Z
        a, l, s = (linalg.as_device(v).reshape(()) for v in (amp, ls, noise))
        st = self._forward_posterior(Z, a, l, s)
        return st["m"], st["A"]

    def _kzz_factors(self, Kzz, s, infos, fork):
        """The three Cholesky + inverse factorizations that need only Kzz (Kzz + jitter I for the
        VGP, Kzz + (noise + 1e-6) I for the KL prior, Kzz itself for log|det A|), each on its own
        side stream, so that their latency-bound leaves run beside one another and beside the
        Kzx assembly and the split-K Kzx Kzx^T already enqueued on the main stream.  ``fork`` is
        the main-stream event recorded right after Kzz: the side chains depend on nothing later.
        (Captured into the step's HIP graph, the heavy main-stream nodes come first in capture
        order, so they are dispatched first.)  The caller waits on the returned streams."""
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = [torch.cuda.Stream() for _ in range(3)]
        res = []
        for i, st in enumerate(self._side):
            st.wait_event(fork)
            Kzz.record_stream(st)
            s.record_stream(st)
            with torch.cuda.stream(st):
                A = Kzz.clone()
                if i == 0:
                    A.diagonal().add_(self.j)
                elif i == 1:  # computed on this stream: it depends only on s (before the fork)
                    A.diagonal().add_(s + 1e-6)
                mine = []
                Li, ld = _chol_inv(A, mine, self.mixed, inplace=True,
                                   mixed_iters=self.mixed_iters)
                res.append((Li, ld, _spd_inv(Li), mine))
        (Lzi, _, Kzj_inv, i1), (Lpi, ldp, Kp_inv, i2), (Lki, ldk, Kzz_inv, i3) = res
        infos.extend(i1 + i2 + i3)
        out = dict(Lzi=Lzi, Kzj_inv=Kzj_inv, Lpi=Lpi, ldp=ldp, Kp_inv=Kp_inv, Kzz_inv=Kzz_inv,
                   ldk=ldk)
        for t in list(out.values()) + infos:
            t.record_stream(main)
        return out, self._side

    def _forward_posterior(self, Z, a, l, s, infos=None, side=False):
        """The optimal posterior's pieces.  side=True (the training step) also forms the three
        Kzz-only inverse factors: fp64 as ONE batched Cholesky + inverse of [Sinv, Kzz + jI,
        Kzz + (s + 1e-6) I, Kzz] after the SYRK (every launch of the recursion covers the four,
        so the latency-bound chain is paid once) and one batched L^-T L^-1; mixed precision on
        three side streams beside the Kzx assembly and SYRK."""
        M = Z.shape[0]
        Kzz = linalg.kernel_matrix(self.kind, Z, Z, a, l)[0]
        batched = side and not self.mixed
        fork = None
        if side and not batched:
            fork = torch.cuda.Event()
            fork.record()
        red = torch.empty(M * M + M, dtype=F64, device=Z.device)
        P0 = red[:M * M].view(M, M)
        c = red[M * M:].view(M, 1)
        Kzx = self._kzx(Z, a, l, c)  # c = Kzx y fused into the assembly
        linalg.gemm(Kzx, Kzx, P0, transb=True, lower_c=True, splitk=True)
        fac = self._kzz_factors(Kzz, s, infos, fork) if fork is not None else None
        self._allreduce(red)
        # P0 -> symmetric in place, Sinv = Kzz + P0 / s + pj I (+ the Kzz matrices), one launch
        nf = 4 if batched else 1
        F = torch.empty((nf, M, M), dtype=F64, device=Z.device)
        call("vgposp_vgp_sinv", _p(P0), M, M, _p(Kzz), _p(s), self.pj, self.j, _p(F), nf,
             _stream())
        c = c.reshape(-1)
        st = {}
        if batched:
            F, ld, info = linalg.cholesky_(F, invert=True, check=infos is None)
            if infos is not None:
                infos.append(info)
            # L^-T L^-1 of all four (Sinv's is the reverse pass's Sinv^-1)
            spd = linalg.gemm_batched(F, F, transa=True, tri_a=True, tri_b=True)
            Li, lds = F[0], ld[0]
            st.update(LiLi=spd[0], Lzi=F[1], Kzj_inv=spd[1], Lpi=F[2], ldp=ld[2], Kp_inv=spd[2],
                      Kzz_inv=spd[3], ldk=ld[3])
        else:
            Li, lds = _chol_inv(F[0], infos, self.mixed, inplace=True,
                                mixed_iters=self.mixed_iters)
        t = linalg.gemm(Li, linalg.gemm(Li, _col(c), tri_a=True), transa=True, tri_a=True)
        m = linalg.gemm(Kzz, t).reshape(-1) / s
        A = linalg.gemm(Li, Kzz, tri_a=True)
        st.update(Kzz=Kzz, Kzx=Kzx, P0=P0, c=c, Li=Li, lds=lds, t=t.reshape(-1), m=m, A=A)
        if fac is not None:
            for stream in fac[1]:
                torch.cuda.current_stream().wait_stream(stream)
            st.update(fac[0])
        return st

    def loss_and_grads(self, Z, amp, ls, noise, Xb, yb, kl_weight, want_grads=True, infos=None,
                       zbar_out=None):
        """-> (loss, d/damp, d/dls, d/dnoise, d/dZ [M, d]) as 0-d / [M, d] device tensors
        (d/dZ written into ``zbar_out`` when given).

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
        # the minibatch's Kzb depends only on the inputs: with side streams on (bit 1) it is
        # assembled beside the forward posterior's Kzx assembly and SYRK
        main = torch.cuda.current_stream()
        if self._tail is None:
            # Side stream use, bit 1: Kzb beside the forward pass, 2: the vector chain beside the
            # M x M products, 4: VJPs and reductions beside G Kzx.  Measured per segment
            # (tools/vgp_ab.py, profiles/r3_vgp_ab_streams_segments_*.jsonl): the fp64 step is
            # fastest on ONE stream (C3 6.14 ms with none, 6.19-6.28 with any; C5 7.25 against
            # 7.40-7.54), the mixed one with all three (9.15 against 9.72 ms: its factorizations
            # already run on side streams).
            self._tail = torch.cuda.Stream()
        use = self._streams
        tail = self._tail if use & 1 else main
        _wait(tail, main)
        with torch.cuda.stream(tail):
            Kzb = linalg.kernel_matrix(self.kind, Z, Xb, a, l)[0]
        Kzb.record_stream(main)
        st = self._forward_posterior(Z, a, l, s, infos, side=True)
        Kzz, Kzx, P0, c, Li, t, m, A = (st[k] for k in
                                        ("Kzz", "Kzx", "P0", "c", "Li", "t", "m", "A"))
        _wait(main, tail)
        Kzj_inv, Lpi, Kp_inv, Kzz_inv = (st[k] for k in ("Kzj_inv", "Lpi", "Kp_inv", "Kzz_inv"))
        dev = Z.device
        # ---- variational loss (every scalar is taken at the end by vgposp_dots / _scalars) ----
        # The vector chain (v, r, u, m_b, c_b: GEMVs) is independent of the matrix products until
        # the Kzz adjoint; with side streams on (bit 2) it runs on its own stream beside them.
        # Every operand comes from before the fork; every result is read only after the join.
        tail = self._tail if use & 2 else main
        _wait(tail, main)
        with torch.cuda.stream(tail):
            v = linalg.gemm(Kzj_inv, _col(m))
            r = yb.clone()
            linalg.gemm(Kzb, v, _col(r), alpha=-1.0, beta=1.0, transa=True)  # r = yb - Kzb^T v
            v = v.reshape(-1)
            qm = linalg.gemm(Lpi, _col(m), tri_a=True)
            if want_grads:
                mu_b = _lincomb([(r, 1.0, -1)], s, shift=j)  # r / (s + j)
                u = linalg.gemm(Kzj_inv, linalg.gemm(Kzb, _col(mu_b))).reshape(-1)
                qv = linalg.gemm(Kp_inv, _col(m)).reshape(-1)
                m_b = _lincomb([(u, 1.0, 0), (qv, -w, 0)])
                t_b = linalg.gemm(Kzz, _col(m_b)) / s
                c_b = linalg.gemm(Li, linalg.gemm(Li, t_b, tri_a=True), transa=True,
                                  tri_a=True).reshape(-1)
        # Trace terms from ONE M x B product, the SYRK Sb = Kzb Kzb^T: with H = Kzj^-1 Kzb
        # (Kzj^-1 = Lzi^T Lzi) and R = op(A) H,  tr(G^T G) = <Kzb, H> = <Sb, Kzj^-1> for
        # G = Lzi Kzb, and tr(R^T R) = <Q, H H^T> with Q = A^T A (A A^T for the trace_adjoint
        # form) and H H^T = Kzj^-1 Sb Kzj^-1 (M x M products); H itself is never formed.
        # The M x M products go in dependency levels, each level ONE grouped launch
        # (linalg.gemm_group): they are latency-bound and fill only a few dozen CUs each.
        Sb = linalg.gemm(Kzb, Kzb, transb=True, lower_c=True)
        call("vgposp_sym_from_lower", _p(Sb), M, M, _stream())
        ta = self.trace_adjoint
        lv = [dict(A=Kzj_inv, B=Sb), dict(A=A, B=A, transa=not ta, transb=ta),
              dict(A=Lpi, B=A, tri_a=True)]
        if want_grads:
            lv.append(dict(A=Kp_inv, B=A))
        T1, Q, PA, *rest = linalg.gemm_group(lv, self.grouped)
        HHt = torch.empty((M, M), dtype=F64, device=dev)  # lower product, then mirrored
        lv = [dict(A=T1, B=Kzj_inv, C=HHt, lower_c=True)]
        if want_grads:
            QA = rest[0]
            lv += [dict(A=Kzj_inv, B=Q), dict(A=QA, B=QA, transb=True)]
        _, *rest = linalg.gemm_group(lv, self.grouped)
        call("vgposp_sym_from_lower", _p(HHt), M, M, _stream())
        sums = torch.zeros(13, dtype=F64, device=dev)  # VGPOSP_S_* of vgposp.h
        fwd = [(r, 1, r, 1, nb, 0), (Sb, 1, Kzj_inv, 1, M * M, 0), (Q, 1, HHt, 1, M * M, 0),
               (PA, 1, PA, 1, M * M, 0), (qm, 1, qm, 1, M, 0), (st["lds"], 1, None, 0, M, 1),
               (st["ldp"], 1, None, 0, M, 1), (st["ldk"], 1, None, 0, M, 1)]
        if not want_grads:
            _wait(main, tail)
            _dots(fwd, sums)
            zero = torch.zeros(2, dtype=F64, device=dev)
            out = torch.empty(4, dtype=F64, device=dev)
            call("vgposp_vgp_scalars", _p(sums), _p(s), _p(a), _p(zero), _p(zero), _p(zero),
                 float(nb), float(M), w, j, _p(out), _stream())
            if check:
                for info in infos:
                    linalg.check_info(info)
            return out[0], None, None, None, None
        P, QAQA = rest
        # ---- reverse pass (d E) ----
        # dE/dR = -R / s gives A_b = -(1/s) A HHt (HHt A for trace_adjoint) and H_b = -(1/s) Q H;
        # through H = Kzj^-1 Kzb: Kzb_b += Kzj^-1 H_b, Kzz_b -= Kzj^-1 H_b H^T.  With
        # P = Kzj^-1 Q all of it is M x M work plus one M x B product:
        #   Kzb_b = H / s + Kzj^-1 H_b = ((I - P) / s) H = (W Kzj^-1) Kzb,  Kzz_b += (1/s) P HHt.
        AH, PHH = linalg.gemm_group([dict(A=HHt, B=A) if ta else dict(A=A, B=HHt),
                                     dict(A=P, B=HHt)], self.grouped)
        A_b = _lincomb([(AH, -1.0, -1), (QA, -w, 0)], s)
        W = _lincomb([(P, -1.0, -1)], s, diag=(1.0, -1))  # (I - P) / s
        WK, LiA, ABt = linalg.gemm_group([dict(A=W, B=Kzj_inv),
                                          dict(A=Li, B=A_b, transa=True, tri_a=True),
                                          dict(A=A_b, B=A, transb=True)], self.grouped)
        Kzb_b = linalg.gemm(WK, Kzb)
        LiLi = st["LiLi"] if "LiLi" in st else _spd_inv(Li)
        # Cholesky adjoint: L^T Lbar = -A_b A^T  ->  sym(L^-T Phi(-A_b A^T) L^-1); Phi's lower
        # triangle (halved diagonal) is read through tri_a, its upper part is ignored
        Pm = _lincomb([(ABt, -1.0, 0)], diag_scale=0.5)
        Sc = linalg.gemm(Li, linalg.gemm(Pm, Li, tri_a=True, tri_b=True), transa=True, tri_a=True)
        _wait(main, tail)
        KzzS = torch.empty((M, M), dtype=F64, device=dev)
        G = torch.empty((M, M), dtype=F64, device=dev)
        call("vgposp_vgp_kzz_bar", M, _ptrs([u, v, qv, m_b, st["t"], c_b]),
             _ptrs([HHt, PHH, Kp_inv, QAQA, Kzz_inv, LiLi, Sc, LiA]), _p(s), w, _p(KzzS), _p(G),
             _stream())
        # The two small kernel VJPs and every reduction of the loss read nothing the big product
        # below writes: with side streams on (bit 4) they run beside it.  Every tensor they read
        # was made on the main stream before the fork and stays referenced until the join.
        _wait(tail, main)
        with torch.cuda.stream(tail):
            g1, Zb1 = kernel_vjp(self.kind, Z, Z, a, l, KzzS)
            g3, Zb3 = kernel_vjp(self.kind, Z, Xb, a, l, Kzb_b, v, mu_b)
            rev = [(Kp_inv, M + 1, None, 0, M, 0), (qv, 1, qv, 1, M, 0),
                   (QAQA, M + 1, None, 0, M, 0), (m_b, 1, m, 1, M, 0), (G, 1, P0, 1, M * M, 0)]
            _dots(fwd + rev, sums)
        # Kzx_bar = G Kzx + c_b y^T, G = (2 / s) Sinv_b (rank-1 term fused into the VJP).  A GEMM
        # whose epilogue reduced each tile straight into the VJP partials (Kzx_bar never written)
        # was measured slower: 2.92 ms against 2.30 + 0.43 ms for the two passes
        Kzx_b = linalg.gemm(G, Kzx)
        g2, Zb2 = kernel_vjp(self.kind, Z, self.X, a, l, Kzx_b, c_b, self.y)
        if self.group is not None:
            red = torch.cat([g2, Zb2.reshape(-1)])
            self._allreduce(red)
            g2, Zb2 = red[:2], red[2:].view_as(Z)
        _wait(main, tail)
        out = torch.empty(4, dtype=F64, device=dev)
        call("vgposp_vgp_scalars", _p(sums), _p(s), _p(a), _p(g1), _p(g2), _p(g3), float(nb),
             float(M), w, j, _p(out), _stream())
        Z_b = _lincomb([(Zb1, -1.0, 0), (Zb2, -1.0, 0), (Zb3, -1.0, 0)], out=zbar_out)
        if check:
            for info in infos:
                linalg.check_info(info)
        return out[0], out[1], out[2], out[3], Z_b


__all__ = ["VGPObjective", "kernel_vjp"]

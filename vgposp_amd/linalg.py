"""Device-side linear algebra on libvgposp (PyTorch tensors are only the HBM containers).

Every function here enqueues HIP kernels from libvgposp.so on the current torch stream; nothing is
computed by torch itself.  Shapes: a matrix argument is [n, m] or a batch [B, n, m] (row-major,
contiguous, float64, on a ROCm device).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import FULL, LOWER, KERNEL_KINDS, CholeskyError, call, query

F64 = torch.float64


def device():
    if not torch.cuda.is_available():
        raise _lib.VgpospUnavailable("vgposp_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _p(t):
    """Device pointer of a tensor for the C-ABI.  Refuses host tensors: every libvgposp buffer
    argument is a device pointer, and a host address reaching a kernel is a memory fault."""
    if t is None:
        return ctypes.c_void_p(0)
    if t.device.type != "cuda":
        raise ValueError(f"libvgposp needs device tensors, got one on {t.device}")
    return ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def as_device(x, dtype=F64):
    """numpy / list / tensor -> contiguous device tensor (no copy if already there)."""
    if isinstance(x, torch.Tensor):
        t = x
        if t.device.type != "cuda":
            t = t.to(device())
        if t.dtype != dtype:
            t = t.to(dtype)
        return t.contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device()).contiguous()


def _vec(x, B=None):
    t = as_device(np.atleast_1d(np.asarray(x, dtype=np.float64)) if not isinstance(x, torch.Tensor) else x.reshape(-1))
    if B is not None and t.numel() == 1 and B > 1:
        t = t.expand(B).contiguous()
    return t


def workspace(nbytes):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device())


def kind_id(kind):
    if isinstance(kind, int):
        return kind
    try:
        return KERNEL_KINDS[kind]
    except KeyError:
        raise ValueError(f"unknown kernel kind {kind!r}; expected one of {list(KERNEL_KINDS)}")


def kernel_matrix(kind, X1, X2=None, amp=1.0, ls=1.0, diag_shift=None, lower=False, out=None):
    """K[b, i, j] = exp(2 log amp_b + log k(|X1_i - X2_j| / ls_b)) (+ diag_shift_b on i == j).

    Returns a [B, n1, n2] float64 device tensor (B = broadcast size of amp / ls)."""
    X1 = as_device(X1)
    if X1.dim() == 1:
        X1 = X1[:, None]
    X2 = X1 if X2 is None else as_device(X2)
    if X2.dim() == 1:
        X2 = X2[:, None]
    if X1.shape[1] != X2.shape[1]:
        raise ValueError("X1 and X2 must have the same number of features")
    a = _vec(amp)
    l = _vec(ls)
    B = max(a.numel(), l.numel())
    a, l = _vec(a, B), _vec(l, B)
    if a.numel() != B or l.numel() != B:
        raise ValueError("amp and ls must broadcast to one batch size")
    sh = None if diag_shift is None else _vec(diag_shift, B)
    n1, n2, d = X1.shape[0], X2.shape[0], X1.shape[1]
    if out is None:
        out = torch.empty((B, n1, n2), dtype=F64, device=X1.device)
    call("vgposp_kernel_matrix", kind_id(kind), _p(X1), n1, _p(X2), n2, d, _p(a), _p(l), _p(sh), B,
         LOWER if lower else FULL, _p(out), out.stride(-2), out.stride(0) if out.dim() == 3 else 0,
         _stream())
    return out


def kernel_matrix_matvec(kind, X1, X2, amp, ls, v, out_K, out_v):
    """out_K [n1, n2] <- K(X1, X2) (one amplitude / length scale) and out_v [n1] <- K v in one
    pass (vgposp_kernel_matrix_matvec: K is never re-read for the product)."""
    X1, X2, v = as_device(X1), as_device(X2), as_device(v).reshape(-1)
    X1 = X1[:, None] if X1.dim() == 1 else X1
    X2 = X2[:, None] if X2.dim() == 1 else X2
    n1, n2, d = X1.shape[0], X2.shape[0], X1.shape[1]
    if out_K.shape[-2:] != (n1, n2) or v.numel() != n2 or out_v.numel() != n1:
        raise ValueError("kernel_matrix_matvec: shapes do not match")
    a, l = _vec(amp, 1), _vec(ls, 1)
    ws = workspace(query("vgposp_kernel_matrix_matvec_workspace_bytes", n1, n2))
    call("vgposp_kernel_matrix_matvec", kind_id(kind), _p(X1), n1, _p(X2), n2, d, _p(a), _p(l),
         _p(out_K), out_K.stride(-2), _p(v), _p(out_v), _p(ws), ws.numel(), _stream())
    return out_K, out_v


def gemm(A, B, C=None, alpha=1.0, beta=0.0, transa=False, transb=False, lower_c=False,
         tri_a=False, tri_b=False, splitk=True):
    """C = alpha op(A) op(B) + beta C on fp64 MFMA (2-D operands).  ``splitk=True`` lets the
    library split a long K over extra workgroups when there are few output tiles (deterministic
    two-pass reduction through a workspace)."""
    A, B = as_device(A), as_device(B)
    m = A.shape[1] if transa else A.shape[0]
    k = A.shape[0] if transa else A.shape[1]
    kb = B.shape[1] if transb else B.shape[0]
    n = B.shape[0] if transb else B.shape[1]
    if k != kb:
        raise ValueError(f"inner dimensions differ: {k} vs {kb}")
    if C is None:  # a lower-C result keeps a zero upper triangle; a full one is written entirely
        C = (torch.zeros if lower_c else torch.empty)((m, n), dtype=F64, device=A.device)
        beta = 0.0
    uplo = LOWER if lower_c else FULL
    if splitk:
        nbytes = query("vgposp_gemm_splitk_workspace_bytes", m, n, k, uplo, 0)
        if nbytes:
            ws = workspace(nbytes)
            call("vgposp_gemm_splitk", int(transa), int(transb), m, n, k, float(alpha), _p(A),
                 A.stride(0), _p(B), B.stride(0), float(beta), _p(C), C.stride(0), uplo,
                 int(tri_a), int(tri_b), 0, _p(ws), ws.numel(), _stream())
            return C
    call("vgposp_gemm", int(transa), int(transb), m, n, k, float(alpha), _p(A), A.stride(0), _p(B),
         B.stride(0), float(beta), _p(C), C.stride(0), uplo, int(tri_a), int(tri_b), _stream())
    return C


def gemm_group(specs, grouped=True):
    """Independent GEMMs in ONE launch (vgposp_gemm_group): ``specs`` is a list of dicts with the
    arguments of :func:`gemm` (A, B and optionally C, alpha, beta, transa, transb, lower_c, tri_a,
    tri_b).  Returns the list of C.  For latency-bound small products (each filling a few dozen
    CUs) that a single stream would otherwise issue one after another.  ``grouped=False`` issues
    one launch per product (the A/B reference)."""
    n = len(specs)
    if n == 0:
        return []
    if not grouped:
        return [gemm(**sp) for sp in specs]
    flags, dims, al, be, As, lda, Bs, ldb, Cs, ldc, outs = ([] for _ in range(11))
    keep = []  # device copies of host operands stay alive until the launch is enqueued
    for sp in specs:
        A, B = as_device(sp["A"]), as_device(sp["B"])
        keep += [A, B]
        ta, tb = bool(sp.get("transa", False)), bool(sp.get("transb", False))
        lower = bool(sp.get("lower_c", False))
        m = A.shape[1] if ta else A.shape[0]
        k = A.shape[0] if ta else A.shape[1]
        kb = B.shape[1] if tb else B.shape[0]
        nn = B.shape[0] if tb else B.shape[1]
        if k != kb:
            raise ValueError(f"gemm_group: inner dimensions differ: {k} vs {kb}")
        C, beta = sp.get("C"), float(sp.get("beta", 0.0))
        if C is None:
            C = (torch.zeros if lower else torch.empty)((m, nn), dtype=F64, device=A.device)
            beta = 0.0
        flags += [int(ta), int(tb), LOWER if lower else FULL, int(bool(sp.get("tri_a", False))),
                  int(bool(sp.get("tri_b", False)))]
        dims += [m, nn, k]
        al.append(float(sp.get("alpha", 1.0)))
        be.append(beta)
        As.append(A.data_ptr())
        lda.append(A.stride(0))
        Bs.append(B.data_ptr())
        ldb.append(B.stride(0))
        Cs.append(C.data_ptr())
        ldc.append(C.stride(0))
        outs.append(C)
    fl = (ctypes.c_int * len(flags))(*flags)
    dm = (ctypes.c_int64 * len(dims))(*dims)
    ws = workspace(query("vgposp_gemm_group_workspace_bytes", n, fl, dm))
    vp = ctypes.c_void_p
    call("vgposp_gemm_group", n, fl, dm, (ctypes.c_double * n)(*al), (ctypes.c_double * n)(*be),
         (vp * n)(*As), (ctypes.c_int64 * n)(*lda), (vp * n)(*Bs), (ctypes.c_int64 * n)(*ldb),
         (vp * n)(*Cs), (ctypes.c_int64 * n)(*ldc), _p(ws), ws.numel(), _stream())
    return outs


def gemm_batched(A, B, C=None, alpha=1.0, beta=0.0, transa=False, transb=False, lower_c=False,
                 tri_a=False, tri_b=False):
    """C[b] = alpha op(A[b]) op(B[b]) + beta C[b] for [batch, rows, cols] contiguous operands, one
    launch (vgposp_gemm_batched, split-K when few output tiles)."""
    A, B = as_device(A), as_device(B)
    nb = A.shape[0]
    m = A.shape[2] if transa else A.shape[1]
    k = A.shape[1] if transa else A.shape[2]
    n = B.shape[1] if transb else B.shape[2]
    if B.shape[0] != nb or (B.shape[2] if transb else B.shape[1]) != k:
        raise ValueError("gemm_batched: shapes do not match")
    if C is None:
        C = (torch.zeros if lower_c else torch.empty)((nb, m, n), dtype=F64, device=A.device)
        beta = 0.0
    uplo = LOWER if lower_c else FULL
    ws = workspace(query("vgposp_gemm_batched_workspace_bytes", m, n, k, uplo, nb))
    call("vgposp_gemm_batched", int(transa), int(transb), m, n, k, float(alpha), _p(A),
         A.stride(1), A.stride(0), _p(B), B.stride(1), B.stride(0), float(beta), _p(C),
         C.stride(1), C.stride(0), uplo, int(tri_a), int(tri_b), nb, _p(ws), ws.numel(),
         _stream())
    return C


def _batched(A):
    if A.dim() == 2:
        return A.unsqueeze(0), True
    return A, False


def check_info(info):
    """Synchronise on the device status of a factorization; raise CholeskyError if not PD."""
    bad = torch.nonzero(info).flatten()
    if bad.numel():
        b = int(bad[0])
        raise CholeskyError(int(info[b]), b)


def cholesky_(A, invert=False, check=True, ldiag=None):
    """In-place blocked Cholesky of the lower triangle of A ([n, n] or [B, n, n]).

    invert=False: lower(A) <- L;  invert=True: lower(A) <- L^-1.  The strictly upper triangle is
    untouched.  Returns (A, ldiag[B, n] = diag(L), info[B])."""
    A3, _ = _batched(A)
    Bn, n = A3.shape[0], A3.shape[-1]
    # rows contiguous; a padded row stride (lda > n) is allowed
    if A3.stride(2) != 1 or A3.stride(1) < n or (Bn > 1 and A3.stride(0) < n * A3.stride(1)):
        raise ValueError("A must have contiguous rows (row stride >= n, batch stride >= n * lda)")
    if ldiag is None:
        ldiag = torch.empty((Bn, n), dtype=F64, device=A3.device)
    info = torch.empty(Bn, dtype=torch.int32, device=A3.device)
    # a batch of n > 128 matrices runs as ONE recursion (every launch covers the batch)
    ws = workspace(query("vgposp_potrf_batched_workspace_bytes", n, Bn) if Bn > 1 and n > 128
                   else query("vgposp_potrf_workspace_bytes", n))
    call("vgposp_potrf_lower", _p(A3), n, A3.stride(1), A3.stride(0), Bn, int(invert), _p(ldiag),
         _p(info), _p(ws), ws.numel(), _stream())
    if check:
        check_info(info)
    return A, ldiag, info


def cholesky_inv_mixed(A, iters=None, check=True):
    """Mixed-precision inverse Cholesky factor of a full symmetric [n, n] A (config C5): fp32 factor
    on the f32 matrix cores, ``iters`` fp64 refinement steps (vgposp_potrf_mixed; default 3).
    Returns
    (L^-1 with zeros above the diagonal, diag(L) [n], info [1], resid [1] = max|X A X^T - I| of the
    last step); A is not modified."""
    if iters is None:
        iters = 3
    A = as_device(A)
    if A.dim() != 2 or A.shape[0] != A.shape[1]:
        raise ValueError("A must be square")
    if not A.is_contiguous():
        A = A.contiguous()
    n = A.shape[0]
    Li = torch.empty((n, n), dtype=F64, device=A.device)
    ldiag = torch.empty(n, dtype=F64, device=A.device)
    info = torch.empty(1, dtype=torch.int32, device=A.device)
    resid = torch.empty(1, dtype=F64, device=A.device)
    ws = workspace(query("vgposp_potrf_mixed_workspace_bytes", n))
    call("vgposp_potrf_mixed", _p(A), n, A.stride(0), _p(Li), Li.stride(0), _p(ldiag), int(iters),
         _p(resid), _p(info), _p(ws), ws.numel(), _stream())
    if check:
        check_info(info)
    return Li, ldiag, info, resid


def cholesky(A):
    """Return the lower Cholesky factor L (zeros above the diagonal) of a copy of A."""
    L = as_device(A).clone()
    cholesky_(L)
    return torch.tril(L)


def trsm(L, B, trans=False):
    """X = L^-1 B (trans=False) or L^-T B (trans=True) for a lower factor L [n, n] (upper triangle
    ignored) and B [n] or [n, m]; returns a new device tensor (tf.linalg.triangular_solve)."""
    L = as_device(L)
    X = as_device(B).clone()
    vec = X.dim() == 1
    X2 = X.reshape(-1, 1) if vec else X
    n = L.shape[-1]
    if L.dim() != 2 or L.shape[0] != n or X2.shape[0] != n:
        raise ValueError(f"trsm: L {tuple(L.shape)} and B {tuple(X.shape)} do not conform")
    if not L.is_contiguous():
        L = L.contiguous()
    ws = workspace(query("vgposp_trsm_workspace_bytes", n, X2.shape[1]))
    call("vgposp_trsm_lower", _p(L), n, L.stride(0), int(bool(trans)), _p(X2), X2.shape[1],
         X2.stride(0), _p(ws), ws.numel(), _stream())
    return X


def tri_inverse_from_factor(Minv):
    """Lower-triangular part of an in-place inverted factor."""
    return torch.tril(Minv)


def lml_from_inverse(Minv, ldiag, y, want_alpha=False):
    """LML[B] = -0.5|M y|^2 - sum log diag(L) - n/2 log 2pi (and alpha = C^-1 y)."""
    M3, _ = _batched(Minv)
    Bn, n = M3.shape[0], M3.shape[-1]
    y = as_device(y).reshape(-1)
    if y.numel() != n:
        raise ValueError(f"y has {y.numel()} entries, expected {n}")
    out = torch.empty(Bn, dtype=F64, device=M3.device)
    alpha = torch.empty((Bn, n), dtype=F64, device=M3.device) if want_alpha else None
    ws = workspace(query("vgposp_lml_workspace_bytes", n, Bn))
    call("vgposp_lml", _p(M3), n, M3.stride(1), M3.stride(0), Bn, _p(ldiag), _p(y), _p(alpha),
         _p(out), _p(ws), ws.numel(), _stream())
    return (out, alpha) if want_alpha else out


def inverse_from_factor_inverse(Minv):
    """C^-1 = M^T M from M = L^-1 (lower triangle of the result is filled; [B, n, n])."""
    M3, _ = _batched(Minv)
    Bn, n = M3.shape[0], M3.shape[-1]
    Q = torch.empty((Bn, n, n), dtype=F64, device=M3.device)
    for b in range(Bn):
        call("vgposp_gemm", 1, 0, n, n, n, 1.0, _p(M3[b]), M3.stride(1), _p(M3[b]), M3.stride(1),
             0.0, _p(Q[b]), Q.stride(1), LOWER, 1, 1, _stream())
    return Q


def lml_grad(kind, X, amp, ls, Cinv, alpha):
    """[B, 3] = dLML/d(amp, ls, noise) given C^-1 (lower triangle) and alpha = C^-1 y."""
    X = as_device(X)
    if X.dim() == 1:
        X = X[:, None]
    C3, _ = _batched(Cinv)
    Bn, n = C3.shape[0], C3.shape[-1]
    a, l = _vec(amp, Bn), _vec(ls, Bn)
    grad = torch.empty((Bn, 3), dtype=F64, device=C3.device)
    ws = workspace(query("vgposp_lml_grad_workspace_bytes", n, Bn))
    call("vgposp_lml_grad", kind_id(kind), _p(X), n, X.shape[1], _p(a), _p(l), _p(C3),
         C3.stride(1), C3.stride(0), _p(alpha), Bn, _p(grad), _p(ws), ws.numel(), _stream())
    return grad

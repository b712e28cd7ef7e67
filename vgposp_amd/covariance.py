"""Covariance builders that produce ``cov_vv`` on device.

The reference assembles cov_vv pair by pair in TF while loops:
* the empirical covariance of tracer samples per location (``main.py:125-350``);
* the VGP-predicted variant (``main_architecture_2_sampledistribution.py:423-542``);
* the beta-decay "local kernel" filter (``:361-421``).

Here each is one or two libvgposp launches:

* ``empirical_cov(T)``: centre every location's S samples (``vgposp_center_rows``), then one fp64
  MFMA SYRK.  The result is ``tfp.stats.covariance(t_i, t_j, sample_axis=0)`` for all pairs at
  once (biased, sample-mean centred; the reference's fixed standardisation
  ``(t - tr_mean) / tr_stdev`` only rescales by 1 / tr_stdev^2).
* ``vgp_tracer_samples(vgp, locations, tp_samples)``: the VGP predictive mean at every
  (location, temperature/pressure sample) 5-D point.  It uses the fused kernel-matrix-vector product
  ``vgposp_kernel_matvec``; K_*z is never materialised.
* ``index_taper_(C, COVER_spatial, beta)``: C[i][j] *= exp(-(beta delta_ij)^2 / (2 pi)), zeroed
  below 0.01.  delta_ij is the index-space distance on the C-order grid.
"""
from __future__ import annotations

import numpy as np
import torch

from . import linalg
from ._lib import FULL, LOWER, call
from .linalg import F64, _p, _stream, kind_id


def kernel_matvec(kind, X1, X2, amp, ls, v, out=None, beta=0.0):
    """out = K(X1, X2) v (+ beta out) for one kernel, K never formed."""
    X1, X2 = linalg.as_device(X1), linalg.as_device(X2)
    X1 = X1[:, None] if X1.dim() == 1 else X1
    X2 = X2[:, None] if X2.dim() == 1 else X2
    v = linalg.as_device(v).reshape(-1)
    if v.numel() != X2.shape[0] or X1.shape[1] != X2.shape[1]:
        raise ValueError("kernel_matvec: shapes do not match")
    if out is None:
        out = torch.zeros(X1.shape[0], dtype=F64, device=X1.device)
        beta = 0.0
    # parameter tensors held in locals until the launch: an inline temporary would be freed as
    # soon as _p() returned and its cached block reused by the next argument's upload
    a, l = linalg._vec(amp), linalg._vec(ls)
    call("vgposp_kernel_matvec", kind_id(kind), _p(X1), X1.shape[0], _p(X2), X2.shape[0],
         X1.shape[1], _p(a), _p(l), _p(v), float(beta), _p(out), _stream())
    return out


def center_rows_(T, scale=1.0):
    """In place: T[i] <- (T[i] - mean(T[i])) * scale (device [N, S])."""
    if T.dim() != 2 or T.stride(1) != 1:
        raise ValueError("T must be a row-major [N, S] device tensor")
    call("vgposp_center_rows", _p(T), T.shape[0], T.shape[1], T.stride(0), float(scale), _stream())
    return T


def empirical_cov(samples, tr_mean=0.0, tr_stdev=1.0, out=None):
    """cov_vv[i][j] = tfp.stats.covariance(t_i, t_j, sample_axis=0) with t = (T - tr_mean) / tr_stdev,
    for ``samples`` [N locations, S samples].  The input is copied, then centred in place."""
    T = linalg.as_device(samples).clone()
    if T.dim() != 2:
        raise ValueError("samples must be [N, S]")
    del tr_mean  # removed by the centring
    N, S = T.shape
    center_rows_(T, 1.0 / float(tr_stdev))
    if out is None:
        out = torch.empty((N, N), dtype=F64, device=T.device)
    # FULL output: C[i][j] and C[j][i] accumulate the same products in the same K order, so the
    # result is exactly symmetric
    linalg.gemm(T, T, out, alpha=1.0 / S, transb=True)
    return out


def index_taper_(C, COVER_spatial, beta, threshold=0.01, lower=False):
    """In place beta-decay local kernel filter (main_architecture_2_sampledistribution.py:361-421)."""
    I0, I1, I2 = (int(c) for c in COVER_spatial[:3])
    n = C.shape[-1]
    call("vgposp_index_taper", _p(C), n, C.stride(0), I0, I1, I2, float(beta), float(threshold),
         LOWER if lower else FULL, _stream())
    return C


def vgp_tracer_samples(vgp, locations, tp_samples, chunk_points=1 << 24):
    """T[i][s] = the VGP predictive mean at the 5-D point (locations[i], tp_samples[s])
    (main_architecture_2_sampledistribution.py:432-458, one vgp.mean() per point there)."""
    loc = linalg.as_device(locations)
    tp = linalg.as_device(tp_samples)
    loc = loc[:, None] if loc.dim() == 1 else loc
    tp = tp[:, None] if tp.dim() == 1 else tp
    N, S = loc.shape[0], tp.shape[0]
    w, mz_free = vgp.mean_weights()
    Z = linalg.as_device(vgp._Z())
    amp, ls = vgp.kernel.params()
    T = torch.empty((N, S), dtype=F64, device=loc.device)
    rows = max(1, chunk_points // S)
    for r0 in range(0, N, rows):
        r1 = min(N, r0 + rows)
        pts = torch.cat([loc[r0:r1, None, :].expand(r1 - r0, S, loc.shape[1]),
                         tp[None, :, :].expand(r1 - r0, S, tp.shape[1])], dim=2)
        pts = pts.reshape(-1, loc.shape[1] + tp.shape[1]).contiguous()
        kernel_matvec(vgp.kernel.kind, pts, Z, amp[0:1], ls[0:1], w, out=T[r0:r1].reshape(-1))
    if not mz_free:
        raise NotImplementedError("vgp_tracer_samples supports the zero mean function only")
    return T


def cov_vv_from_vgp(vgp, locations, tp_samples, tr_mean=0.0, tr_stdev=1.0):
    """The arch2 covariance: empirical covariance over the T/P samples of the VGP tracer field."""
    return empirical_cov(vgp_tracer_samples(vgp, locations, tp_samples), tr_mean, tr_stdev)


__all__ = ["kernel_matvec", "center_rows_", "empirical_cov", "index_taper_", "vgp_tracer_samples",
           "cov_vv_from_vgp"]

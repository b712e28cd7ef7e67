"""GP distributions with the ``tfp.distributions`` surface the reference uses, computed on MI355X.

* ``GaussianProcess``                  <- tfd.GaussianProcess (gp_functions.py:166-172)
* ``GaussianProcessRegressionModel``   <- tfd.GaussianProcessRegressionModel (gp_functions.py:283-297)
* ``VariationalGaussianProcess``       <- tfd.VariationalGaussianProcess
  (variational_Gaussian_process_example.py:68-99, main_architecture_2_sampledistribution.py:223-262)

Semantics restated from TFP ~0.7 (TF/TFP are not installed; see oracle/gp.py and DESIGN.md):
the marginal covariance is K + (noise + jitter) I with jitter = 1e-6 by default, parameters may be
batched (shape [B] -> a batch of B GPs), and ``log_prob`` of an [n] value returns [B].

All heavy operations run in libvgposp: kernel assembly, recursive Cholesky + triangular inverse,
MFMA GEMMs, the LML and its gradient.  Results are float64 device tensors; ``LogProb`` is an
array-like wrapper that also remembers how to re-evaluate itself (the eager counterpart of a TF1
graph tensor), which ``gp_functions.tf_train_gp_adam`` uses to build its training op.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import linalg
from .psd_kernels import _pts
from .variables import Placeholder, Softplus, Variable, fed, resolve

LOG_2PI = math.log(2.0 * math.pi)


def _as_obs(value, n):
    y = linalg.as_device(value).reshape(-1)
    if y.numel() != n:
        raise ValueError(f"observations have {y.numel()} entries, expected {n} (event shape)")
    return y


class LogProb:
    """Array-like result of ``log_prob`` (shape [B] or scalar) that can be re-evaluated."""

    def __init__(self, value, dist, observations):
        self.value = value
        self.dist = dist
        self.observations = observations

    def numpy(self):
        return self.value.detach().cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __getitem__(self, i):
        return self.numpy()[i]

    @property
    def shape(self):
        return tuple(self.value.shape)

    def __float__(self):
        return float(self.numpy().reshape(-1)[0])

    def __repr__(self):
        return f"LogProb({self.numpy()!r})"


class GaussianProcess:
    def __init__(self, kernel, index_points=None, mean_fn=None, observation_noise_variance=0.0,
                 jitter=1e-6, validate_args=False, allow_nan_stats=False,
                 name="GaussianProcess"):
        self.kernel = kernel
        self.index_points = index_points
        self.mean_fn = mean_fn
        self.observation_noise_variance = observation_noise_variance
        self.jitter = float(jitter)
        self.validate_args = validate_args
        self.name = name

    # -- shapes -------------------------------------------------------------------------------
    @property
    def batch_shape(self):
        return self.kernel.batch_shape

    @property
    def event_shape(self):
        return (int(_pts(self.index_points).shape[0]),)

    def _B(self):
        return self.kernel.batch_size

    def _noise(self):
        return resolve(self.observation_noise_variance, self._B())

    def _mean(self, X):
        n = int(_pts(X).shape[0])
        if self.mean_fn is None:
            return torch.zeros(n, dtype=torch.float64, device=linalg.device())
        return linalg.as_device(self.mean_fn(X)).reshape(-1)

    # -- factorization ------------------------------------------------------------------------
    def _factor_inverse(self, X):
        """C = K + (noise + jitter) I, lower(C) <- L^-1 in place; returns (Minv[B,n,n], diag(L))."""
        shift = self._noise() + self.jitter
        C = self.kernel.matrix(X, X, diag_shift=shift, lower=True, keep_batch=True)
        C, ldiag, _ = linalg.cholesky_(C, invert=True, check=True)
        return C, ldiag

    def _factor(self, X, extra_shift=0.0):
        shift = self._noise() + self.jitter + extra_shift
        C = self.kernel.matrix(X, X, diag_shift=shift, lower=True, keep_batch=True)
        C, ldiag, _ = linalg.cholesky_(C, invert=False, check=True)
        return C, ldiag

    # -- API ----------------------------------------------------------------------------------
    def log_prob(self, value, index_points=None):
        X = self.index_points if index_points is None else index_points
        n = int(_pts(X).shape[0])
        y = _as_obs(value, n) - self._mean(X)
        Minv, ldiag = self._factor_inverse(X)
        out = linalg.lml_from_inverse(Minv, ldiag, y)
        if self.batch_shape == ():
            out = out[0]
        return LogProb(out, self, value)

    def log_prob_and_grads(self, value, index_points=None):
        """(LML[B], dLML/damp[B], dLML/dls[B], dLML/dnoise[B]) on device."""
        X = self.index_points if index_points is None else index_points
        Xp = _pts(X)
        n = int(Xp.shape[0])
        y = _as_obs(value, n) - self._mean(X)
        Minv, ldiag = self._factor_inverse(X)
        lml, alpha = linalg.lml_from_inverse(Minv, ldiag, y, want_alpha=True)
        Q = linalg.inverse_from_factor_inverse(Minv)
        amp, ls = self.kernel.params()
        g = linalg.lml_grad(self.kernel.kind, Xp, amp, ls, Q, alpha)
        return lml, g[:, 0], g[:, 1], g[:, 2]

    def mean(self, index_points=None):
        X = self.index_points if index_points is None else index_points
        m = self._mean(X)
        return m.expand(self._B(), -1) if self.batch_shape != () else m

    def covariance(self, index_points=None):
        X = self.index_points if index_points is None else index_points
        C = self.kernel.matrix(X, X, diag_shift=self._noise(), keep_batch=True)
        return C if self.batch_shape != () else C[0]

    def variance(self, index_points=None):
        return torch.diagonal(self.covariance(index_points), dim1=-2, dim2=-1)

    def stddev(self, index_points=None):
        return torch.sqrt(self.variance(index_points))

    def sample(self, sample_shape=(), seed=None, index_points=None):
        X = self.index_points if index_points is None else index_points
        L, _ = self._factor(X)
        return _mvn_sample(self.mean(X), L, sample_shape, seed, self.batch_shape != ())


def _mvn_sample(mean, L, sample_shape, seed, batched):
    """mean + L z,  z ~ N(0, I): [S] + batch + [n] (L lower, upper garbage ignored)."""
    S = int(np.prod(sample_shape)) if sample_shape not in ((), None) else 1
    B, n = L.shape[0], L.shape[-1]
    gen = torch.Generator(device=L.device)
    if seed is not None:
        gen.manual_seed(int(seed))
    else:
        gen.seed()
    z = torch.randn((B, n, S), generator=gen, dtype=torch.float64, device=L.device)
    out = torch.empty((B, n, S), dtype=torch.float64, device=L.device)
    mean = mean.reshape(-1, n) if mean.dim() > 1 else mean.reshape(1, n).expand(B, n)
    for b in range(B):
        out[b].copy_(mean[b].reshape(n, 1).expand(n, S))
        linalg.gemm(L[b], z[b], out[b], alpha=1.0, beta=1.0, tri_a=True)
    out = out.permute(2, 0, 1)  # [S, B, n]
    if not batched:
        out = out[:, 0]
    if sample_shape in ((), None):
        out = out[0]
    else:
        out = out.reshape(tuple(np.atleast_1d(sample_shape)) + tuple(out.shape[1:]))
    return out


class GaussianProcessRegressionModel(GaussianProcess):
    """Posterior predictive of an exact GP:  C = K_xx + (noise + jitter) I,
    mean = m(X*) + K_*x C^-1 (y - m(X)),  cov = K_** - K_*x C^-1 K_x* + pred_noise I."""

    def __init__(self, kernel, index_points=None, observation_index_points=None, observations=None,
                 observation_noise_variance=0.0, predictive_noise_variance=None, mean_fn=None,
                 jitter=1e-6, validate_args=False, allow_nan_stats=False,
                 name="GaussianProcessRegressionModel"):
        super().__init__(kernel, index_points, mean_fn, observation_noise_variance, jitter,
                         validate_args, allow_nan_stats, name)
        self.observation_index_points = observation_index_points
        self.observations = observations
        self.predictive_noise_variance = (observation_noise_variance if predictive_noise_variance
                                          is None else predictive_noise_variance)

    def _posterior(self, want_cov=True):
        X = self.observation_index_points
        Xs = self.index_points
        n = int(_pts(X).shape[0])
        y = _as_obs(self.observations, n) - self._mean(X)
        Minv, ldiag = self._factor_inverse(X)
        _, alpha = linalg.lml_from_inverse(Minv, ldiag, y, want_alpha=True)
        Ksx = self.kernel.matrix(Xs, X, keep_batch=True)  # [B, M, n]
        B, M = Ksx.shape[0], Ksx.shape[1]
        mean = torch.empty((B, M), dtype=torch.float64, device=Ksx.device)
        for b in range(B):
            linalg.gemm(Ksx[b], alpha[b].reshape(n, 1), mean[b].reshape(M, 1))
        mean = mean + self._mean(Xs)
        if not want_cov:
            return mean, None
        pn = resolve(self.predictive_noise_variance, B)
        cov = self.kernel.matrix(Xs, Xs, diag_shift=pn, keep_batch=True)
        V = torch.empty((B, M, n), dtype=torch.float64, device=Ksx.device)
        for b in range(B):
            # V = K_*x M^T  (M = L^-1 lower, stored [j][k]);  cov -= V V^T
            linalg.gemm(Ksx[b], Minv[b], V[b], transb=True, tri_b=True)
            linalg.gemm(V[b], V[b], cov[b], alpha=-1.0, beta=1.0, transb=True)
        return mean, cov

    def mean(self, index_points=None):
        m, _ = self._posterior(want_cov=False)
        return m if self.batch_shape != () else m[0]

    def covariance(self, index_points=None):
        _, c = self._posterior()
        return c if self.batch_shape != () else c[0]

    def sample(self, sample_shape=(), seed=None, index_points=None):
        mean, cov = self._posterior()
        B, M = cov.shape[0], cov.shape[-1]
        cov.diagonal(dim1=-2, dim2=-1).add_(self.jitter)
        L, _, _ = linalg.cholesky_(cov, invert=False, check=True)
        return _mvn_sample(mean, L, sample_shape, seed, self.batch_shape != ())

    def log_prob(self, value, index_points=None):
        mean, cov = self._posterior()
        M = cov.shape[-1]
        cov.diagonal(dim1=-2, dim2=-1).add_(self.jitter)
        Minv, ldiag, _ = linalg.cholesky_(cov, invert=True, check=True)
        y = _as_obs(value, M)
        out = torch.stack([linalg.lml_from_inverse(Minv[b:b + 1], ldiag[b:b + 1], y - mean[b])[0]
                           for b in range(cov.shape[0])])
        if self.batch_shape == ():
            out = out[0]
        return LogProb(out, self, value)


class VariationalGaussianProcess(GaussianProcess):
    """Sparse variational GP with inducing points Z (TFP ~0.7 semantics).

    ``variational_inducing_observations_scale`` is used as a full matrix A with S = A A^T for the
    KL term and the predictive covariance; the trace term of ``variational_loss`` follows TFP 0.7's
    ``scale.matmul(kzz_inv_kzx)`` (i.e. ||A Kzz^-1 Kzx||_F^2) unless ``trace_adjoint=True``
    (||A^T Kzz^-1 Kzx||_F^2, the later TFP fix) — unpinned by any reference test.
    """

    def __init__(self, kernel, index_points, inducing_index_points,
                 variational_inducing_observations_loc, variational_inducing_observations_scale,
                 mean_fn=None, observation_noise_variance=0.0, predictive_noise_variance=None,
                 jitter=1e-6, validate_args=False, allow_nan_stats=False, trace_adjoint=False,
                 name="VariationalGaussianProcess"):
        super().__init__(kernel, index_points, mean_fn, observation_noise_variance, jitter,
                         validate_args, allow_nan_stats, name)
        self.inducing_index_points = inducing_index_points
        self.variational_loc = variational_inducing_observations_loc
        self.variational_scale = variational_inducing_observations_scale
        self.predictive_noise_variance = (observation_noise_variance if predictive_noise_variance
                                          is None else predictive_noise_variance)
        self.trace_adjoint = trace_adjoint

    # -- helpers --------------------------------------------------------------------------------
    def _Z(self):
        Z = self.inducing_index_points
        return Z.value if isinstance(Z, Variable) else Z

    def _loc_scale(self):
        B = self._B()
        loc, scale = self.variational_loc, self.variational_scale
        spec = getattr(loc, "_vgposp_posterior", None)
        if spec is not None and getattr(scale, "_vgposp_posterior", None) is spec:
            # the reference's loc / scale are graph tensors of optimal_variational_posterior:
            # re-evaluate them with the current parameter values, as every sess.run does
            loc, scale = VariationalGaussianProcess.optimal_variational_posterior(**spec)
        loc = linalg.as_device(loc)
        scale = linalg.as_device(scale)
        M = scale.shape[-1]
        loc = loc.reshape(-1, M).expand(B, M).contiguous() if loc.numel() in (M, B * M) else loc
        scale = scale.reshape(-1, M, M).expand(B, M, M).contiguous()
        return loc, scale

    def _kzz_factor(self):
        """Lz^-1 with Lz = chol(Kzz + jitter I) (lower triangles), and the [B, M, M] inverse."""
        Z = self._Z()
        Kzz = self.kernel.matrix(Z, Z, diag_shift=self.jitter, lower=True, keep_batch=True)
        Lzinv, ldiag, _ = linalg.cholesky_(Kzz, invert=True, check=True)
        return Lzinv, ldiag

    @staticmethod
    def optimal_variational_posterior(kernel, inducing_index_points, observation_index_points,
                                      observations, observation_noise_variance, mean_fn=None,
                                      jitter=1e-6, name=None):
        """Titsias' optimal q(u): Sigma^-1 = Kzz + noise^-1 Kzx Kxz (+ jitter I),
        loc = m(Z) + noise^-1 Kzz Sigma (Kzx (y - m(X))),  scale = chol(Sigma^-1)^-1 Kzz.
        The Kzx Kxz contraction (2 M^2 N flops) is the fp64 MFMA hot spot."""
        Z = inducing_index_points.value if isinstance(inducing_index_points, Variable) else inducing_index_points
        X = observation_index_points
        B = kernel.batch_size
        noise = resolve(observation_noise_variance, B)
        N = int(_pts(X).shape[0])
        y = linalg.as_device(observations).reshape(-1)
        if y.numel() != N:
            raise ValueError("observations do not match observation_index_points")
        if mean_fn is not None:
            y = y - linalg.as_device(mean_fn(X)).reshape(-1)
        Kzz = kernel.matrix(Z, Z, keep_batch=True)                 # [B, M, M]
        Kzx = kernel.matrix(Z, X, keep_batch=True)                 # [B, M, N]
        M = Kzz.shape[-1]
        Sinv = Kzz.clone()
        Sinv.diagonal(dim1=-2, dim2=-1).add_(jitter)
        kzx_y = torch.empty((B, M), dtype=torch.float64, device=Kzz.device)
        for b in range(B):
            inv_noise = float(1.0 / noise[b])
            linalg.gemm(Kzx[b], Kzx[b], Sinv[b], alpha=inv_noise, beta=1.0, transb=True, lower_c=True)
            linalg.gemm(Kzx[b], y.reshape(N, 1), kzx_y[b].reshape(M, 1))
        Linv, ldiag, _ = linalg.cholesky_(Sinv, invert=True, check=True)   # Linv = chol(Sinv)^-1
        loc = torch.empty((B, M), dtype=torch.float64, device=Kzz.device)
        scale = torch.empty((B, M, M), dtype=torch.float64, device=Kzz.device)
        tmp = torch.empty((M, 1), dtype=torch.float64, device=Kzz.device)
        for b in range(B):
            # Sigma (Kzx y) = Linv^T Linv (Kzx y)
            v = linalg.gemm(Linv[b], kzx_y[b].reshape(M, 1), tri_a=True)
            linalg.gemm(Linv[b], v, tmp, transa=True, tri_a=True)
            linalg.gemm(Kzz[b], tmp, loc[b].reshape(M, 1), alpha=float(1.0 / noise[b]))
            linalg.gemm(Linv[b], Kzz[b], scale[b], tri_a=True)
        if mean_fn is not None:
            loc = loc + linalg.as_device(mean_fn(Z)).reshape(1, -1)
        if kernel.batch_shape == ():
            loc, scale = loc[0], scale[0]
        # remember how these were made, so a VGP built on them re-evaluates them when the kernel
        # parameters / inducing points change (and VGPTrainOp can differentiate through them)
        spec = dict(kernel=kernel, inducing_index_points=inducing_index_points,
                    observation_index_points=observation_index_points, observations=observations,
                    observation_noise_variance=observation_noise_variance, mean_fn=mean_fn,
                    jitter=jitter)
        loc._vgposp_posterior = spec
        scale._vgposp_posterior = spec
        return loc, scale

    def variational_loss(self, observations, observation_index_points=None, kl_weight=1.0,
                         name="variational_loss"):
        """Negative ELBO averaged over the kernel batch (TFP ~0.7 variational_loss).  Returns a
        ``VariationalLoss``: evaluated now when its inputs are concrete, re-evaluable through
        ``Session.run`` (placeholders fed), and trainable with ``AdamOptimizer.minimize``."""
        return VariationalLoss(self, observations, observation_index_points, kl_weight)

    def _variational_loss_value(self, observations, observation_index_points=None, kl_weight=1.0):
        Xb = self.index_points if observation_index_points is None else observation_index_points
        Z = self._Z()
        B = self._B()
        noise = self._noise()
        nb = int(_pts(Xb).shape[0])
        y = _as_obs(observations, nb) - self._mean(Xb)
        loc, scale = self._loc_scale()
        M = scale.shape[-1]
        mz = self._mean(Z)
        Lzinv, lzdiag = self._kzz_factor()
        Kzx = self.kernel.matrix(Z, Xb, keep_batch=True)           # [B, M, nb]
        amp, _ = self.kernel.params()
        # KL prior p(u) = N(m(Z), Kzz + (noise + 1e-6) I)  (TFP GaussianProcess default jitter)
        Kp = self.kernel.matrix(Z, Z, diag_shift=noise + 1e-6, lower=True, keep_batch=True)
        Lpinv, lpdiag, _ = linalg.cholesky_(Kp, invert=True, check=True)
        out = []
        for b in range(B):
            Lzi = Lzinv[b]
            # Kzz^-1 (m - m(Z))
            d = (loc[b] - mz).reshape(M, 1)
            w = linalg.gemm(Lzi, d, tri_a=True)
            kinv_loc = linalg.gemm(Lzi, w, transa=True, tri_a=True)
            pred = linalg.gemm(Kzx[b], kinv_loc, transa=True).reshape(-1)   # Kxz Kzz^-1 m
            s2 = noise[b] + self.jitter
            r = y - pred
            obs_ll = -0.5 * torch.sum(r * r) / s2 - 0.5 * nb * (LOG_2PI + torch.log(s2))
            G = linalg.gemm(Lzi, Kzx[b], tri_a=True)                        # Lz^-1 Kzx
            H = linalg.gemm(Lzi, G, transa=True, tri_a=True)                # Kzz^-1 Kzx
            ktilde = nb * amp[b] ** 2 - torch.sum(G * G)
            AH = linalg.gemm(scale[b], H, transa=self.trace_adjoint)
            other = torch.sum(AH * AH)
            trace_term = 0.5 * (ktilde + other) / noise[b]
            # KL(N(m, A A^T) || N(m(Z), Lp Lp^T))
            P = linalg.gemm(Lpinv[b], scale[b], tri_a=True)                 # Lp^-1 A
            q = linalg.gemm(Lpinv[b], (mz - loc[b]).reshape(M, 1), tri_a=True)
            AtA = linalg.gemm(scale[b], scale[b], transa=True)
            _, ad, _ = linalg.cholesky_(AtA, invert=False, check=True)
            logdet_A = torch.sum(torch.log(ad))                              # 0.5 log det(A^T A)
            kl = (torch.sum(torch.log(lpdiag[b])) - logdet_A
                  + 0.5 * (-M + torch.sum(P * P) + torch.sum(q * q)))
            out.append(obs_ll - trace_term - kl_weight * kl)
        return -torch.mean(torch.stack(out))

    def mean_weights(self):
        """(w = Kzz^-1 (loc - m(Z)) [M] for kernel batch entry 0, zero-mean flag): the predictive
        mean is K(x*, Z) w (+ m(x*)), which vgposp_kernel_matvec evaluates without forming K."""
        loc, _ = self._loc_scale()
        M = loc.shape[-1]
        Lzinv, _ = self._kzz_factor()
        d = (loc[0] - self._mean(self._Z())).reshape(M, 1)
        w = linalg.gemm(Lzinv[0], linalg.gemm(Lzinv[0], d, tri_a=True), transa=True, tri_a=True)
        return w.reshape(-1), self.mean_fn is None

    def _predictive(self, want_cov=True):
        Xs = self.index_points
        Z = self._Z()
        B = self._B()
        loc, scale = self._loc_scale()
        M = scale.shape[-1]
        mz = self._mean(Z)
        Lzinv, _ = self._kzz_factor()
        Ksz = self.kernel.matrix(Xs, Z, keep_batch=True)          # [B, P, M]
        P = Ksz.shape[1]
        mean = torch.empty((B, P), dtype=torch.float64, device=Ksz.device)
        covs = []
        for b in range(B):
            d = (loc[b] - mz).reshape(M, 1)
            w = linalg.gemm(Lzinv[b], d, tri_a=True)
            kinv_loc = linalg.gemm(Lzinv[b], w, transa=True, tri_a=True)
            linalg.gemm(Ksz[b], kinv_loc, mean[b].reshape(P, 1))
            if want_cov:
                # cov = K** - Q** + K*z Kzz^-1 A A^T Kzz^-1 Kz*  (+ predictive noise)
                V = linalg.gemm(Ksz[b], Lzinv[b], transb=True, tri_b=True)   # K*z Lz^-T
                T = linalg.gemm(Lzinv[b], V.t().contiguous(), transa=True, tri_a=True)  # Kzz^-1 Kz*
                U = linalg.gemm(scale[b], T, transa=True)                     # A^T Kzz^-1 Kz*
                pn = resolve(self.predictive_noise_variance, B)[b:b + 1]
                C = self.kernel.matrix(Xs, Xs, diag_shift=pn, keep_batch=True)[b if self.kernel.batch_size > 1 else 0]
                linalg.gemm(V, V, C, alpha=-1.0, beta=1.0, transb=True)
                linalg.gemm(U, U, C, alpha=1.0, beta=1.0, transa=True)
                covs.append(C)
        mean = mean + self._mean(Xs)
        return mean, (torch.stack(covs) if want_cov else None)

    def mean(self, index_points=None):
        m, _ = self._predictive(want_cov=False)
        return m if self.batch_shape != () else m[0]

    def covariance(self, index_points=None):
        _, c = self._predictive()
        return c if self.batch_shape != () else c[0]

    def sample(self, sample_shape=(), seed=None, index_points=None):
        mean, cov = self._predictive()
        cov.diagonal(dim1=-2, dim2=-1).add_(self.jitter)
        L, _, _ = linalg.cholesky_(cov, invert=False, check=True)
        return _mvn_sample(mean, L, sample_shape, seed, self.batch_shape != ())


class VariationalLoss:
    """Array-like scalar -ELBO of a VGP (the eager counterpart of the TF1 loss tensor)."""

    def __init__(self, vgp, observations, observation_index_points, kl_weight):
        self.vgp = vgp
        self.observations = observations
        self.observation_index_points = observation_index_points
        self.kl_weight = float(kl_weight)
        concrete = not any(isinstance(x, Placeholder)
                           for x in (observations, observation_index_points))
        self.value = self.evaluate() if concrete else None

    def inputs(self, feed=None):
        return fed(self.observations, feed), fed(self.observation_index_points, feed)

    def evaluate(self, feed=None):
        yb, Xb = self.inputs(feed)
        self.value = self.vgp._variational_loss_value(yb, Xb, self.kl_weight)
        return self.value

    def numpy(self):
        if self.value is None:
            raise ValueError("variational_loss has unfed placeholders: evaluate it with "
                             "Session.run(loss, feed_dict=...)")
        return self.value.detach().cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __float__(self):
        return float(self.numpy())

    def item(self):
        return float(self)

    def __repr__(self):
        return f"VariationalLoss({self.value!r})"


__all__ = ["GaussianProcess", "GaussianProcessRegressionModel", "VariationalGaussianProcess",
           "LogProb", "VariationalLoss", "Softplus", "Variable"]

"""Oracle (TEST INFRASTRUCTURE ONLY): numpy restatement of the TFP (~0.7) GP semantics the
reference reaches through ``gp_functions.py``.

TF / TFP are not installed here and are un-vendored in the reference, so this is a restatement of
TFP's documented / published algorithms, anchored on the reference's call sites:

* PSD kernels (``tfkern.ExponentiatedQuadratic`` ``3D_sin_wave.py:158-159``,
  ``main_tests.py:617-619``; ``MaternOneHalf`` ``gp_functions.py:160-163``;
  ``MaternFiveHalves`` ``main_architecture_2_sampledistribution.py:211``): TFP evaluates
  ``exp(2*log(amp) + log_k(r/ls))``; reproduced here in that form.
* ``tfd.GaussianProcess(...).log_prob`` (``gp_functions.py:166-172``, ``main.py:105``): MVN with
  ``scale = chol(K + (noise + jitter) I)``, jitter default 1e-6.  Cross-checked against
  scikit-learn's ``log_marginal_likelihood`` (alpha = noise + jitter) in tests.
* ``tf_Variable`` constraint ``tiny + softplus(v)`` (``gp_functions.py:124-135``).
* TF1 ``AdamOptimizer`` (``gp_functions.py:179-182``): lr_t = lr*sqrt(1-b2^t)/(1-b1^t),
  theta -= lr_t * m / (sqrt(v) + eps).
* ``GaussianProcessRegressionModel`` (``gp_functions.py:283-297``) and
  ``VariationalGaussianProcess`` (``variational_Gaussian_process_example.py:68-99``).

Parity at the TFP boundary is UNPINNED (no reference test holds numbers there); see DESIGN.md.
"""
from __future__ import annotations

import numpy as np

TINY = np.finfo(np.float64).tiny
LOG_2PI = np.log(2.0 * np.pi)

KERNELS = ("eq", "matern12", "matern32", "matern52")


def softplus(v):
    v = np.asarray(v, dtype=np.float64)
    return np.where(v > 30, v, np.log1p(np.exp(np.minimum(v, 30))))


def sigmoid(v):
    return 1.0 / (1.0 + np.exp(-np.asarray(v, dtype=np.float64)))


def constrain(v):
    """gp_functions.py:132-134: tiny + softplus(v)."""
    return TINY + softplus(v)


def invert_softplus(x):
    """gp_functions.py:106-109: v = log(exp(x) - 1)."""
    return np.log(np.exp(np.asarray(x, dtype=np.float64)) - 1)


def sqdist(X1, X2):
    X1 = np.asarray(X1, dtype=np.float64)
    X2 = np.asarray(X2, dtype=np.float64)
    if X1.ndim == 1:
        X1 = X1[:, None]
    if X2.ndim == 1:
        X2 = X2[:, None]
    return np.sum((X1[:, None, :] - X2[None, :, :]) ** 2, axis=-1)


def _log_k(kind, d2, ls):
    if kind == "eq":
        return -0.5 * d2 / ls ** 2
    r = np.sqrt(d2) / ls
    if kind == "matern12":
        return -r
    if kind == "matern32":
        s = np.sqrt(3.0) * r
        return np.log1p(s) - s
    if kind == "matern52":
        s = np.sqrt(5.0) * r
        return np.log1p(s + s ** 2 / 3.0) - s
    raise ValueError(kind)


def kernel_matrix(kind, X1, X2, amp, ls):
    """K[b, i, j] = exp(2 log amp_b + log_k(|x1_i - x2_j| / ls_b)); amp/ls broadcast to [B]."""
    amp = np.atleast_1d(np.asarray(amp, dtype=np.float64))
    ls = np.atleast_1d(np.asarray(ls, dtype=np.float64))
    amp, ls = np.broadcast_arrays(amp, ls)
    d2 = sqdist(X1, X2)
    return np.stack([np.exp(2.0 * np.log(a) + _log_k(kind, d2, l)) for a, l in zip(amp, ls)])


def kernel_matrix_grads(kind, X1, X2, amp, ls):
    """(dK/damp, dK/dls) per batch entry, [B, n, m] each."""
    amp = np.atleast_1d(np.asarray(amp, dtype=np.float64))
    ls = np.atleast_1d(np.asarray(ls, dtype=np.float64))
    amp, ls = np.broadcast_arrays(amp, ls)
    d2 = sqdist(X1, X2)
    r0 = np.sqrt(d2)
    dA, dL = [], []
    for a, l in zip(amp, ls):
        K = np.exp(2.0 * np.log(a) + _log_k(kind, d2, l))
        dA.append(2.0 * K / a)
        r = r0 / l
        if kind == "eq":
            dL.append(K * d2 / l ** 3)
        elif kind == "matern12":
            dL.append(K * r / l)
        elif kind == "matern32":
            s = np.sqrt(3.0) * r
            dL.append(a ** 2 * np.exp(-s) * s * s / l)
        elif kind == "matern52":
            s = np.sqrt(5.0) * r
            dL.append(a ** 2 * np.exp(-s) * (s * s / 3.0) * (1.0 + s) / l)
        else:
            raise ValueError(kind)
    return np.stack(dA), np.stack(dL)


def gp_log_prob(kind, X, y, amp, ls, noise, jitter=1e-6):
    """tfd.GaussianProcess(kernel, X, noise).log_prob(y) -> [B]."""
    K = kernel_matrix(kind, X, X, amp, ls)
    n = K.shape[-1]
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    out = []
    for Kb in K:
        C = Kb + (noise + jitter) * np.eye(n)
        L = np.linalg.cholesky(C)
        z = np.linalg.solve(L, y)
        out.append(-0.5 * z @ z - np.sum(np.log(np.diag(L))) - 0.5 * n * LOG_2PI)
    return np.array(out)


def gp_log_prob_and_grads(kind, X, y, amp, ls, noise, jitter=1e-6):
    """LML[B] and its gradient w.r.t. amp[B], ls[B] and the (shared) noise variance:
    dLML/dtheta = 0.5 * sum_ij (alpha alpha^T - C^-1)_ij dC_ij/dtheta."""
    K = kernel_matrix(kind, X, X, amp, ls)
    dA, dL = kernel_matrix_grads(kind, X, X, amp, ls)
    n = K.shape[-1]
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    lml, ga, gl, gn = [], [], [], []
    for b in range(K.shape[0]):
        C = K[b] + (noise + jitter) * np.eye(n)
        L = np.linalg.cholesky(C)
        z = np.linalg.solve(L, y)
        Linv = np.linalg.inv(L)
        Q = Linv.T @ Linv
        alpha = Q @ y
        G = np.outer(alpha, alpha) - Q
        lml.append(-0.5 * z @ z - np.sum(np.log(np.diag(L))) - 0.5 * n * LOG_2PI)
        ga.append(0.5 * np.sum(G * dA[b]))
        gl.append(0.5 * np.sum(G * dL[b]))
        gn.append(0.5 * np.trace(G))
    return np.array(lml), np.array(ga), np.array(gl), np.array(gn)


class AdamTF1:
    """tf.train.AdamOptimizer (TF1) on a flat float64 parameter vector."""

    def __init__(self, lr, beta1=0.9, beta2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.m = self.v = None
        self.t = 0

    def step(self, theta, grad):
        if self.m is None:
            self.m = np.zeros_like(theta)
            self.v = np.zeros_like(theta)
        self.t += 1
        lr_t = self.lr * np.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        self.m = self.b1 * self.m + (1 - self.b1) * grad
        self.v = self.b2 * self.v + (1 - self.b2) * grad * grad
        return theta - lr_t * self.m / (np.sqrt(self.v) + self.eps)


def fit_gp_adam(kind, X, y, v_amp, v_ls, v_noise, lr, num_iters, jitter=1e-6):
    """gp_functions.tf_train_gp_adam + tf_optimize_model_params (gp_functions.py:179-182, 228-259):
    minimise -sum_b LML_b over the pre-softplus variables; one warm-up step (:248-250) then
    num_iters+1 logged steps; lls[i] is the pre-update LML.  Returns (lls[num_iters+1, B], v)."""
    v_amp = np.atleast_1d(np.asarray(v_amp, dtype=np.float64)).copy()
    v_ls = np.atleast_1d(np.asarray(v_ls, dtype=np.float64)).copy()
    B = max(v_amp.size, v_ls.size)
    v_amp = np.broadcast_to(v_amp, (B,)).copy()
    v_ls = np.broadcast_to(v_ls, (B,)).copy()
    theta = np.concatenate([v_amp, v_ls, [float(v_noise)]])
    opt = AdamTF1(lr)
    lls = np.zeros([num_iters + 1, B])

    def step():
        nonlocal theta
        va, vl, vn = theta[:B], theta[B:2 * B], theta[2 * B]
        amp, ls, noise = constrain(va), constrain(vl), constrain(vn)
        lml, ga, gl, gn = gp_log_prob_and_grads(kind, X, y, amp, ls, noise, jitter)
        # loss = -sum_b LML_b ; chain rule through tiny + softplus
        g = -np.concatenate([ga * sigmoid(va), gl * sigmoid(vl), [np.sum(gn) * sigmoid(vn)]])
        theta = opt.step(theta, g)
        return lml

    step()
    for i in range(num_iters + 1):
        lls[i] = step()
    return lls, theta


def gprm_mean_cov(kind, Xs, X, y, amp, ls, noise, pred_noise=0.0, jitter=1e-6):
    """GaussianProcessRegressionModel: mean[B, M] and covariance[B, M, M] (without the sampling
    jitter):  C = K_xx + (noise + jitter) I; mean = K_sx C^-1 y;
    cov = K_ss - K_sx C^-1 K_xs + pred_noise I."""
    Kxx = kernel_matrix(kind, X, X, amp, ls)
    Ksx = kernel_matrix(kind, Xs, X, amp, ls)
    Kss = kernel_matrix(kind, Xs, Xs, amp, ls)
    n = Kxx.shape[-1]
    M = Kss.shape[-1]
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    means, covs = [], []
    for b in range(Kxx.shape[0]):
        L = np.linalg.cholesky(Kxx[b] + (noise + jitter) * np.eye(n))
        A = np.linalg.solve(L, Ksx[b].T)
        z = np.linalg.solve(L, y)
        means.append(A.T @ z)
        covs.append(Kss[b] - A.T @ A + pred_noise * np.eye(M))
    return np.stack(means), np.stack(covs)


def calc_H(kind, X, y, noise, XEDGES, YEDGES, jitter=1e-6, scale=40.0):
    """gp_functions.calc_H (gp_functions.py:864-876): LML[0] on the grid
    ls = scale*(1+i)/XEDGES, amp = scale*(1+j)/YEDGES."""
    H = np.zeros([XEDGES, YEDGES])
    for i in range(XEDGES):
        for j in range(YEDGES):
            ls = scale * np.double((1 + i) / XEDGES)
            amp = scale * np.double((1 + j) / YEDGES)
            H[i, j] = gp_log_prob(kind, X, y, [amp], [ls], noise, jitter)[0]
    return H


def vgp_optimal_posterior(kind, Z, X, y, amp, ls, noise, jitter=1e-6):
    """Titsias optimal q(u) (TFP ~0.7 optimal_variational_posterior), kernel batch [B]."""
    Kzz = kernel_matrix(kind, Z, Z, amp, ls)
    Kzx = kernel_matrix(kind, Z, X, amp, ls)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    locs, scales = [], []
    for b in range(Kzz.shape[0]):
        M = Kzz.shape[-1]
        Sinv = Kzz[b] + Kzx[b] @ Kzx[b].T / noise + jitter * np.eye(M)
        L = np.linalg.cholesky(Sinv)
        v = np.linalg.solve(L.T, np.linalg.solve(L, Kzx[b] @ y))
        locs.append(Kzz[b] @ v / noise)
        scales.append(np.linalg.solve(L, Kzz[b]))
    return np.stack(locs), np.stack(scales)


def vgp_variational_loss(kind, Z, Xb, yb, loc, scale, amp, ls, noise, kl_weight, jitter=1e-6,
                         trace_adjoint=False):
    """Negative ELBO averaged over the kernel batch (TFP ~0.7 variational_loss restated)."""
    amp = np.atleast_1d(np.asarray(amp, dtype=np.float64))
    ls = np.atleast_1d(np.asarray(ls, dtype=np.float64))
    amp, ls = np.broadcast_arrays(amp, ls)
    Kzz = kernel_matrix(kind, Z, Z, amp, ls)
    Kzx = kernel_matrix(kind, Z, Xb, amp, ls)
    yb = np.asarray(yb, dtype=np.float64).reshape(-1)
    nb = yb.size
    M = Kzz.shape[-1]
    loc = np.asarray(loc).reshape(-1, M)
    scale = np.asarray(scale).reshape(-1, M, M)
    out = []
    for b in range(Kzz.shape[0]):
        lo = loc[b if loc.shape[0] > 1 else 0]
        A = scale[b if scale.shape[0] > 1 else 0]
        Lz = np.linalg.cholesky(Kzz[b] + jitter * np.eye(M))
        kinv_loc = np.linalg.solve(Lz.T, np.linalg.solve(Lz, lo))
        pred = Kzx[b].T @ kinv_loc
        s2 = noise + jitter
        obs_ll = np.sum(-0.5 * (yb - pred) ** 2 / s2 - 0.5 * np.log(2 * np.pi * s2))
        G = np.linalg.solve(Lz, Kzx[b])
        H = np.linalg.solve(Lz.T, G)
        ktilde = nb * amp[b] ** 2 - np.sum(G ** 2)
        AH = (A.T if trace_adjoint else A) @ H
        trace_term = 0.5 * (ktilde + np.sum(AH ** 2)) / noise
        Lp = np.linalg.cholesky(Kzz[b] + (noise + 1e-6) * np.eye(M))
        P = np.linalg.solve(Lp, A)
        q = np.linalg.solve(Lp, -lo)
        kl = (np.sum(np.log(np.diag(Lp))) - np.linalg.slogdet(A)[1]
              + 0.5 * (-M + np.sum(P ** 2) + np.sum(q ** 2)))
        out.append(obs_ll - trace_term - kl_weight * kl)
    return -np.mean(out)


def vgp_predictive(kind, Xs, Z, loc, scale, amp, ls, pred_noise, jitter=1e-6):
    """VGP posterior predictive mean [B, P] and covariance [B, P, P]."""
    Kzz = kernel_matrix(kind, Z, Z, amp, ls)
    Ksz = kernel_matrix(kind, Xs, Z, amp, ls)
    Kss = kernel_matrix(kind, Xs, Xs, amp, ls)
    M = Kzz.shape[-1]
    loc = np.asarray(loc).reshape(-1, M)
    scale = np.asarray(scale).reshape(-1, M, M)
    means, covs = [], []
    for b in range(Kzz.shape[0]):
        lo = loc[b if loc.shape[0] > 1 else 0]
        A = scale[b if scale.shape[0] > 1 else 0]
        Lz = np.linalg.cholesky(Kzz[b] + jitter * np.eye(M))
        T = np.linalg.solve(Lz.T, np.linalg.solve(Lz, Ksz[b].T))   # Kzz^-1 Kz*
        means.append(T.T @ lo)
        V = np.linalg.solve(Lz, Ksz[b].T)
        U = A.T @ T
        covs.append(Kss[b] - V.T @ V + U.T @ U + pred_noise * np.eye(Kss.shape[-1]))
    return np.stack(means), np.stack(covs)


# ---------------------------------------------------------------------------------------------
# VGP training objective of variational_Gaussian_process_example.py:51-102: the minibatch
# variational_loss of a VGP whose q(u) is optimal_variational_posterior over the FULL data,
# differentiated w.r.t. (amp, ls, noise, Z).  The analytic gradient below is checked against
# central finite differences of vgp_training_loss in tests/test_gp_oracle.py.
# ---------------------------------------------------------------------------------------------
def vgp_training_loss(kind, Z, X, y, Xb, yb, amp, ls, noise, kl_weight, jitter=1e-6,
                      trace_adjoint=False):
    loc, scale = vgp_optimal_posterior(kind, Z, X, y, amp, ls, noise, jitter)
    return vgp_variational_loss(kind, Z, Xb, yb, loc, scale, amp, ls, noise, kl_weight, jitter,
                                trace_adjoint)


def kernel_vjp(kind, X1, X2, amp, ls, Kbar):
    """sum_ij Kbar_ij dK_ij/d(amp, ls, X1_i): returns (g_amp, g_ls, X1bar [n1, d])."""
    X1 = np.asarray(X1, dtype=np.float64).reshape(len(X1), -1)
    X2 = np.asarray(X2, dtype=np.float64).reshape(len(X2), -1)
    K = kernel_matrix(kind, X1, X2, amp, ls)[0]
    dA, dL = kernel_matrix_grads(kind, X1, X2, amp, ls)
    diff = X1[:, None, :] - X2[None, :, :]
    r = np.sqrt(np.sum(diff ** 2, axis=-1)) / ls
    a2 = amp ** 2
    # dK/dx1 = a^2 g(r) (x1 - x2) / ls^2 with g = f'(r) / r
    with np.errstate(divide="ignore", invalid="ignore"):
        if kind == "eq":
            g = -K / a2
        elif kind == "matern12":
            g = np.where(r > 0, -np.exp(-r) / r, 0.0)
        elif kind == "matern32":
            g = -3.0 * np.exp(-np.sqrt(3.0) * r)
        elif kind == "matern52":
            s = np.sqrt(5.0) * r
            g = -(5.0 / 3.0) * (1.0 + s) * np.exp(-s)
    coef = Kbar * a2 * g / ls ** 2
    X1bar = np.einsum("ij,ijk->ik", coef, diff)
    return np.sum(Kbar * dA[0]), np.sum(Kbar * dL[0]), X1bar


def _chol_backward(Li, Lbar):
    """Symmetric adjoint of A = L L^T given Lbar (lower): sym(L^-T Phi(L^T Lbar) L^-1)."""
    L = np.linalg.inv(Li)
    P = np.tril(L.T @ Lbar)
    P[np.diag_indices_from(P)] *= 0.5
    S = Li.T @ P @ Li
    return 0.5 * (S + S.T)


def vgp_training_loss_grads(kind, Z, X, y, Xb, yb, amp, ls, noise, kl_weight, jitter=1e-6,
                            trace_adjoint=False):
    """(loss, d/damp, d/dls, d/dnoise, d/dZ) of vgp_training_loss for one kernel (B = 1)."""
    Z = np.asarray(Z, dtype=np.float64).reshape(len(Z), -1)
    X = np.asarray(X, dtype=np.float64).reshape(len(X), -1)
    Xb = np.asarray(Xb, dtype=np.float64).reshape(len(Xb), -1)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    yb = np.asarray(yb, dtype=np.float64).reshape(-1)
    a, l, s, j, w = float(amp), float(ls), float(noise), float(jitter), float(kl_weight)
    M, nb = Z.shape[0], yb.size
    I = np.eye(M)
    Kzz = kernel_matrix(kind, Z, Z, a, l)[0]
    Kzx = kernel_matrix(kind, Z, X, a, l)[0]
    Kzb = kernel_matrix(kind, Z, Xb, a, l)[0]
    # optimal posterior
    P0 = Kzx @ Kzx.T
    Sinv = Kzz + P0 / s + j * I
    Li = np.linalg.inv(np.linalg.cholesky(Sinv))
    c = Kzx @ y
    t = Li.T @ (Li @ c)
    m = Kzz @ t / s
    A = Li @ Kzz
    # variational loss
    Lzi = np.linalg.inv(np.linalg.cholesky(Kzz + j * I))
    Kzj_inv = Lzi.T @ Lzi
    v = Kzj_inv @ m
    r = yb - Kzb.T @ v
    s2 = s + j
    obs = -0.5 * r @ r / s2 - 0.5 * nb * np.log(2 * np.pi * s2)
    G = Lzi @ Kzb
    H = Lzi.T @ G
    R = (A.T if trace_adjoint else A) @ H
    T = 0.5 * (nb * a * a - np.sum(G * G) + np.sum(R * R)) / s
    Lpi = np.linalg.inv(np.linalg.cholesky(Kzz + (s + 1e-6) * I))
    Kp_inv = Lpi.T @ Lpi
    Lk = np.linalg.cholesky(Kzz)
    logdetA = 2 * np.sum(np.log(np.diag(Lk))) + np.sum(np.log(np.diag(Li)))
    KL = (np.sum(np.log(np.diag(np.linalg.inv(Lpi)))) - logdetA
          + 0.5 * (-M + np.sum((Lpi @ A) ** 2) + np.sum((Lpi @ m) ** 2)))
    E = obs - T - w * KL
    # ---- reverse pass for E ----
    Kzz_b = np.zeros((M, M))
    Kzb_b = np.zeros_like(Kzb)
    a_b = 0.0
    # obs
    mu_b = r / s2
    s_b = 0.5 * (r @ r) / s2 ** 2 - 0.5 * nb / s2
    Kzb_b += np.outer(v, mu_b)
    u = Kzj_inv @ (Kzb @ mu_b)
    m_b = u.copy()
    Kzz_b -= np.outer(u, v)
    # trace term
    s_b += T / s
    a_b += -nb * a / s
    Kzb_b += H / s
    Kzz_b -= H @ H.T / (2 * s)
    if trace_adjoint:
        A_b = -H @ R.T / s
        H_b = -A @ R / s
    else:
        A_b = -R @ H.T / s
        H_b = -A.T @ R / s
    Kzb_b += Kzj_inv @ H_b
    Kzz_b -= Kzj_inv @ H_b @ H.T
    # KL
    A_b += -w * Kp_inv @ A
    m_b += -w * Kp_inv @ m
    Kp_b = -0.5 * w * (Kp_inv - Kp_inv @ (A @ A.T + np.outer(m, m)) @ Kp_inv)
    Kzz_b += Kp_b
    s_b += np.trace(Kp_b)
    Lki = np.linalg.inv(Lk)
    Kzz_b += w * Lki.T @ Lki
    Sinv_b = -0.5 * w * Li.T @ Li
    # optimal posterior
    Kzz_b += np.outer(m_b, t) / s
    t_b = Kzz @ m_b / s
    s_b += -(m_b @ m) / s
    c_b = Li.T @ (Li @ t_b)
    Sinv_b -= 0.5 * (np.outer(c_b, t) + np.outer(t, c_b))
    Kzz_b += Li.T @ A_b
    Sinv_b += _chol_backward(Li, -Li.T @ A_b @ A.T)
    Kzz_b += Sinv_b
    Kzx_b = np.outer(c_b, y) + 2.0 * Sinv_b @ Kzx / s
    s_b += -np.sum(Sinv_b * P0) / s ** 2
    # kernel VJPs
    ga1, gl1, Zb1 = kernel_vjp(kind, Z, Z, a, l, Kzz_b + Kzz_b.T)
    ga2, gl2, Zb2 = kernel_vjp(kind, Z, X, a, l, Kzx_b)
    ga3, gl3, Zb3 = kernel_vjp(kind, Z, Xb, a, l, Kzb_b)
    a_b += 0.5 * ga1 + ga2 + ga3
    l_b = 0.5 * gl1 + gl2 + gl3
    Z_b = Zb1 + Zb2 + Zb3
    return -E, -a_b, -l_b, -s_b, -Z_b

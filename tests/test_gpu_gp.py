"""GPU parity of the GP surfaces (GaussianProcess / GPRM / VGP / gp_functions) vs oracle/gp.py.
Tolerance: north_star's 1e-5 relative for LML / ELBO (observed ~1e-12)."""
import numpy as np
import pytest

from oracle import gp as ogp

pytestmark = pytest.mark.gpu
RTOL = 1e-8   # well inside the 1e-5 relative bar of north_star


@pytest.fixture(scope="module")
def mods():
    import torch
    torch.cuda.set_device(0)
    from vgposp_amd import distributions, gp_functions, psd_kernels, variables
    return distributions, psd_kernels, gp_functions, variables


def _data(n=200, d=3, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-2, 2, (n, d))
    y = np.sin(2 * np.pi * X).sum(1) + rng.normal(0, 0.03, n)
    return X, y


@pytest.mark.parametrize("cls,kind", [("ExponentiatedQuadratic", "eq"), ("MaternOneHalf", "matern12"),
                                      ("MaternThreeHalves", "matern32"), ("MaternFiveHalves", "matern52")])
@pytest.mark.parametrize("n", [60, 257])
def test_gp_log_prob_batched(mods, cls, kind, n):
    dist, psd, _, _ = mods
    X, y = _data(n)
    amp, ls = np.array([0.7444, 1.3]), np.array([0.7444, 0.4])
    k = getattr(psd, cls)(amp, ls)
    gp = dist.GaussianProcess(k, X, observation_noise_variance=0.6931)
    got = np.asarray(gp.log_prob(y))
    np.testing.assert_allclose(got, ogp.gp_log_prob(kind, X, y, amp, ls, 0.6931), rtol=RTOL)
    assert gp.batch_shape == (2,) and gp.event_shape == (n,)


def test_gp_unbatched_and_sample(mods):
    dist, psd, _, _ = mods
    X, y = _data(100, 2)
    gp = dist.GaussianProcess(psd.ExponentiatedQuadratic(1.1, 0.6), X, observation_noise_variance=0.1)
    lp = gp.log_prob(y)
    assert lp.shape == ()
    assert float(lp) == pytest.approx(ogp.gp_log_prob("eq", X, y, 1.1, 0.6, 0.1)[0], rel=RTOL)
    s = gp.sample(4000, seed=3).cpu().numpy()
    assert s.shape == (4000, 100)
    emp = np.cov(s.T)
    ref = ogp.kernel_matrix("eq", X, X, 1.1, 0.6)[0] + 0.1 * np.eye(100)
    assert np.abs(emp - ref).max() < 0.15


def test_gprm_mean_cov_sample(mods):
    dist, psd, gpf, _ = mods
    X, y = _data(150, 2, seed=4)
    Xs = gpf.create_meshgrid(np.linspace(-2, 2, 12), np.linspace(-2, 2, 10))
    assert Xs.shape == (120, 2)
    k = psd.ExponentiatedQuadratic(np.array([0.9, 1.2]), np.array([0.5, 0.7]))
    gprm = gpf.tf_gp_regression_model(k, Xs, X, y, 0.05, 0.0)
    m = gprm.mean().cpu().numpy()
    c = gprm.covariance().cpu().numpy()
    rm, rc = ogp.gprm_mean_cov("eq", Xs, X, y, [0.9, 1.2], [0.5, 0.7], 0.05, 0.0)
    np.testing.assert_allclose(m, rm, rtol=1e-8, atol=1e-10)
    il = np.tril_indices(120)
    np.testing.assert_allclose(c[:, il[0], il[1]], rc[:, il[0], il[1]], rtol=1e-7, atol=1e-9)
    s = gprm.sample(8, seed=1).cpu().numpy()
    assert s.shape == (8, 2, 120) and np.isfinite(s).all()


def test_gp_fit_loop_matches_oracle(mods):
    """gp_functions fit loop (warm-up + num_iters+1 Adam steps) == oracle fit_gp_adam."""
    _, _, gpf, _ = mods
    from vgposp_amd.data_generation import grid_points, grid_observations
    X = grid_points((6, 6, 6), jitter=0.05, seed=0)
    y = grid_observations(X)
    sess = gpf.reset_session()
    amp, amp_assign, amp_p, lensc, lensc_assign, lensc_p, emb, emb_assign, emb_p, noise = \
        gpf.tf_Placeholder_assign_test(np.array([.1, .1]), np.array([.1, .1]), 1e-6)
    kernel = gpf.create_cov_kernel(amp, lensc)
    gp = gpf.fit_gp(kernel, X, noise)
    ll = gp.log_prob(y)
    train_op = gpf.tf_train_gp_adam(ll, 0.1)
    summ, writer, saver = gpf.tf_summary_writer_saver(sess, None)
    lls = gpf.tf_optimize_model_params(sess, 40, train_op, ll, summ, writer, saver, None, None, y, None)
    ref, theta = ogp.fit_gp_adam("matern12", X, y, [.1, .1], [.1, .1], 1e-6, 0.1, 40)
    assert lls.shape == (41, 2)
    np.testing.assert_allclose(lls, ref, rtol=1e-7)
    np.testing.assert_allclose(amp.numpy(), ogp.constrain(theta[:2]), rtol=1e-7)
    np.testing.assert_allclose(noise.numpy(), ogp.constrain(theta[4]), rtol=1e-7)


def test_calc_H_surface(mods):
    _, _, gpf, _ = mods
    X, y = _data(60, 2, seed=5)
    sess = gpf.reset_session()
    amp, amp_assign, amp_p, lensc, lensc_assign, lensc_p, _, _, _, noise = \
        gpf.tf_Placeholder_assign_test(np.array([.1]), np.array([.1]), 1e-3)
    gp = gpf.fit_gp(gpf.create_cov_kernel(amp, lensc), X, noise)
    ll = gp.log_prob(y)
    H = gpf.calc_H(12, 10, lensc, lensc_assign, lensc_p, amp, amp_assign, amp_p, ll, sess, None, y)
    ref = ogp.calc_H("matern12", X, y, float(noise.numpy()), 12, 10)
    np.testing.assert_allclose(H, ref, rtol=1e-8)
    assert lensc.numpy()[0] == pytest.approx(40.0, rel=1e-12)  # left at the last assigned pair


def test_session_assign_and_run(mods):
    _, _, gpf, _ = mods
    sess = gpf.reset_session()
    amp, amp_assign, amp_p, *_ = gpf.tf_Placeholder_assign_test(np.array([.1, .1]), np.array([.1, .1]), 1e-6)
    _, a = sess.run([amp_assign, amp], feed_dict={amp_p: [0.5, 0.25]})
    np.testing.assert_allclose(a, [0.5, 0.25], rtol=1e-12)


@pytest.mark.parametrize("kind", ["eq", "matern52"])
def test_vgp_optimal_posterior_loss_predictive(mods, kind):
    dist, psd, _, _ = mods
    rng = np.random.default_rng(7)
    N, M, nb = 600, 40, 64
    X = rng.uniform(-2, 2, (N, 2))
    y = np.sin(2 * X).sum(1) + rng.normal(0, 0.1, N)
    Z = rng.uniform(-2, 2, (M, 2))
    Xs = rng.uniform(-2, 2, (50, 2))
    cls = {"eq": psd.ExponentiatedQuadratic, "matern52": psd.MaternFiveHalves}[kind]
    k = cls(0.9, 0.7)
    loc, scale = dist.VariationalGaussianProcess.optimal_variational_posterior(k, Z, X, y, 0.05)
    rloc, rscale = ogp.vgp_optimal_posterior(kind, Z, X, y, 0.9, 0.7, 0.05)
    np.testing.assert_allclose(loc.cpu().numpy(), rloc[0], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(scale.cpu().numpy(), rscale[0], rtol=1e-7, atol=1e-9)
    vgp = dist.VariationalGaussianProcess(k, Xs, Z, loc, scale, observation_noise_variance=0.05)
    idx = rng.integers(0, N, nb)
    L = float(vgp.variational_loss(y[idx], X[idx], kl_weight=nb / N))
    ref = ogp.vgp_variational_loss(kind, Z, X[idx], y[idx], rloc, rscale, 0.9, 0.7, 0.05, nb / N)
    assert L == pytest.approx(ref, rel=1e-8)
    m = vgp.mean().cpu().numpy()
    c = vgp.covariance().cpu().numpy()
    rm, rc = ogp.vgp_predictive(kind, Xs, Z, rloc, rscale, 0.9, 0.7, 0.05)
    np.testing.assert_allclose(m, rm[0], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(c, rc[0], rtol=1e-6, atol=1e-8)


def test_gprm_posterior_sampling_at_scale(mods):
    """GPRM joint samples over a 50 x 50 prediction mesh (M = 2,500, as
    gp_functions.create_meshgrid / tf_gp_regression_model build it, gp_functions.py:262-297),
    conditioned on 512 observations: posterior mean / covariance vs the oracle, the M x M
    posterior Cholesky vs numpy, and the sample moments."""
    import torch
    dist, psd, gpf, _ = mods
    X, y = _data(512, 2, seed=8)
    Xs = gpf.create_meshgrid(np.linspace(-2, 2, 50), np.linspace(-2, 2, 50))
    k = psd.ExponentiatedQuadratic(0.9, 0.6)
    gprm = gpf.tf_gp_regression_model(k, Xs, X, y, 0.05, 0.0)
    mean, cov = gprm._posterior()
    rm, rc = ogp.gprm_mean_cov("eq", Xs, X, y, 0.9, 0.6, 0.05, 0.0)
    np.testing.assert_allclose(mean[0].cpu().numpy(), rm[0], rtol=1e-7, atol=1e-9)
    np.testing.assert_allclose(cov[0].cpu().numpy(), rc[0], rtol=1e-6, atol=1e-9)
    C = cov.clone()
    C.diagonal(dim1=-2, dim2=-1).add_(gprm.jitter)
    from vgposp_amd import linalg
    L, _, _ = linalg.cholesky_(C, invert=False, check=True)
    Lref = np.linalg.cholesky(rc[0] + gprm.jitter * np.eye(2500))
    got = torch.tril(L[0]).cpu().numpy()
    np.testing.assert_allclose(got, Lref, rtol=1e-5, atol=1e-8 * np.abs(Lref).max())
    s = gprm.sample(4000, seed=3).cpu().numpy()  # [S, M]
    assert s.shape == (4000, 2500) and np.isfinite(s).all()
    emp_mean = s.mean(0)
    sd = np.sqrt(np.diag(rc[0]) + gprm.jitter)
    assert np.all(np.abs(emp_mean - rm[0]) < 5 * sd / np.sqrt(4000) + 1e-9)


def test_c1_sin_wave_eq_fit_8cube(mods):
    """C1 as named: the RBF fit of 3D_sin_wave.py:126-209 on the 8 x 8 x 8 grid (main_GP_fit.py
    shape).  Amplitude and length scale are assigned 0.5 through the softplus placeholders
    (:190-197), the noise variance starts at softplus(INIT_OBSNOISEVAR), then Adam maximises
    gp.log_prob (:181-183, :207-208).  The LML trajectory and the trained parameters equal the
    oracle's fit_gp_adam over the same 512 points (rtol 1e-7)."""
    _, _, gpf, _ = mods
    from vgposp_amd.data_generation import grid_points, grid_observations
    from vgposp_amd.psd_kernels import ExponentiatedQuadratic
    X = grid_points((8, 8, 8), jitter=0.05, seed=2)
    y = grid_observations(X, seed=3)
    sess = gpf.reset_session()
    amp, amp_assign, amp_p, lensc, lensc_assign, lensc_p, _, _, _, noise = \
        gpf.tf_Placeholder_assign_test(np.array([1.0]), np.array([1.0]), 0.1)
    _, a = sess.run([amp_assign, amp], feed_dict={amp_p: [0.5]})
    _, l = sess.run([lensc_assign, lensc], feed_dict={lensc_p: [0.5]})
    np.testing.assert_allclose([a[0], l[0]], [0.5, 0.5], rtol=1e-12)
    gp = gpf.fit_gp(ExponentiatedQuadratic(amp, lensc), X, noise)
    ll = gp.log_prob(y)
    train_op = gpf.tf_train_gp_adam(ll, 0.05)
    lls = gpf.tf_optimize_model_params(sess, 30, train_op, ll, None, None, None, None, None, y, None)
    v0 = ogp.invert_softplus(0.5)
    ref, theta = ogp.fit_gp_adam("eq", X, y, [v0], [v0], 0.1, 0.05, 30)
    assert lls.shape == (31, 1)
    np.testing.assert_allclose(lls, ref, rtol=1e-7)
    assert lls[-1, 0] > lls[0, 0]  # the fit improves the likelihood
    np.testing.assert_allclose(amp.numpy(), ogp.constrain(theta[:1]), rtol=1e-7)
    np.testing.assert_allclose(lensc.numpy(), ogp.constrain(theta[1:2]), rtol=1e-7)
    np.testing.assert_allclose(noise.numpy(), ogp.constrain(theta[2]), rtol=1e-7)

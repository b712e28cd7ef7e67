"""CPU checks of the TFP-semantics oracle (oracle/gp.py): LML against scikit-learn (exact match of
the formula, jitter folded into alpha), gradients against finite differences, TF1 Adam."""
import numpy as np
import pytest

from oracle import gp as ogp


def test_lml_matches_sklearn():
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, ConstantKernel
    from vgposp_amd.data_generation import grid_points, grid_observations
    X = grid_points((5, 5, 5), jitter=0.05, seed=0)
    y = grid_observations(X)
    amp, ls, noise = 0.7444, 0.7444, 0.6931
    lml = ogp.gp_log_prob("eq", X, y, amp, ls, noise)[0]
    k = ConstantKernel(amp ** 2, "fixed") * RBF(ls, "fixed")
    gpr = GaussianProcessRegressor(k, alpha=noise + 1e-6, optimizer=None, normalize_y=False).fit(X, y)
    assert lml == pytest.approx(gpr.log_marginal_likelihood_value_, rel=1e-12)


@pytest.mark.parametrize("kind", ogp.KERNELS)
def test_lml_gradient_finite_difference(kind):
    rng = np.random.default_rng(1)
    X = rng.uniform(-2, 2, (40, 2))
    y = np.sin(X).sum(1)
    amp, ls, noise = np.array([0.9, 1.3]), np.array([0.5, 0.8]), 0.05
    _, ga, gl, gn = ogp.gp_log_prob_and_grads(kind, X, y, amp, ls, noise)
    h = 1e-6
    for b in range(2):
        e = np.eye(2)[b] * h
        fa = (ogp.gp_log_prob(kind, X, y, amp + e, ls, noise) - ogp.gp_log_prob(kind, X, y, amp - e, ls, noise))[b] / (2 * h)
        fl = (ogp.gp_log_prob(kind, X, y, amp, ls + e, noise) - ogp.gp_log_prob(kind, X, y, amp, ls - e, noise))[b] / (2 * h)
        assert ga[b] == pytest.approx(fa, rel=1e-5, abs=1e-6)
        assert gl[b] == pytest.approx(fl, rel=1e-5, abs=1e-6)
    fn = (ogp.gp_log_prob(kind, X, y, amp, ls, noise + h) - ogp.gp_log_prob(kind, X, y, amp, ls, noise - h)) / (2 * h)
    np.testing.assert_allclose(gn, fn, rtol=1e-5, atol=1e-6)


def test_softplus_constraint_values():
    # INIT 0.1 -> 0.7444, INIT 1e-6 -> 0.6931
    assert ogp.constrain(0.1) == pytest.approx(0.744396660073571, rel=1e-12)
    assert ogp.constrain(1e-6) == pytest.approx(0.6931476805599453, rel=1e-12)
    assert ogp.constrain(ogp.invert_softplus(0.5)) == pytest.approx(0.5, rel=1e-14)


def test_adam_tf1_first_step():
    opt = ogp.AdamTF1(0.1)
    th = opt.step(np.array([1.0, -2.0]), np.array([0.3, -4.0]))
    # first TF1 Adam step moves every coordinate by ~lr * sign(g)
    np.testing.assert_allclose(th, [1.0 - 0.1, -2.0 + 0.1], rtol=1e-6)


def test_fit_increases_lml():
    from vgposp_amd.data_generation import grid_points, grid_observations
    X = grid_points((4, 4, 4), jitter=0.05, seed=0)
    y = grid_observations(X)
    lls, _ = ogp.fit_gp_adam("eq", X, y, [0.1, 0.1], [0.1, 0.1], 1e-6, 0.1, 30)
    assert lls.shape == (31, 2)
    assert np.all(lls[-1] > lls[0])


def test_vgp_oracle_shapes_and_tightness():
    """With Z = X the optimal variational posterior reproduces the exact posterior mean."""
    rng = np.random.default_rng(2)
    X = rng.uniform(-2, 2, (30, 1))
    y = np.sin(3 * X[:, 0])
    loc, scale = ogp.vgp_optimal_posterior("eq", X, X, y, 1.0, 0.5, 0.1)
    assert loc.shape == (1, 30) and scale.shape == (1, 30, 30)
    m_vgp, _ = ogp.vgp_predictive("eq", X, X, loc, scale, 1.0, 0.5, 0.0)
    m_exact, _ = ogp.gprm_mean_cov("eq", X, X, y, 1.0, 0.5, 0.1, jitter=0.0)
    np.testing.assert_allclose(m_vgp[0], m_exact[0], rtol=1e-4, atol=1e-6)
    L = ogp.vgp_variational_loss("eq", X, X[:10], y[:10], loc, scale, 1.0, 0.5, 0.1, 10 / 30)
    assert np.isfinite(L)


@pytest.mark.parametrize("kind", ogp.KERNELS)
@pytest.mark.parametrize("adjoint", [False, True])
def test_vgp_training_grads_match_finite_differences(kind, adjoint):
    """The analytic reverse pass of the VGP training objective (the derivation the HIP path
    implements) against central differences of the restated loss."""
    rng = np.random.default_rng(7)
    N, M, nb = 50, 6, 8
    X = rng.uniform(-2, 2, (N, 2))
    y = np.sin(X).sum(1) + 0.1 * rng.normal(size=N)
    Z = rng.uniform(-2, 2, (M, 2))
    idx = rng.integers(0, N, nb)
    a, l, s, w = 0.9, 0.8, 0.3, nb / N
    L, ga, gl, gs, gZ = ogp.vgp_training_loss_grads(kind, Z, X, y, X[idx], y[idx], a, l, s, w,
                                                    trace_adjoint=adjoint)

    def f(a_, l_, s_, Z_):
        return ogp.vgp_training_loss(kind, Z_, X, y, X[idx], y[idx], a_, l_, s_, w,
                                     trace_adjoint=adjoint)
    assert L == pytest.approx(f(a, l, s, Z), rel=1e-10)
    h = 1e-6
    assert ga == pytest.approx((f(a + h, l, s, Z) - f(a - h, l, s, Z)) / (2 * h), rel=1e-5, abs=1e-6)
    assert gl == pytest.approx((f(a, l + h, s, Z) - f(a, l - h, s, Z)) / (2 * h), rel=1e-5, abs=1e-6)
    assert gs == pytest.approx((f(a, l, s + h, Z) - f(a, l, s - h, Z)) / (2 * h), rel=1e-5, abs=1e-6)
    fz = np.zeros_like(Z)
    for i in range(M):
        for k in range(2):
            Zp, Zm = Z.copy(), Z.copy()
            Zp[i, k] += h
            Zm[i, k] -= h
            fz[i, k] = (f(a, l, s, Zp) - f(a, l, s, Zm)) / (2 * h)
    np.testing.assert_allclose(gZ, fz, rtol=1e-5, atol=1e-6 * np.abs(fz).max())


def test_data_generation_helpers():
    """data_generation.py:24-122 restated: shapes, ranges and the polynomial columns."""
    from vgposp_amd import data_generation as dg
    rng = np.random.default_rng(0)
    P = dg.generate_random_points(100, [-2.0, 2.0], rng)
    assert P.shape == (100, 2) and P.min() >= -2.0 and P.max() < 2.0
    assert np.array_equal(dg.create_line(np.array([3.0, 1.0, 2.0]), np.array([1.0, 1.0, 0.5])),
                          [2.0, 0.0, 1.5])
    for deg, f in ((6, dg.generate_6d_polinomials), (4, dg.generate_4d_polinomials)):
        D = f(np.random.default_rng(1))
        assert D.shape == (1200, deg)
        np.testing.assert_allclose(D, D[:, :1] ** np.arange(1, deg + 1), rtol=1e-15)
    X, y = dg.generate_noisy_2Dsin_data(50, 1e-3, [[-2, 2], [-1, 1]], np.random.default_rng(2))
    assert X.shape == (50, 2) and y.shape == (50,) and (np.abs(X[:, 1]) <= 1).all()
    C = dg.create_random_cov(7, np.random.default_rng(3))
    assert np.allclose(C, C.T) and np.linalg.eigvalsh(C).min() > -1e-12


def test_gprm_oracle_matches_reference_fixture():
    """oracle.gp.gprm_mean_cov pinned to the REFERENCE's own numpy GP posterior
    (plot_confidence_interval.py:38-51, executed by tests/golden/make_golden_gprm.py): 5 noiseless
    training points, EQ with l^2 = 0.3 (amplitude 1), K + 5e-5 I, mu and s2 at 700 test points.
    The reference forms sqdist as |a|^2 + |b|^2 - 2ab, the oracle as (a - b)^2: absolute 1e-13."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "gprm_confidence.npz"))
    m, c = ogp.gprm_mean_cov("eq", z["Xtest"], z["Xtrain"], z["ytrain"].reshape(-1), 1.0,
                             np.sqrt(float(z["param"])), float(z["diag_shift"]), 0.0, jitter=0.0)
    np.testing.assert_allclose(m[0], z["mu"], rtol=0, atol=1e-13)
    np.testing.assert_allclose(np.diag(c[0]), z["s2"], rtol=0, atol=1e-13)
    assert z["mu"].shape == (700,) and float(z["s2"].min()) > 0

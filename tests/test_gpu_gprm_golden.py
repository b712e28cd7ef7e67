"""GPU: the GP regression model against the REFERENCE's own numpy GP posterior.

tests/golden/gprm_confidence.npz was produced by executing plot_confidence_interval.py:38-51
(tests/golden/make_golden_gprm.py): Xtrain = [-4, -3, -2, -1, 1], ytrain = sin(Xtrain), the kernel
exp(-0.5 sqdist / 0.3), i.e. ExponentiatedQuadratic(amplitude 1, length_scale sqrt(0.3)),
K + 5e-5 I, and at 700 test points in [-15, 15] the posterior mean mu and variance
s2 = diag(K_ss) - sum(Lk^2).  The HIP path (kernel_matrix + fused Cholesky / inverse + GEMMs)
runs with observation noise 5e-5, GPRM jitter 0 (total diagonal shift 5e-5, as the reference) and
predictive noise 0.  Tolerance: absolute 1e-13 (the reference forms sqdist as |a|^2 + |b|^2 - 2ab;
s2 reaches 9.7e-5 at the training points, where 1 - sum(Lk^2) cancels)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gprm_confidence.npz")


@pytest.fixture(scope="module")
def model():
    import torch
    torch.cuda.set_device(0)
    from vgposp_amd import distributions, psd_kernels
    z = np.load(FIX)
    k = psd_kernels.ExponentiatedQuadratic(1.0, np.sqrt(float(z["param"])))
    gprm = distributions.GaussianProcessRegressionModel(
        k, index_points=z["Xtest"], observation_index_points=z["Xtrain"],
        observations=z["ytrain"].reshape(-1), observation_noise_variance=float(z["diag_shift"]),
        predictive_noise_variance=0.0, jitter=0.0)
    return gprm, z


def test_gprm_mean_matches_reference(model):
    gprm, z = model
    mu = gprm.mean().cpu().numpy()
    assert mu.shape == (700,)
    np.testing.assert_allclose(mu, z["mu"], rtol=0, atol=1e-13)


def test_gprm_variance_matches_reference(model):
    gprm, z = model
    c = gprm.covariance().cpu().numpy()
    assert c.shape == (700, 700)
    np.testing.assert_allclose(np.diag(c), z["s2"], rtol=0, atol=1e-13)
    np.testing.assert_allclose(gprm.variance().cpu().numpy(), z["s2"], rtol=0, atol=1e-13)

"""GPU parity of the cov_vv builders against the oracle (oracle/covariance.py)."""
import numpy as np
import pytest

from oracle import covariance as oc
from oracle import gp as ogp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cov():
    import torch
    torch.cuda.set_device(0)
    from vgposp_amd import covariance
    return covariance


@pytest.mark.parametrize("N,S", [(300, 41), (1024, 300), (130, 2)])
def test_empirical_cov(cov, N, S):
    rng = np.random.default_rng(N)
    T = rng.normal(size=(N, S)) * 0.3 + 2.0
    C = cov.empirical_cov(T, tr_mean=0.0018, tr_stdev=0.7).cpu().numpy()
    ref = oc.empirical_cov(T, 0.0018, 0.7)
    np.testing.assert_allclose(C, ref, rtol=1e-10, atol=1e-13)
    assert (C == C.T).all()  # exactly symmetric


@pytest.mark.parametrize("cover,beta,lower", [((5, 4, 3), 1.0, False), ((4, 4, 4), 0.5, True),
                                              ((8, 1, 6), 2.0, False)])
def test_index_taper(cov, cover, beta, lower):
    import torch
    n = int(np.prod(cover))
    rng = np.random.default_rng(n)
    C0 = rng.normal(size=(n, n))
    C = torch.as_tensor(C0, device="cuda").clone()
    cov.index_taper_(C, cover, beta, lower=lower)
    ref = oc.index_taper(C0, cover, beta)
    got = C.cpu().numpy()
    if lower:
        il = np.tril_indices(n)
        np.testing.assert_allclose(got[il], ref[il], rtol=1e-13, atol=0)
        iu = np.triu_indices(n, 1)
        assert (got[iu] == C0[iu]).all()
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-13, atol=0)


@pytest.mark.parametrize("kind", ogp.KERNELS)
@pytest.mark.parametrize("n1,n2,d", [(1000, 300, 5), (257, 1, 3), (5000, 1024, 2)])
def test_kernel_matvec(cov, kind, n1, n2, d):
    rng = np.random.default_rng(n1 + n2)
    X1 = rng.uniform(-2, 2, (n1, d))
    X2 = rng.uniform(-2, 2, (n2, d))
    v = rng.normal(size=n2)
    got = cov.kernel_matvec(kind, X1, X2, 0.8, 0.9, v).cpu().numpy()
    ref = ogp.kernel_matrix(kind, X1, X2, 0.8, 0.9)[0] @ v
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12 * np.abs(v).sum())


def test_vgp_tracer_samples_and_cov(cov):
    """The arch2 pipeline: VGP mean at every (location, T/P sample) 5-D point, then cov_vv."""
    from vgposp_amd import distributions as tfd
    from vgposp_amd import psd_kernels as tfk
    rng = np.random.default_rng(3)
    X5 = rng.uniform(-2, 2, (800, 5))
    y = np.sin(X5).sum(1)
    Z = rng.uniform(-2, 2, (40, 5))
    k = tfk.ExponentiatedQuadratic(1.0, 1.5)
    loc, scale = tfd.VariationalGaussianProcess.optimal_variational_posterior(k, Z, X5, y, 0.1)
    vgp = tfd.VariationalGaussianProcess(k, X5[:4], Z, loc, scale, observation_noise_variance=0.1)
    locs = rng.uniform(-2, 2, (27, 3))
    tp = rng.uniform(-2, 2, (30, 2))
    T = cov.vgp_tracer_samples(vgp, locs, tp).cpu().numpy()
    pts = np.concatenate([np.repeat(locs, 30, 0), np.tile(tp, (27, 1))], 1)
    rloc, rscale = ogp.vgp_optimal_posterior("eq", Z, X5, y, 1.0, 1.5, 0.1)
    rm, _ = ogp.vgp_predictive("eq", pts, Z, rloc, rscale, 1.0, 1.5, 0.1)
    np.testing.assert_allclose(T.reshape(-1), rm[0], rtol=1e-7, atol=1e-9)
    C = cov.cov_vv_from_vgp(vgp, locs, tp).cpu().numpy()
    np.testing.assert_allclose(C, oc.empirical_cov(T), rtol=1e-9, atol=1e-12)

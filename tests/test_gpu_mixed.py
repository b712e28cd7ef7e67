"""Mixed-precision Cholesky (vgposp_potrf_mixed, config C5): fp32 factor on the f32 matrix cores +
fp64 refinement must give the fp64 inverse factor (vgposp_potrf_lower(invert = 1)) to rounding."""
import numpy as np
import pytest
import torch

from oracle import gp as ogp

pytestmark = pytest.mark.gpu


def _spd(n, seed, shift=1e-3, ls=0.8):
    X = np.random.default_rng(seed).uniform(-2, 2, (n, 3))
    return ogp.kernel_matrix("eq", X, X, 1.0, ls)[0] + shift * np.eye(n)


@pytest.mark.parametrize("n,shift", [(1, 0.5), (63, 1e-2), (64, 1e-2), (200, 1e-3), (700, 1e-3),
                                     (1024, 1e-2), (1500, 1e-2)])
def test_mixed_matches_fp64(n, shift):
    from vgposp_amd import linalg
    S = _spd(n, n, shift)
    A = torch.as_tensor(S, device="cuda")
    Li, ld, info, resid = linalg.cholesky_inv_mixed(A)
    ref, ldr, _ = linalg.cholesky_(A.clone(), invert=True)
    ref = torch.tril(ref)
    torch.cuda.synchronize()
    assert int(info.item()) == 0
    assert float(resid.item()) < 1e-6
    scale = float(ref.abs().max())
    np.testing.assert_allclose(Li.cpu().numpy(), ref.cpu().numpy(), rtol=0, atol=1e-10 * scale)
    np.testing.assert_allclose(ld.cpu().numpy(), ldr.reshape(-1).cpu().numpy(), rtol=1e-11)
    assert not torch.triu(Li, 1).any()
    # against numpy
    L = np.linalg.cholesky(S)
    np.testing.assert_allclose(2 * np.log(ld.cpu().numpy()).sum(), 2 * np.log(np.diag(L)).sum(),
                               rtol=1e-11)
    # the input is not modified
    assert torch.equal(A, torch.as_tensor(S, device="cuda"))


def test_mixed_fp32_only_when_iters_zero():
    """iters = 0 leaves the fp32 factor's inverse: close to fp64 only at fp32 accuracy."""
    from vgposp_amd import linalg
    from vgposp_amd._lib import call, query
    from vgposp_amd.linalg import _p
    n = 300
    A = torch.as_tensor(_spd(n, 1, 1e-2), device="cuda")
    Li = torch.empty_like(A)
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    ws = linalg.workspace(query("vgposp_potrf_mixed_workspace_bytes", n))
    call("vgposp_potrf_mixed", _p(A), n, n, _p(Li), n, None, 0, None, _p(info), _p(ws), ws.numel(),
         None)
    ref, _, _ = linalg.cholesky_(A.clone(), invert=True)
    err = float((Li - torch.tril(ref)).abs().max() / torch.tril(ref).abs().max())
    assert int(info.item()) == 0
    assert 1e-12 < err < 1e-3


def test_mixed_not_positive_definite():
    from vgposp_amd import linalg
    n = 150
    S = _spd(n, 2, 1e-2)
    S[40, 40] = -1.0
    _, _, info, _ = linalg.cholesky_inv_mixed(torch.as_tensor(S, device="cuda"), check=False)
    assert 0 < int(info.item()) <= 41
    with pytest.raises(Exception):
        linalg.cholesky_inv_mixed(torch.as_tensor(S, device="cuda"))

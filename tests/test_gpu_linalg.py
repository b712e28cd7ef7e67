"""GPU parity: kernel assembly, MFMA GEMM, Cholesky (+ fused inverse), LML vs the CPU oracle."""
import numpy as np
import pytest

from oracle import gp as ogp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    import torch
    from vgposp_amd import linalg
    torch.cuda.set_device(0)
    return linalg


@pytest.mark.parametrize("kind", ["eq", "matern12", "matern32", "matern52"])
@pytest.mark.parametrize("d,n1,n2", [(1, 7, 300), (2, 130, 129), (3, 513, 257), (5, 33, 64)])
def test_kernel_matrix(L, kind, d, n1, n2):
    rng = np.random.default_rng(d * 1000 + n1)
    X1 = rng.uniform(-2, 2, (n1, d))
    X2 = rng.uniform(-2, 2, (n2, d))
    amp, ls = [0.7, 1.3], [0.4, 1.9]
    K = L.kernel_matrix(kind, X1, X2, amp, ls).cpu().numpy()
    ref = ogp.kernel_matrix(kind, X1, X2, amp, ls)
    # exp(x) at x ~ -80 carries ~|x| ulp of relative error: 1e-13 covers it
    np.testing.assert_allclose(K, ref, rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("n", [1, 31, 200])
def test_kernel_matrix_lower_and_shift(L, n):
    import torch
    rng = np.random.default_rng(n)
    X = rng.uniform(-2, 2, (n, 3))
    out = torch.full((1, n, n), 7.0, dtype=torch.float64, device="cuda")
    L.kernel_matrix("eq", X, None, 1.1, 0.6, diag_shift=0.25, lower=True, out=out)
    K = out[0].cpu().numpy()
    ref = ogp.kernel_matrix("eq", X, X, 1.1, 0.6)[0] + 0.25 * np.eye(n)
    il = np.tril_indices(n)
    np.testing.assert_allclose(K[il], ref[il], rtol=2e-14)
    iu = np.triu_indices(n, 1)
    assert np.all(K[iu] == 7.0)  # upper triangle untouched


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (17, 33, 5), (128, 128, 16), (130, 257, 300)])
def test_gemm(L, ta, tb, m, n, k):
    rng = np.random.default_rng(m + 7 * n + 13 * k + ta + 2 * tb)
    A = rng.standard_normal((k, m) if ta else (m, k))
    B = rng.standard_normal((n, k) if tb else (k, n))
    C0 = rng.standard_normal((m, n))
    opA = A.T if ta else A
    opB = B.T if tb else B
    C = L.as_device(C0.copy())
    L.gemm(A, B, C, alpha=-1.5, beta=0.5, transa=bool(ta), transb=bool(tb))
    np.testing.assert_allclose(C.cpu().numpy(), -1.5 * opA @ opB + 0.5 * C0, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("ta,tb,tri_a,tri_b", [(0, 0, 0, 0), (0, 1, 0, 0), (1, 0, 0, 0),
                                               (1, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1),
                                               (0, 1, 0, 1), (1, 0, 1, 1)])
def test_gemm_many_tiles(L, ta, tb, tri_a, tri_b):
    """Enough output tiles (>= 512 of 256x128) for the wide-tile kernel when it is enabled
    (VGPOSP_GEMM_BMW=2); ragged m / n / k exercise the clamped loads and masks."""
    m, n, k = 4352, 4224, 200
    if tri_a or tri_b:
        k = m if tri_a else n
    rng = np.random.default_rng(ta + 2 * tb + 4 * tri_a + 8 * tri_b)
    A = rng.standard_normal((k, m) if ta else (m, k))
    B = rng.standard_normal((n, k) if tb else (k, n))
    opA = A.T if ta else A
    opB = B.T if tb else B
    if tri_a:  # the stored matrix is lower triangular
        opA = np.tril(A).T if ta else np.tril(A)
    if tri_b:
        opB = np.tril(B).T if tb else np.tril(B)
    C0 = rng.standard_normal((m, n))
    C = L.as_device(C0.copy())
    L.gemm(A, B, C, alpha=0.75, beta=-0.5, transa=bool(ta), transb=bool(tb), tri_a=bool(tri_a),
           tri_b=bool(tri_b))
    ref = 0.75 * opA @ opB - 0.5 * C0
    np.testing.assert_allclose(C.cpu().numpy(), ref, rtol=1e-11, atol=1e-10)


def test_gemm_asymmetric_layout(L):
    """A = I with an asymmetric B catches a transposed C/D fragment map."""
    A = np.eye(16)
    B = np.arange(16 * 16, dtype=np.float64).reshape(16, 16)
    np.testing.assert_array_equal(L.gemm(A, B).cpu().numpy(), B)
    np.testing.assert_array_equal(L.gemm(B, A).cpu().numpy(), B)


@pytest.mark.parametrize("n", [40, 300])
def test_gemm_lower_tri(L, n):
    rng = np.random.default_rng(n)
    M = np.tril(rng.standard_normal((n, n)))
    Mstore = M + np.triu(rng.standard_normal((n, n)), 1) * 1e3  # garbage above the diagonal
    Q = L.as_device(np.full((n, n), 5.0))
    L.gemm(Mstore, Mstore, Q, transa=True, lower_c=True, tri_a=True, tri_b=True)
    Qh = Q.cpu().numpy()
    il = np.tril_indices(n)
    np.testing.assert_allclose(Qh[il], (M.T @ M)[il], rtol=1e-12, atol=1e-12)
    assert np.all(Qh[np.triu_indices(n, 1)] == 5.0)


def _spd(n, rng):
    X = rng.uniform(-2, 2, (n, 3))
    return ogp.kernel_matrix("eq", X, X, 1.0, 0.7)[0] + 0.05 * np.eye(n)


@pytest.mark.parametrize("n", [1, 5, 127, 128, 129, 300, 513, 1000, 1536, 2100, 4100])
@pytest.mark.parametrize("invert", [False, True])
def test_cholesky(L, n, invert):
    rng = np.random.default_rng(n)
    S = _spd(n, rng)
    U = np.triu(S, 1)
    A = L.as_device(S.copy())
    A, ld, _ = L.cholesky_(A, invert=invert)
    Ah = A.cpu().numpy()
    Lref = np.linalg.cholesky(S)
    ref = np.linalg.inv(Lref) if invert else Lref
    il = np.tril_indices(n)
    np.testing.assert_allclose(Ah[il], ref[il], rtol=1e-9, atol=1e-10 * np.abs(ref).max())
    np.testing.assert_array_equal(np.triu(Ah, 1), U)  # strictly upper untouched
    np.testing.assert_allclose(ld[0].cpu().numpy(), np.diag(Lref), rtol=1e-12)


def test_cholesky_batched_and_not_pd(L):
    rng = np.random.default_rng(3)
    S1, S2 = _spd(200, rng), _spd(200, rng)
    S2[150, 150] = -1.0
    A = L.as_device(np.stack([S1, S2]))
    with pytest.raises(L.CholeskyError) as ei:
        L.cholesky_(A)
    assert ei.value.batch_index == 1 and ei.value.info >= 1
    A = L.as_device(np.stack([S1, S1 * 2]))
    L.cholesky_(A)
    np.testing.assert_allclose(np.tril(A[1].cpu().numpy()), np.linalg.cholesky(2 * S1), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("kind", ["eq", "matern12", "matern52"])
@pytest.mark.parametrize("n", [64, 300])
def test_lml_and_grad(L, kind, n):
    rng = np.random.default_rng(n)
    X = rng.uniform(-2, 2, (n, 2))
    y = np.sin(2 * np.pi * X).sum(1) + rng.normal(0, 0.03, n)
    amp, ls, noise = [0.8, 1.2], [0.3, 0.9], 0.05
    C = L.kernel_matrix(kind, X, None, amp, ls, diag_shift=noise + 1e-6, lower=True)
    C, ld, _ = L.cholesky_(C, invert=True)
    lml, alpha = L.lml_from_inverse(C, ld, y, want_alpha=True)
    Q = L.inverse_from_factor_inverse(C)
    g = L.lml_grad(kind, X, amp, ls, Q, alpha).cpu().numpy()
    rl, ga, gl, gn = ogp.gp_log_prob_and_grads(kind, X, y, amp, ls, noise)
    np.testing.assert_allclose(lml.cpu().numpy(), rl, rtol=1e-10)
    np.testing.assert_allclose(g[:, 0], ga, rtol=1e-8)
    np.testing.assert_allclose(g[:, 1], gl, rtol=1e-8)
    np.testing.assert_allclose(g[:, 2], gn, rtol=1e-8)


@pytest.mark.parametrize("n", [1, 5, 128, 129, 300, 1000, 2100])
@pytest.mark.parametrize("nrhs", [1, 7, 300])
@pytest.mark.parametrize("trans", [False, True])
def test_trsm(L, n, nrhs, trans):
    """vgposp_trsm_lower vs a dense solve with the numpy factor: L^-1 B and L^-T B (the two
    triangular solves of tfd.GaussianProcess.log_prob / GPRM)."""
    rng = np.random.default_rng(n + 3 * nrhs + int(trans))
    S = _spd(n, rng)
    Lf = np.linalg.cholesky(S)
    Lstore = Lf + np.triu(rng.standard_normal((n, n)), 1) * 1e3  # garbage above the diagonal
    B = rng.standard_normal((n, nrhs))
    X = L.trsm(Lstore, B, trans=trans).cpu().numpy()
    ref = np.linalg.solve(Lf.T if trans else Lf, B)
    np.testing.assert_allclose(X, ref, rtol=1e-9, atol=1e-9 * np.abs(ref).max())
    if nrhs == 1:
        x1 = L.trsm(Lstore, B[:, 0], trans=trans).cpu().numpy()
        np.testing.assert_allclose(x1, ref[:, 0], rtol=1e-9, atol=1e-9 * np.abs(ref).max())


@pytest.mark.parametrize("ta", [0, 1])
@pytest.mark.parametrize("tb", [0, 1])
@pytest.mark.parametrize("tri_a", [0, 1])
@pytest.mark.parametrize("tri_b", [0, 1])
@pytest.mark.parametrize("shape", ["square", "vector"])
def test_gemm_all_flags(L, ta, tb, tri_a, tri_b, shape):
    """Every (transa, transb, tri_a, tri_b) combination on the fast kernel, and the triangular
    mat-vec paths (n == 1): a stored triangular operand has garbage above its diagonal."""
    if shape == "vector" and (tri_b or tb):
        pytest.skip("a column vector B is neither transposed nor triangular here")
    m = k = 320
    n = 1 if shape == "vector" else (k if tri_b else 256)
    rng = np.random.default_rng(ta + 2 * tb + 4 * tri_a + 8 * tri_b + (16 if n == 1 else 0))
    As = rng.standard_normal((k, m) if ta else (m, k))
    Bs = rng.standard_normal((n, k) if tb else (k, n))
    Ae = np.tril(As) if tri_a else As
    Be = np.tril(Bs) if tri_b else Bs
    opA = Ae.T if ta else Ae
    opB = Be.T if tb else Be
    C0 = rng.standard_normal((m, n))
    C = L.as_device(C0.copy())
    L.gemm(As, Bs, C, alpha=1.25, beta=-0.5, transa=bool(ta), transb=bool(tb), tri_a=bool(tri_a),
           tri_b=bool(tri_b))
    np.testing.assert_allclose(C.cpu().numpy(), 1.25 * opA @ opB - 0.5 * C0, rtol=1e-11,
                               atol=1e-11)


@pytest.mark.parametrize("ta,tb,tri_a,tri_b", [(a, b, c, d) for a in (0, 1) for b in (0, 1)
                                               for c in (0, 1) for d in (0, 1)])
@pytest.mark.parametrize("beta,lower,splitk", [(0.0, 0, 0), (1.0, 0, 1), (1.0, 1, 0), (0.0, 1, 1)])
def test_gemm_beta01(L, ta, tb, tri_a, tri_b, beta, lower, splitk):
    """beta in {0, 1} (the Cholesky / inverse products): every flag combination, a lower-triangular
    C, split-K, and ragged sizes that cut every tile shape (128x128, 128x256, 256x128) and the
    16-deep K tiles; C's entries outside the written region keep their garbage."""
    m = 390 if not lower else 398
    n = m if (lower or tri_b) else 302
    k = m if tri_a else (n if tri_b else 278)
    if tri_a and tri_b and not lower:
        n = k = m
    rng = np.random.default_rng(ta + 2 * tb + 4 * tri_a + 8 * tri_b + 16 * lower + 32 * splitk)
    As = rng.standard_normal((k, m) if ta else (m, k))
    Bs = rng.standard_normal((n, k) if tb else (k, n))
    opA = (np.tril(As) if tri_a else As)
    opB = (np.tril(Bs) if tri_b else Bs)
    opA = opA.T if ta else opA
    opB = opB.T if tb else opB
    C0 = rng.standard_normal((m, n))
    C = L.as_device(C0.copy())
    L.gemm(As, Bs, C, alpha=-1.0, beta=beta, transa=bool(ta), transb=bool(tb), lower_c=bool(lower),
           tri_a=bool(tri_a), tri_b=bool(tri_b), splitk=bool(splitk))
    ref = -opA @ opB + beta * C0
    got = C.cpu().numpy()
    if lower:
        il, iu = np.tril_indices(m), np.triu_indices(m, 1)
        np.testing.assert_allclose(got[il], ref[il], rtol=1e-11, atol=1e-11)
        assert np.array_equal(got[iu], C0[iu])
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("tri_a,splitk", [(1, 1), (0, 1), (1, 0)])
def test_gemm_bottom_right_block(L, tri_a, splitk):
    """Operands and output are the bottom-right blocks of one large matrix (the trtri product
    X21 = -X22 W of the last recursion level): no load may run past the last valid element."""
    import torch
    N, b = 2048, 512
    rng = np.random.default_rng(5 + tri_a)
    big = L.as_device(rng.standard_normal((N, N)))
    W = L.as_device(rng.standard_normal((b, b)))
    X22 = big[N - b:, N - b:]
    C = big[N - b:, N - 2 * b:N - b]
    ref = -(np.tril(X22.cpu().numpy()) if tri_a else X22.cpu().numpy()) @ W.cpu().numpy()
    L.gemm(X22, W, C, alpha=-1.0, beta=0.0, tri_a=bool(tri_a), splitk=bool(splitk))
    torch.cuda.synchronize()
    np.testing.assert_allclose(C.cpu().numpy(), ref, rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("n", [200, 513, 701, 1100])
@pytest.mark.parametrize("invert", [False, True])
def test_cholesky_batched_one_recursion(L, n, invert):
    """B > 1 matrices of n > 128 run as ONE recursion (vgposp_potrf_batched_workspace_bytes):
    every factor, inverse and diagonal equals the single-matrix result; odd n takes the
    reference GEMM kernel's batched grid, n > 512 the block-inverse path."""
    rng = np.random.default_rng(n + invert)
    S = np.stack([_spd(n, rng) * (1.0 + 0.5 * b) for b in range(3)])
    A = L.as_device(S.copy())
    A, ld, info = L.cholesky_(A, invert=invert)
    assert int(info.abs().sum()) == 0
    il = np.tril_indices(n)
    for b in range(3):
        Lref = np.linalg.cholesky(S[b])
        ref = np.linalg.inv(Lref) if invert else Lref
        np.testing.assert_allclose(A[b].cpu().numpy()[il], ref[il], rtol=1e-9,
                                   atol=1e-10 * np.abs(ref).max())
        np.testing.assert_array_equal(np.triu(A[b].cpu().numpy(), 1), np.triu(S[b], 1))
        np.testing.assert_allclose(ld[b].cpu().numpy(), np.diag(Lref), rtol=1e-12)


@pytest.mark.parametrize("ta,tb,tri_a,tri_b,lower", [(0, 0, 0, 0, 0), (1, 0, 1, 1, 0),
                                                     (0, 1, 0, 0, 1), (0, 0, 1, 0, 0),
                                                     (1, 1, 0, 0, 0)])
@pytest.mark.parametrize("m,n,k", [(512, 512, 512), (130, 257, 300), (64, 96, 2048)])
def test_gemm_batched(L, ta, tb, tri_a, tri_b, lower, m, n, k):
    if lower:
        n = m
    if tri_a:
        k = m
    if tri_b:
        k = n
    rng = np.random.default_rng(m + n + k + 5 * ta + 7 * tb + 11 * tri_a)
    nb = 3
    A = rng.standard_normal((nb, k, m) if ta else (nb, m, k))
    B = rng.standard_normal((nb, n, k) if tb else (nb, k, n))
    C0 = rng.standard_normal((nb, m, n))
    C = L.as_device(C0.copy())
    L.gemm_batched(A, B, C, alpha=0.5, beta=-1.0, transa=bool(ta), transb=bool(tb),
                   lower_c=bool(lower), tri_a=bool(tri_a), tri_b=bool(tri_b))
    Ch = C.cpu().numpy()
    for b in range(nb):
        opA = np.swapaxes(A[b], 0, 1) if ta else A[b]
        opB = np.swapaxes(B[b], 0, 1) if tb else B[b]
        if tri_a:
            opA = np.tril(A[b]).T if ta else np.tril(A[b])
        if tri_b:
            opB = np.tril(B[b]).T if tb else np.tril(B[b])
        ref = 0.5 * opA @ opB - C0[b]
        if lower:
            il = np.tril_indices(m)
            np.testing.assert_allclose(Ch[b][il], ref[il], rtol=1e-11, atol=1e-10)
            np.testing.assert_array_equal(Ch[b][np.triu_indices(m, 1)],
                                          C0[b][np.triu_indices(m, 1)])
        else:
            np.testing.assert_allclose(Ch[b], ref, rtol=1e-11, atol=1e-10)


@pytest.mark.parametrize("kind", ["eq", "matern52"])
@pytest.mark.parametrize("n1,n2,d", [(512, 5000, 3), (37, 129, 5), (1, 1, 1)])
def test_kernel_matrix_matvec(L, kind, n1, n2, d):
    """Fused K(X1, X2) assembly + K v (the VGP's Kzx and c = Kzx y in one pass)."""
    import torch
    rng = np.random.default_rng(n1 + n2)
    X1 = rng.uniform(-2, 2, (n1, d))
    X2 = rng.uniform(-2, 2, (n2, d))
    v = rng.standard_normal(n2)
    K = torch.empty((n1, n2), dtype=torch.float64, device="cuda")
    out = torch.empty(n1, dtype=torch.float64, device="cuda")
    L.kernel_matrix_matvec(kind, X1, X2, 0.8, 0.9, v, K, out)
    ref = ogp.kernel_matrix(kind, X1, X2, 0.8, 0.9)[0]
    np.testing.assert_allclose(K.cpu().numpy(), ref, rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(out.cpu().numpy(), ref @ v, rtol=1e-11, atol=1e-12)


# (ta, tb, tri_a, tri_b, lower, m, n, k): every flag the grouped kernel dispatches on, shapes that
# split (512^3), that do not (long tiles), odd / GEMV ones that fall back to single launches
GROUP_CASES = [(0, 0, 0, 0, 0, 512, 512, 512), (1, 0, 0, 0, 0, 512, 512, 512),
               (0, 0, 1, 0, 0, 512, 384, 512), (0, 1, 0, 0, 1, 256, 256, 1024),
               (1, 0, 1, 1, 0, 384, 384, 384), (0, 0, 0, 1, 0, 130, 256, 256),
               (1, 1, 0, 0, 0, 64, 96, 2048), (0, 0, 0, 0, 0, 129, 1, 77)]


@pytest.mark.gpu
@pytest.mark.parametrize("order", [0, 1])
def test_gemm_group_matches_numpy(L, order):
    cases = GROUP_CASES if order == 0 else GROUP_CASES[::-1]
    rng = np.random.default_rng(11 + order)
    specs, refs, C0s = [], [], []
    for ta, tb, tri_a, tri_b, lower, m, n, k in cases:
        A = rng.standard_normal((k, m) if ta else (m, k))
        B = rng.standard_normal((n, k) if tb else (k, n))
        C0 = rng.standard_normal((m, n))
        opA = np.tril(A).T if (tri_a and ta) else np.tril(A) if tri_a else (A.T if ta else A)
        opB = np.tril(B).T if (tri_b and tb) else np.tril(B) if tri_b else (B.T if tb else B)
        refs.append(0.5 * opA @ opB - C0)
        C0s.append(C0)
        specs.append(dict(A=A, B=B, C=L.as_device(C0.copy()), alpha=0.5, beta=-1.0,
                          transa=bool(ta), transb=bool(tb), lower_c=bool(lower),
                          tri_a=bool(tri_a), tri_b=bool(tri_b)))
    outs = L.gemm_group(specs)
    for (ta, tb, tri_a, tri_b, lower, m, n, k), C, ref, C0 in zip(cases, outs, refs, C0s):
        Ch = C.cpu().numpy()
        if lower:
            il = np.tril_indices(m)
            np.testing.assert_allclose(Ch[il], ref[il], rtol=1e-11, atol=1e-10)
            np.testing.assert_array_equal(Ch[np.triu_indices(m, 1)], C0[np.triu_indices(m, 1)])
        else:
            np.testing.assert_allclose(Ch, ref, rtol=1e-11, atol=1e-10)

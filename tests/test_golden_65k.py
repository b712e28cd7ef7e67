"""The CPU fixture of the headline's own 50 picks at N = 65,536 (tests/golden/bench65k_cpu_picks.json,
made by tests/golden/make_golden_65k.py in the build container in ~53 min) and the algebra that
made it, checked on CPU at small sizes:

* the blocked in-place Cholesky + triangular inverse equals numpy's inverse factor, reading only
  the lower triangle (the buffer's upper triangle is garbage there);
* the column norms / M^T (M e_a) helpers equal the dense products;
* the whole generator at 8^3 (N = 512, k = 12) reproduces oracle.placement.placement_lazy_incremental,
  the restatement test_oracle.py pins to the reference-executed goldens (placement_algorithm2.py:151-219);
* the committed fixture is well formed: 50 distinct in-range picks, positive per-round margins.

The GPU side (tests/test_gpu_fullsize.py) requires the HIP path's 50 picks to EQUAL the fixture and
its deltas to agree to 1e-9 relative."""
import json
import os

import numpy as np
import pytest

from tests.golden import make_golden_65k as g65

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "bench65k_cpu_picks.json")


def _spd(n, seed=0):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, n))
    return A @ A.T + n * np.eye(n)


def test_blocked_cholesky_inverse_lower_only():
    n = 300
    S = _spd(n)
    F = np.asfortranarray(np.full((n, n), np.nan))   # garbage (NaN) above the diagonal
    F[np.tril_indices(n)] = S[np.tril_indices(n)]
    g65.blocked_cholesky_inverse(F, nb=64, log=lambda m: None)
    M = np.tril(F)
    want = np.linalg.inv(np.linalg.cholesky(S))
    np.testing.assert_allclose(M, want, rtol=0, atol=1e-13 * np.abs(want).max())


def test_lower_helpers_match_dense():
    n = 257
    S = _spd(n, 1)
    M = np.linalg.inv(np.linalg.cholesky(S))
    F = np.asfortranarray(np.full((n, n), np.nan))
    F[np.tril_indices(n)] = M[np.tril_indices(n)]
    Q = M.T @ M
    np.testing.assert_allclose(g65.lower_colnorms2(F, nb=64), np.diag(Q), rtol=1e-12)
    for a in (0, 63, 64, 200, n - 1):
        np.testing.assert_allclose(g65.lower_mtm_col(F, a, nb=64), Q[:, a], rtol=1e-12,
                                   atol=1e-15 * np.abs(Q).max())


def test_generator_matches_incremental_oracle_at_8cube(tmp_path, monkeypatch):
    from oracle import placement as op
    from vgposp_amd.workloads import placement_split
    out = tmp_path / "g8.json"
    monkeypatch.setattr("sys.argv", ["make_golden_65k.py", "--shape", "8", "8", "8", "--k", "12",
                                     "--nb", "128", "--out", str(out)])
    g65.main()
    got = json.loads(out.read_text())
    X, ls = placement_split((8, 8, 8), 0)
    d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    S = np.exp(-0.5 * d2 / ls ** 2) + (1e-2 + 1e-6) * np.eye(len(X))
    want_d = []
    want = op.placement_lazy_incremental(S, 12, deltas_out=want_d)
    assert got["picks"] == want
    np.testing.assert_allclose(got["deltas"], want_d, rtol=1e-11)
    assert min(got["margins"]) >= 0.0


def test_committed_65k_fixture_well_formed():
    if not os.path.exists(FIXTURE):
        pytest.skip("tests/golden/bench65k_cpu_picks.json not generated")
    with open(FIXTURE) as f:
        fx = json.load(f)
    assert fx["N"] == 65536 and fx["k"] == 50 and fx["shape"] == [64, 32, 32]
    picks = fx["picks"]
    assert len(picks) == 50 and len(set(picks)) == 50
    assert all(0 <= p < 65536 for p in picks)
    assert len(fx["deltas"]) == 50 and all(np.isfinite(fx["deltas"]))
    # the smallest margin a rounding difference would have to overcome to flip a pick: 5.9e-7
    # relative (round 49), against ~1e-12 relative differences between two fp64 factorizations
    assert min(fx["margins"]) > 1e-8 * max(fx["deltas"])

"""Config C4, exact (vgposp_amd.sparse_placement): algorithm 3 on the beta-decay tapered covariance
without a dense cov_vv, checked against the reference semantics.

* diag((Sigma + eps I)^-1) from the multifrontal selected inverse against a dense inverse;
* the CG columns Q e_a against the dense inverse's columns;
* picks, pick deltas and delta_cached_iters against the oracle's restatement of
  snippets_a3.sparse_placement_algorithm_3 on the dense tapered matrix (small grids);
* picks against the plain-C restatement (oracle/c4_exact.c) at 48x40x56 .. 128^3;
* picks against the dense algorithm-3 engine on the GPU (snippets_a3.placement_algorithm_3 over
  the dense tapered covariance) on every grid where that matrix fits: 16^3, 24^3, 32^3, 40^3."""
import numpy as np
import pytest
import torch

from oracle import taper as lp
from oracle import placement as op
from vgposp_amd.data_generation import grid_points, grid_spacing

pytestmark = pytest.mark.gpu

SHIFT = 0.01 + 1e-6


def _grid(shape, seed=0):
    return grid_points(shape, jitter=0.05, seed=seed), 2.0 * grid_spacing(shape)


def _dense(X, shape, beta, ls, kind="eq"):
    return lp.tapered_cov(X, shape, beta, kind=kind, ls=ls, diag_shift=SHIFT)


@pytest.mark.parametrize("shape,beta,leaf,kind", [
    ((12, 11, 10), 4.0, 512, "eq"),
    ((12, 11, 10), 4.0, 40, "eq"),
    ((9, 10, 11), 2.5, 64, "eq"),
    ((10, 9, 8), 3.0, 100, "matern52"),
    ((16, 16, 16), 4.0, 512, "eq"),
    ((3, 4, 30), 4.0, 16, "matern32"),
])
def test_selected_inverse_diag(shape, beta, leaf, kind):
    from vgposp_amd.sparse_placement import FrontalSelectedInverse, TaperProblem
    X, ls = _grid(shape, seed=sum(shape))
    C = _dense(X, shape, beta, ls, kind) + 1e-6 * np.eye(len(X))
    ref = np.diag(np.linalg.inv(C))
    prob = TaperProblem(X, shape, beta, kind, ls=ls, diag_shift=SHIFT)
    fs = FrontalSelectedInverse(prob, leaf=leaf)
    q = fs.run().cpu().numpy()
    fs.check()
    np.testing.assert_allclose(q, ref, rtol=1e-12)


@pytest.mark.parametrize("method", ["selinv", "bounds"])
def test_cg_columns_match_dense_inverse(method):
    from vgposp_amd.sparse_placement import ExactTaperPlacement
    shape = (12, 11, 10)
    X, ls = _grid(shape, seed=3)
    run = ExactTaperPlacement(X, shape, 8, 3, ls=ls, diag_shift=SHIFT, leaf=128, method=method)
    picks = run.run().cpu().numpy()
    C = _dense(X, shape, 4.0, ls) + 1e-6 * np.eye(len(X))
    Qinv = np.linalg.inv(C)
    cols = run.greedy.q_columns()
    for t in range(7 if method == "selinv" else 8):  # selinv: the last pick has no column
        np.testing.assert_allclose(cols[t].cpu().numpy(), Qinv[:, picks[t]], rtol=0,
                                   atol=1e-14 * Qinv[picks[t], picks[t]])


@pytest.mark.parametrize("shape,k,cutoff,beta,kind", [
    ((8, 8, 8), 8, 3, 4.0, "eq"),
    ((10, 9, 8), 10, 2, 4.0, "matern52"),
    ((9, 9, 9), 10, 3, 2.5, "eq"),
    ((6, 7, 30), 12, 1, 4.0, "eq"),
])
def test_exact_alg3_matches_oracle(shape, k, cutoff, beta, kind):
    """Picks, pick deltas and every delta_cached_iters column against the oracle's precision-form
    restatement of snippets_a3.py:43-364 on the dense tapered matrix."""
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    X, ls = _grid(shape, seed=shape[0] * 7 + k)
    A, deltas, dci = tapered_placement_algorithm_3(X, k, shape, cutoff, beta, kernel=kind, ls=ls,
                                                   diag_shift=SHIFT, snapshots=True, leaf=96)
    C = _dense(X, shape, beta, ls, kind)
    rA, _, rdci = op.placement_window_precision(C, k, shape, cutoff)
    assert [int(a) for a in A] == rA
    np.testing.assert_allclose(dci, rdci, rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(deltas, [rdci[a, i] for i, a in enumerate(rA)], rtol=1e-10)


@pytest.mark.parametrize("shape,k,cutoff,beta,kind", [
    ((8, 8, 8), 8, 3, 4.0, "eq"),
    ((10, 9, 8), 10, 2, 4.0, "matern52"),
    ((6, 7, 30), 12, 1, 4.0, "eq"),
    ((14, 13, 12), 30, 3, 4.0, "matern32"),
    ((20, 4, 9), 25, 2, 4.0, "matern12"),
])
def test_bounded_alg3_matches_oracle(shape, k, cutoff, beta, kind):
    """The bounded-lazy rounds (upper bounds of Q_yy from K-step CG, refinement by the CG column
    whenever the arg-max lands on a bounded candidate) pick the oracle's sensors with the
    oracle's pick deltas."""
    from vgposp_amd.sparse_placement import ExactTaperPlacement
    X, ls = _grid(shape, seed=shape[0] * 7 + k)
    run = ExactTaperPlacement(X, shape, k, cutoff, beta, kind, ls=ls, diag_shift=SHIFT,
                              method="bounds")
    A = [int(a) for a in run.run().cpu().numpy()]
    assert run.used == "bounds"
    C = _dense(X, shape, beta, ls, kind)
    rA, _, rdci = op.placement_window_precision(C, k, shape, cutoff)
    assert A == rA
    np.testing.assert_allclose(run.greedy.pick_delta[:k].cpu().numpy(),
                               [rdci[a, i] for i, a in enumerate(rA)], rtol=1e-10)
    g = run.greedy
    from vgposp_amd.sparse_placement import REFINE_BATCH
    assert g.refine_batches <= 2 * k and k <= g.refinements <= REFINE_BATCH * g.refine_batches


@pytest.mark.parametrize("shape,k,cutoff,kind,pre", [
    ((14, 13, 12), 30, 3, "matern32", 0),
    ((20, 16, 14), 40, 2, "eq", 0),
    ((20, 16, 14), 40, 2, "eq", 24),
    ((14, 13, 12), 30, 3, "matern32", 300),
    ((20, 16, 14), 40, 3, "eq", 100000),
])
def test_two_bound_levels_equal_one(shape, k, cutoff, kind, pre):
    """The K_lo bounds + tightening to K_hi before a CG column (on demand, and with the `pre`
    best round-0 candidates tightened before the rounds: a few, some hundreds, all), and one
    bound level for all: the same picks and pick deltas (bit for bit: every pick's delta comes
    from its exact Q_yy either way), the oracle's picks."""
    from vgposp_amd.sparse_placement import PRETIGHTEN, ExactTaperPlacement
    X, ls = _grid(shape, seed=k + 3)
    out = []
    for two in (True, False):
        run = ExactTaperPlacement(X, shape, k, cutoff, 4.0, kind, ls=ls, diag_shift=SHIFT,
                                  method="bounds")
        run.greedy.two_level = two
        run.greedy.pretighten = min(pre, 32768)
        A = [int(a) for a in run.run().cpu().numpy()]
        g = run.greedy
        assert (g.tight is not None) == two
        out.append((A, g.pick_delta[:k].cpu().numpy(), g.tightened))
    assert out[0][0] == out[1][0]
    np.testing.assert_array_equal(out[0][1], out[1][1])
    assert out[0][2] > 0 and out[1][2] == 0
    if pre:  # at least the pre-tightened ones (every candidate when pre >= n)
        assert out[0][2] >= min(pre, int(np.prod(shape)))
    assert 1 <= PRETIGHTEN <= 65536
    rA, _, _ = op.placement_window_precision(_dense(X, shape, 4.0, ls, kind), k, shape, cutoff)
    assert out[0][0] == rA


@pytest.mark.parametrize("shape,k,cutoff", [
    ((1, 1, 40), 6, 3),      # a line of candidates
    ((2, 3, 50), 9, 2),
    ((5, 6, 7), 1, 3),       # k = 1: round 0 only
    ((6, 5, 4), 10, 0),      # cutoff 0: empty windows, the top-k of round 0
    ((3, 3, 3), 27, 1),      # every candidate placed
])
def test_bounded_edge_cases_match_oracle(shape, k, cutoff):
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    X, ls = _grid(shape, seed=sum(shape) + k)
    A, d, _ = tapered_placement_algorithm_3(X, k, shape, cutoff, 4.0, ls=ls, diag_shift=SHIFT,
                                            method="bounds")
    C = _dense(X, shape, 4.0, ls)
    rA, _, rdci = op.placement_window_precision(C, k, shape, cutoff)
    assert [int(a) for a in A] == rA
    np.testing.assert_allclose(d, [rdci[a, i] for i, a in enumerate(rA)], rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("shape,beta,kind", [
    ((12, 11, 10), 4.0, "eq"),
    ((9, 10, 11), 4.0, "matern52"),
    ((3, 4, 30), 4.0, "matern12"),
])
@pytest.mark.parametrize("radau", [True, False])
def test_bounds_bracket_dense_inverse(shape, beta, kind, radau):
    """vgposp_exact_bounds: g_K <= Q_yy <= qhi; Chebyshev (mu = 0): qhi within 4 rho^2K (+ margin)
    of Q_yy; Gauss-Radau (mu = the Gershgorin lambda_min, one step fewer): within 4x the
    Chebyshev width of K + 1 steps, and the second level's bounds tighter."""
    from vgposp_amd.sparse_placement import (BOUND_HI_TARGET, BOUND_LO_TARGET, ExactWindowGreedy,
                                             TaperProblem)
    X, ls = _grid(shape, seed=sum(shape) + 1)
    C = _dense(X, shape, beta, ls, kind) + 1e-6 * np.eye(len(X))
    ref = np.diag(np.linalg.inv(C))
    prob = TaperProblem(X, shape, beta, kind, ls=ls, diag_shift=SHIFT)
    g = ExactWindowGreedy(prob, 4, 3)
    g.radau = radau
    q = torch.zeros(prob.n, dtype=torch.float64, device="cuda")
    K, scale, width = g.bound_qdiag(q)
    hi = q.cpu().numpy()
    assert np.all(hi >= ref)
    if radau:
        assert g.bound_mu > 0 and scale == 1.0 + 1e-12
        assert np.all(hi <= ref * (1 + 4 * width))
    else:
        assert g.bound_mu == 0.0
        assert np.all(hi <= ref * scale * (1 + 1e-13))
    assert width <= BOUND_LO_TARGET
    t = g.tight
    if t is not None:             # the second level (the K_hi table) brackets too, tighter
        q3 = torch.zeros_like(q)
        g.bound_qdiag(q3, steps=t, mu=g.bound_mu)
        hi3 = q3.cpu().numpy()
        assert t[0] > K and t[2] <= BOUND_HI_TARGET
        assert np.all(hi3 >= ref)
        if radau:
            assert np.all(hi3 <= ref * (1 + 4 * t[2]))
        else:
            assert np.all(hi3 <= ref * t[1] * (1 + 1e-13))
    # the same bounds slab by slab
    q2 = torch.zeros_like(q)
    n = prob.n
    for c0, c1 in ((0, n // 3), (n // 3, n - 5), (n - 5, n)):
        g.bound_qdiag(q2, c0, c1)
    assert torch.equal(q, q2)


def test_bounds_refuse_without_diagonal_dominance():
    """beta = 2.5: the Gershgorin bounds of the tapered covariance do not bracket its spectrum away
    from 0, so the bounded form refuses and 'auto' takes the selected inverse."""
    from vgposp_amd.sparse_placement import ExactTaperPlacement
    shape = (9, 9, 9)
    X, ls = _grid(shape, seed=5)
    run = ExactTaperPlacement(X, shape, 6, 3, 2.5, ls=ls, diag_shift=SHIFT, method="bounds")
    with pytest.raises(ValueError):
        run.run()
    run = ExactTaperPlacement(X, shape, 6, 3, 2.5, ls=ls, diag_shift=SHIFT, leaf=64)
    A = [int(a) for a in run.run().cpu().numpy()]
    assert run.used == "selinv"
    rA, _, _ = op.placement_window_precision(_dense(X, shape, 2.5, ls), 6, shape, 3)
    assert A == rA


def test_exact_alg3_matches_pinv_oracle_tiny():
    """The reference's own arithmetic (pinv per delta, snippets_a3.py:77-124 restated) on a 5^3
    grid."""
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    shape = (5, 5, 5)
    X, ls = _grid(shape, seed=11)
    A, _, dci = tapered_placement_algorithm_3(X, 6, shape, 2, 4.0, ls=ls, diag_shift=SHIFT,
                                              snapshots=True, leaf=20)
    order = []
    _, _, rdci = op.sparse_placement_algorithm_3(_dense(X, shape, 4.0, ls), 6, shape, 2,
                                                 order=order)
    assert [int(a) for a in A] == order
    np.testing.assert_allclose(dci, rdci, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("n", [16, 24, 32, 40])
def test_exact_alg3_matches_dense_engine(n):
    """Verdict item 1(a): the dense algorithm 3 (snippets_a3.placement_algorithm_3 over the dense
    tapered covariance, beta = 4, cutoff 3, k = 50, TF constants) and the exact sparse path pick
    the same sensors on every grid where the dense matrix fits one GPU (40^3: 33 GB)."""
    from vgposp_amd import linalg
    from vgposp_amd.covariance import index_taper_
    from vgposp_amd.snippets_a3 import placement_algorithm_3
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    shape = (n, n, n)
    X, ls = _grid(shape, seed=n)
    k = 50
    A, deltas, _ = tapered_placement_algorithm_3(X, k, shape, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                                 method="selinv")
    B, deltas_b, _ = tapered_placement_algorithm_3(X, k, shape, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                                   method="bounds")
    assert [int(a) for a in A] == [int(a) for a in B]
    np.testing.assert_allclose(deltas_b, deltas, rtol=1e-12)
    N = len(X)
    S = torch.empty((1, N, N), dtype=torch.float64, device="cuda")
    linalg.kernel_matrix("eq", X, None, 1.0, ls, diag_shift=SHIFT, out=S)
    index_taper_(S[0], shape, 4.0)
    dense = placement_algorithm_3(S[0], k, shape, 3)
    del S
    torch.cuda.empty_cache()
    assert [int(a) for a in A] == [int(a) for a in dense]


def _two_rank_worker(rank, world, port, shape, k, out, method):
    import os

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
        X, ls = _grid(shape, seed=4)
        A, d, _ = tapered_placement_algorithm_3(X, k, shape, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                                leaf=128, method=method)
        out[rank] = ([int(a) for a in A], [float(v) for v in d])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,method", [(2, "selinv"), (4, "selinv"), (2, "bounds"),
                                          (3, "bounds")])
def test_exact_alg3_ranks_on_one_gpu(world, method):
    """The multi-rank C4 paths (subtree-to-subcube selected inverse, or the bounds sharded by
    candidate slabs and all-gathered; transfers host-staged over gloo, every rank on cuda:0) give
    the single-rank picks and deltas bit for bit."""
    import socket

    import torch.multiprocessing as mp
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    shape, k = (16, 14, 12), 20
    X, ls = _grid(shape, seed=4)
    A1, d1, _ = tapered_placement_algorithm_3(X, k, shape, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                              leaf=128, method=method)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_two_rank_worker, args=(world, port, shape, k, out, method), nprocs=world,
                       join=True, start_method="spawn")
    for r in range(world):
        assert out[r][0] == [int(a) for a in A1]
        np.testing.assert_allclose(out[r][1], d1, rtol=1e-13)


@pytest.mark.parametrize("method", ["bounds", "selinv"])
def test_exact_128cube_regression(method):
    """Config C4 at full size (128^3, k = 50) reproduces the picks committed in
    tests/golden/c4_picks.json (written by tools/bench_exact.py with PICKS_OUT; the same sequence
    the 16^3-40^3 tests tie to the dense algorithm 3).  A regression pin, not a reference
    fixture: no dense algorithm 3 fits 128^3."""
    import json
    import os
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    from vgposp_amd.workloads import c4_grid
    with open(os.path.join(os.path.dirname(__file__), "golden", "c4_picks.json")) as f:
        want = json.load(f)["picks"]
    X, shape, ls = c4_grid()
    A, _, _ = tapered_placement_algorithm_3(X, 50, shape, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                            method=method)
    assert [int(a) for a in A] == want


@pytest.mark.parametrize("shape,k,cutoff,kind,seed", [
    ((128, 128, 128), 50, 3, "eq", 1),
    ((64, 64, 64), 50, 2, "matern52", 3),
    ((48, 40, 56), 60, 4, "matern32", 5),
    ((96, 80, 72), 40, 3, "eq", 7),
    # k > 90: nr(nr + 1) exceeds the window kernel's LDS row budget, so the factor rows take the
    # global-memory path (stage_rows / wave_new_row) for the late rounds
    ((48, 48, 48), 110, 3, "eq", 9),
])
def test_bounded_alg3_matches_c_oracle_at_scale(shape, k, cutoff, kind, seed):
    """GPU picks bit-exact against the CPU: the bounded-lazy algorithm 3 on the device and the
    plain-C restatement (oracle/c4_exact.c, tests/test_c4_oracle.py pins it to the dense oracle) on
    the host, at north_star's sizes (no dense matrix fits), with pick deltas within 1e-10."""
    from oracle import c4_exact as ce
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    X, ls = _grid(shape, seed=seed)
    A, d, _ = tapered_placement_algorithm_3(X, k, shape, cutoff, 4.0, kernel=kind, ls=ls,
                                            diag_shift=SHIFT, method="bounds")
    cp, cd = ce.exact_alg3(X, shape, k, cutoff, 4.0, kind=kind, ls=ls, diag_shift=SHIFT)
    assert [int(a) for a in A] == [int(a) for a in cp]
    np.testing.assert_allclose(d, cd, rtol=1e-10)

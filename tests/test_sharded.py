"""Multi-rank candidate-sharded placement with world_size 2 / 3 on gloo (CPU):
the orchestration (slab partition, delta all-gather, owner pivot all-reduce) must reproduce the
reference's selections exactly."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import placement as op
from tests.golden_io import placement_cases, placement_cov
from vgposp_amd.sharded_placement import slab_bounds

CASES = placement_cases()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grid_cov():
    from oracle import gp as ogp
    from vgposp_amd.data_generation import grid_points, grid_spacing
    X = grid_points((12, 10, 9), jitter=0.05, seed=0)
    return ogp.kernel_matrix("eq", X, X, 1.0, 2 * grid_spacing((12, 10, 9)))[0] + 0.010001 * np.eye(len(X))


def _chol_worker(rank, world, port, n, dist_min, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.numpy_greedy_backend import NumpyCholeskyOps
        from vgposp_amd.dist_cholesky import DistCholesky
        X = np.random.default_rng(5).uniform(-2, 2, (n, 3))
        S = np.exp(-0.5 * ((X[:, None] - X[None]) ** 2).sum(-1) / 0.6 ** 2) + 0.05 * np.eye(n)
        A = S.copy()
        dc = DistCholesky(NumpyCholeskyOps(A), dist_min=dist_min)
        dc.factor()
        out[rank] = (A, S, dc.exchanged)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,dist_min", [(2, 700, 129), (3, 700, 129), (3, 1000, 400),
                                              (4, 520, 129)])
def test_dist_cholesky_gloo(world, n, dist_min):
    """DistCholesky: each rank solves its share of every large node's panel and SYRK band; after
    the all-gathers every rank holds the full factor (the upper triangle keeps Sigma)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_chol_worker, args=(world, _free_port(), n, dist_min, out), nprocs=world, join=True)
    A0, S, ex = out[0]
    L = np.linalg.cholesky(S)
    lo = np.tril(np.ones((n, n), dtype=bool))
    assert ex > 0
    for r in range(world):
        A = out[r][0]
        np.testing.assert_allclose(A[lo], L[lo], rtol=1e-10, atol=1e-12)
        np.testing.assert_array_equal(A[~lo], S[~lo])


def test_share_bounds():
    from vgposp_amd.dist_cholesky import even_rows, lower_bands
    for n in (4096, 32768, 1000):
        for world in (1, 2, 3, 8):
            for f in (even_rows, lower_bands):
                e = f(n, world)
                assert e[0][0] == 0 and e[-1][1] == n
                assert all(a <= b for a, b in e)
                assert all(a % 128 == 0 for a, _ in e)
    bands = lower_bands(32768, 8)
    area = [b * (b + 1) / 2 - a * (a + 1) / 2 for a, b in bands]
    assert max(area) / min(area) < 1.1  # 128-row granularity


def _worker(rank, world, port, names, lazy, out, partition=False, dist_min=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.numpy_greedy_backend import NumpyGreedyBackend
        from vgposp_amd.sharded_placement import ShardedGreedyPlacement
        res = {}
        for name in names:
            e = {"k": 12} if name == "grid1080" else CASES[name]
            cov = _grid_cov() if name == "grid1080" else placement_cov(name, e)
            sh = ShardedGreedyPlacement(NumpyGreedyBackend(cov, e["k"]), partition_inverse=partition,
                                        align=4, dist_min=dist_min)
            A, _, _ = sh.run(e["k"], lazy=lazy)
            res[name] = [int(a) for a in A]
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("lazy", [True, False])
def test_sharded_matches_reference(world, lazy):
    names = ["cov4x4", "spd40", "grid4", "grid654"] if lazy else ["cov4x4", "spd40", "grid4"]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), names, lazy, out), nprocs=world, join=True)
    for r in range(world):
        for name in names:
            exp = CASES[name]["alg2" if lazy else "alg1"]
            assert out[r][name] == exp, (r, name)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dist_factor_matches_reference(world):
    """Partitioned inverse on a factor the ranks computed together (DistCholesky, every node above
    128 split): same picks as the precision oracle on a 1,080-point grid."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ["grid1080", "spd40"], True, out, True, 129),
             nprocs=world, join=True)
    exp = [int(a) for a in op.placement_lazy_precision(_grid_cov(), 12)]
    for r in range(world):
        assert out[r]["grid1080"] == exp, r
        assert out[r]["spd40"] == CASES["spd40"]["alg2"], r


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_partitioned_inverse_matches_reference(world):
    """Each rank forms only its slab's columns of L^-1 (the others are NaN in the numpy backend);
    the pick's column reaches every rank through the xcol sum-all-reduce."""
    names = ["cov4x4", "spd40", "grid4", "grid654"]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), names, True, out, True), nprocs=world, join=True)
    for r in range(world):
        for name in names:
            assert out[r][name] == CASES[name]["alg2"], (r, name)


def test_inverse_slabs():
    from vgposp_amd.sharded_placement import inverse_slabs
    n = 65536
    for world in (1, 2, 4, 8):
        sl = inverse_slabs(n, world)
        assert sl[0][0] == 0 and sl[-1][1] == n
        assert all(a % 128 == 0 and a <= b for a, b in sl)
        work = [(n - a) ** 3 - (n - b) ** 3 for a, b in sl]
        assert max(work) / min(work) < 1.05
    assert inverse_slabs(100, 2) == [(0, 0), (0, 100)]


def test_slab_bounds_balanced():
    n = 65536
    for world in (1, 2, 4, 8):
        sl = slab_bounds(n, world)
        assert sl[0][0] == 0 and sl[-1][1] == n
        assert all(a <= b for a, b in sl)
        work = [sum(n - c for c in range(a, b)) for a, b in sl] if n < 5000 else \
            [(b - a) * n - (b * (b - 1) - a * (a - 1)) / 2 for a, b in sl]
        assert max(work) / min(work) < 1.01
    assert slab_bounds(3, 4)[-1][1] == 3


def test_single_rank_numpy_backend_matches_oracle():
    from tests.numpy_greedy_backend import NumpyGreedyBackend
    from vgposp_amd.sharded_placement import ShardedGreedyPlacement
    for name in ["grid5", "randcov11"]:
        e = CASES[name]
        sh = ShardedGreedyPlacement(NumpyGreedyBackend(placement_cov(name, e), e["k"]))
        assert [int(a) for a in sh.run(e["k"])[0]] == e["alg2"]


def _singular_covs():
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, (48, 3))
    X[7] = X[3]                                      # duplicated location
    K = np.exp(-0.5 * ((X[:, None] - X[None]) ** 2).sum(-1) / 0.3 ** 2)
    T = rng.normal(size=(40, 12))                    # 12 samples < 40 locations
    return {"dup": K, "fewsamples": np.cov(T)}


def _singular_worker(rank, world, port, partition, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.numpy_greedy_backend import NumpyGreedyBackend
        from vgposp_amd.sharded_placement import ShardedGreedyPlacement
        res = {}
        for name, cov in _singular_covs().items():
            sh = ShardedGreedyPlacement(NumpyGreedyBackend(cov, 6), partition_inverse=partition,
                                        align=4)
            res[name] = [int(a) for a in sh.run(6)[0]]
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("partition", [False, True])
def test_sharded_singular_cov_matches_pinv(partition):
    """the sharded run takes the single-GPU jitter retry on a singular cov_vv (failed
    factorization or rounding-level pivot), decided identically on both ranks, and picks what
    the reference's pinv picks."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_singular_worker, args=(2, _free_port(), partition, out), nprocs=2, join=True)
    for name, cov in _singular_covs().items():
        exp = [int(a) for a in op.placement_algorithm_2(cov, 6)]
        for r in range(2):
            assert out[r][name] == exp, (r, name)

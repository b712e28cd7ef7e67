"""The epsilon-local APPROXIMATION of config C4 (vgposp_local_*; the exact C4 path is
sparse_placement, tests/test_gpu_exact.py) against the oracle's restatement of the same
approximation (snippets_a3.sparse_placement_algorithm_3 with local deltas) — picks bit-exact, the
delta_cached_iters snapshots to rounding — over every lane-group width (taper supports of 7, 27,
33 and 57 points), four kernels, window cutoffs 0-3, ragged grids, a 2-rank candidate-sharded run
on one GPU, and the full 128^3 k = 50 sequence."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import local_placement as lp
from vgposp_amd.data_generation import grid_points, grid_spacing

pytestmark = pytest.mark.gpu

SHIFT = 0.01 + 1e-6


def _grid(shape, seed=0):
    return grid_points(shape, jitter=0.05, seed=seed), 2.0 * grid_spacing(shape)


@pytest.mark.parametrize("shape,k,cutoff,beta,kind", [
    ((12, 11, 10), 12, 3, 4.0, "eq"),
    ((12, 11, 10), 12, 2, 3.0, "matern52"),
    ((10, 10, 9), 10, 3, 2.5, "eq"),
    ((9, 9, 9), 10, 3, 2.2, "matern32"),
    ((10, 9, 8), 8, 1, 4.0, "matern12"),
    ((8, 8, 8), 6, 0, 4.0, "eq"),
    ((16, 16, 16), 20, 3, 4.0, "eq"),
    ((2, 5, 40), 8, 2, 4.0, "eq"),
])
def test_local_alg3_matches_oracle(shape, k, cutoff, beta, kind):
    from vgposp_amd.local_placement import local_placement_algorithm_3
    X, ls = _grid(shape, seed=shape[0] + k)
    A, deltas, dci = local_placement_algorithm_3(X, k, shape, cutoff, beta, kernel=kind, ls=ls,
                                                 diag_shift=SHIFT, snapshots=True)
    rd = []
    rA, rcache, rdci = lp.local_placement_algorithm_3(X, shape, k, cutoff, beta, kind=kind, ls=ls,
                                                      diag_shift=SHIFT, snapshots=True, deltas=rd)
    assert [int(a) for a in A] == rA
    np.testing.assert_allclose(dci, rdci[:, :k], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(deltas, rd, rtol=1e-12)


def test_local_full_pass_all_candidates():
    """Round 0 of a 64 x 32 x 32 grid (65,536 candidates): every delta against the oracle."""
    import torch
    from vgposp_amd.local_placement import HipLocalBackend
    shape = (64, 32, 32)
    X, ls = _grid(shape, seed=7)
    for beta in (4.0, 2.5):
        b = HipLocalBackend(X, shape, 1, 3, beta, ls=ls, diag_shift=SHIFT)
        b.reset()
        b.score_all()
        torch.cuda.synchronize()
        b.check()
        ref = lp.local_deltas(X, shape, np.arange(len(X)), np.zeros(len(X), bool), beta, ls=ls,
                              diag_shift=SHIFT)
        np.testing.assert_allclose(b.local_cache().cpu().numpy(), ref, rtol=1e-12)


def test_local_128cube_k50_matches_oracle():
    """Config C4's workload on one GPU: 128^3 = 2,097,152 candidates, k = 50, beta = 4
    (BETA_val, main_architecture_2_sampledistribution.py:973), cutoff 3 (snippets_a3.py:374)."""
    from vgposp_amd.local_placement import local_placement_algorithm_3
    from vgposp_amd.workloads import c4_grid
    X, shape, ls = c4_grid()
    A, deltas, _ = local_placement_algorithm_3(X, 50, shape, 3, 4.0, ls=ls, diag_shift=SHIFT)
    rd = []
    rA, _, _ = lp.local_placement_algorithm_3(X, shape, 50, 3, 4.0, ls=ls, diag_shift=SHIFT,
                                              deltas=rd)
    assert [int(a) for a in A] == rA
    np.testing.assert_allclose(deltas, rd, rtol=1e-12)


@pytest.mark.parametrize("beta", [4.0, 3.0, 2.5])
def test_run_all_matches_rounds(beta):
    """vgposp_local_run (the persistent one-workgroup rounds for m <= 16, the launch sequence
    otherwise) picks what the round-by-round path and the oracle pick."""
    from vgposp_amd.local_placement import HipLocalBackend, LocalGreedyPlacement
    shape = (24, 20, 18)
    X, ls = _grid(shape, seed=13)
    b = HipLocalBackend(X, shape, 30, 3, beta, ls=ls, diag_shift=SHIFT)
    g = LocalGreedyPlacement(b)
    fused = g.run(30).cpu().tolist()
    d_fused = b.pick_delta.cpu().numpy().copy()
    rounds = g.run(30, snapshots=[]).cpu().tolist()
    rA, _, _ = lp.local_placement_algorithm_3(X, shape, 30, 3, beta, ls=ls, diag_shift=SHIFT)
    assert fused == rounds == rA
    np.testing.assert_array_equal(d_fused, b.pick_delta.cpu().numpy())


def test_local_not_pd_is_reported():
    from vgposp_amd.local_placement import HipLocalBackend
    shape = (6, 6, 6)
    X, ls = _grid(shape)
    b = HipLocalBackend(X, shape, 2, 3, 3.0, ls=ls, diag_shift=-0.999, jitter=0.0)
    b.reset()
    b.score_all()
    with pytest.raises(np.linalg.LinAlgError):
        b.check()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, k, cutoff, beta, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from vgposp_amd.local_placement import local_placement_algorithm_3
        X, ls = _grid(shape, seed=11)
        A, d, dci = local_placement_algorithm_3(X, k, shape, cutoff, beta, ls=ls,
                                                diag_shift=SHIFT, snapshots=True)
        out[rank] = ([int(a) for a in A], dci)
    finally:
        dist.destroy_process_group()


def test_local_two_ranks_on_one_gpu():
    """Candidate-sharded run (two plane slabs, key all-gather over gloo with host staging): the
    same picks as one rank, and each rank's cache slab equals the oracle's."""
    import torch.multiprocessing as mp
    from vgposp_amd.local_placement import plane_slabs
    shape, k, cutoff, beta = (12, 10, 9), 12, 3, 4.0
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(2, _free_port(), shape, k, cutoff, beta, out), nprocs=2, join=True)
    X, ls = _grid(shape, seed=11)
    rA, _, rdci = lp.local_placement_algorithm_3(X, shape, k, cutoff, beta, ls=ls,
                                                 diag_shift=SHIFT, snapshots=True)
    for r in range(2):
        A, dci = out[r]
        assert A == rA
        c0, c1 = plane_slabs(shape, 2)[r]
        np.testing.assert_allclose(dci, rdci[c0:c1], rtol=1e-12, atol=1e-15)

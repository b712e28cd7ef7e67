"""CPU checks of the exact C4 path's host side: the nested-dissection plan
(vgposp_amd.nested_dissection) and the batched multifrontal selected inversion it drives,
restated in numpy (tests/numpy_frontal_backend.py) against a dense inverse."""
import numpy as np
import pytest

from numpy_frontal_backend import selected_inverse_diag, tapered_entry_matrix
from vgposp_amd.data_generation import grid_points, grid_spacing
from vgposp_amd.taper import taper_support
from vgposp_amd.nested_dissection import FrontalTree, stencil_radius


@pytest.mark.parametrize("shape,beta,leaf", [
    ((6, 7, 8), 4.0, 40),
    ((5, 6, 7), 2.5, 30),
    ((8, 8, 8), 4.0, 64),
    ((3, 4, 20), 4.0, 10),
    ((2, 2, 9), 4.0, 2),
    ((4, 4, 4), 4.0, 512),     # a single leaf front
])
def test_selected_inverse_matches_dense(shape, beta, leaf):
    offs, tau = taper_support(beta)
    X = grid_points(shape, jitter=0.05, seed=1)
    h = 2.0 * grid_spacing(shape)
    C = tapered_entry_matrix(X, shape, offs, tau, lambda r2: np.exp(-0.5 * r2 / h ** 2),
                             0.01 + 1e-6, 1e-6)
    T = FrontalTree(shape, offs, leaf=leaf, pad=4)
    d = selected_inverse_diag(T, C)
    np.testing.assert_allclose(d, np.diag(np.linalg.inv(C)), rtol=1e-12)


@pytest.mark.parametrize("shape,beta", [((16, 16, 16), 4.0), ((12, 9, 10), 2.5),
                                        ((64, 32, 32), 4.0)])
def test_plan_invariants(shape, beta):
    offs, _ = taper_support(beta)
    T = FrontalTree(shape, offs, leaf=512)
    n = int(np.prod(shape))
    assert T.r == max(stencil_radius(offs), 1)
    # every node is a pivot of exactly one front, at its recorded position
    seen = np.zeros(n, dtype=int)
    for f in T.fronts:
        seen[f.piv] += 1
    assert np.all(seen == 1)
    for g in T.groups:
        assert g.p % 16 == 0 and g.u % 16 == 0
        assert g.p >= g.p_max and g.u >= g.u_max
        for s, fi in enumerate(g.fronts):
            f = T.fronts[fi]
            np.testing.assert_array_equal(g.piv[s, :len(f.piv)], f.piv)
            assert np.all(g.piv[s, len(f.piv):] == -1)
            assert np.all(np.diff(g.U[s, :g.ulen[s]]) > 0)
            if f.parent >= 0:
                # the parent-front positions of U are in range and distinct
                pg = T.groups[g.parent_group[s]]
                m = g.pmap[s, :g.ulen[s]]
                assert np.all((m >= 0) & (m < pg.p + pg.u))
                assert len(np.unique(m)) == len(m)
    # groups are in a valid bottom-up order (children before parents)
    for gi, g in enumerate(T.groups):
        assert np.all((g.parent_group > gi) | (g.parent_group < 0))


def test_plan_128cube_sizes():
    """The C4 plan: 13 levels, the root separator is one 128 x 128 plane, ~8.7e13 flops, and the
    size-bucketed groups pad away less than 5 % of them."""
    offs, _ = taper_support(4.0)
    T = FrontalTree((128, 128, 128), offs, leaf=512)
    assert len(T.levels) == 13
    assert T.groups[-1].p == 128 * 128 and T.groups[-1].u == 0
    assert 8e13 < T.flops(padded=False) < 9.5e13
    assert T.flops(padded=True) < 1.05 * T.flops(padded=False)
    # level offsets tile each level's buffers exactly
    for lvl in T.levels:
        end = [0, 0, 0]
        for gi in lvl["groups"]:
            g = T.groups[gi]
            assert list(g.off) == end
            end = [end[0] + g.nf * g.p * g.p, end[1] + g.nf * g.u * g.p, end[2] + g.nf * g.u * g.u]
        assert end == lvl["size"]


def _problem(shape, beta=4.0):
    from numpy_frontal_backend import tapered_entry_matrix
    offs, tau = taper_support(beta)
    X = grid_points(shape, jitter=0.05, seed=2)
    h = 2.0 * grid_spacing(shape)
    C = tapered_entry_matrix(X, shape, offs, tau, lambda r2: np.exp(-0.5 * r2 / h ** 2),
                             0.01 + 1e-6, 1e-6)
    return X, offs, C


class _Prob:
    """The parts of sparse_placement.TaperProblem the orchestration reads."""

    def __init__(self, shape, offs):
        self.shape = tuple(shape)
        self.offs_np = np.asarray(offs).reshape(-1, 3)
        self.n = int(np.prod(shape))


def _selinv_worker(rank, world, port, shape, beta, leaf, out):
    import os

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from numpy_frontal_ops import TorchCpuFrontalOps
        from vgposp_amd.sparse_placement import FrontComm, FrontalSelectedInverse
        X, offs, C = _problem(shape, beta)
        comm = FrontComm() if world > 1 else None
        fs = FrontalSelectedInverse(_Prob(shape, offs), leaf=leaf, comm=comm,
                                    ops=TorchCpuFrontalOps(C))
        q = fs.run().numpy().copy()
        fs.check()
        out[rank] = (q, comm.bytes if comm else 0)
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world,shape,beta,leaf", [
    (1, (6, 7, 8), 4.0, 40),
    (2, (6, 7, 8), 4.0, 40),
    (4, (8, 7, 6), 4.0, 24),
    (8, (8, 8, 6), 4.0, 24),
    (2, (5, 6, 7), 2.5, 30),
])
def test_distributed_selected_inverse_gloo(world, shape, beta, leaf):
    """The subtree-to-subcube selected inverse over `world` gloo ranks (updates and Q_UU blocks
    sent between ranks, diag(Q) summed) equals the dense inverse's diagonal on every rank."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    _, _, C = _problem(shape, beta)
    ref = np.diag(np.linalg.inv(C))
    if world == 1:
        out = {}
        _selinv_worker(0, 1, port, shape, beta, leaf, out)
    else:
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(_selinv_worker, args=(world, port, shape, beta, leaf, out), nprocs=world,
                 join=True)
    for r in range(world):
        np.testing.assert_allclose(out[r][0], ref, rtol=1e-12)
    if world > 1:
        assert sum(out[r][1] for r in range(world)) > 0

"""Data-parallel VGP training step: the N observations sharded over 2 ranks (both on
cuda:0, gloo with host staging) must give the single-process loss and gradient: the only
cross-rank data are the M^2 + M forward partials and the 2 + M d backward partials."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gp as ogp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(21)
    g = (np.arange(3) - 1.0) * 0.9
    Z = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    X = rng.uniform(-1.4, 1.4, (4001, 3))
    y = np.sin(2 * X).sum(1) + rng.normal(0, 0.1, len(X))
    idx = rng.integers(0, len(X), 64)
    return X, y, Z, idx


def _worker(rank, world, port, out):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vgposp_amd.vgp_training import VGPObjective
        X, y, Z, idx = _problem()
        shard = np.array_split(np.arange(len(X)), world)[rank]
        obj = VGPObjective("matern52", X[shard], y[shard], group=dist.group.WORLD)
        L, ga, gl, gs, gZ = obj.loss_and_grads(Z, 0.9, 0.7, 0.05, X[idx], y[idx], 64 / len(X))
        out[rank] = (float(L), float(ga), float(gl), float(gs), gZ.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_vgp_data_parallel_two_ranks():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    X, y, Z, idx = _problem()
    rL, rga, rgl, rgs, rgZ = ogp.vgp_training_loss_grads("matern52", Z, X, y, X[idx], y[idx], 0.9,
                                                         0.7, 0.05, 64 / len(X))
    for r in range(2):
        L, ga, gl, gs, gZ = out[r]
        assert L == pytest.approx(rL, rel=1e-8)
        np.testing.assert_allclose([ga, gl, gs], [rga, rgl, rgs], rtol=1e-6)
        np.testing.assert_allclose(gZ, rgZ, rtol=1e-6, atol=1e-8 * np.abs(rgZ).max())
    # both ranks hold identical results (replicated M x M work after the reductions)
    assert out[0][0] == out[1][0]


def _train_worker(rank, world, port, out, precision):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph
        X, y, Z = vgp_c3_data(n=24, m=4, half=4.0)
        N = len(X)
        B = 1024
        shard = np.array_split(np.arange(N), world)[rank]
        train_op, _, xb, yb = vgp_c3_graph(X[shard], y[shard], Z, B, precision=precision,
                                           group=dist.group.WORLD, n_total=N)
        rng = np.random.default_rng(3)
        Xd, yd = torch.as_tensor(X, device="cuda"), torch.as_tensor(y, device="cuda")
        idx = [torch.as_tensor(rng.integers(0, N, B), device="cuda") for _ in range(6)]
        losses = [float(train_op.run({xb: Xd[i], yb: yd[i]})) for i in idx]
        train_op.check()
        out[rank] = (losses, bool(train_op.graph), len(train_op._g[0]) if train_op._g else 0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["fp64", "mixed:2"])
def test_vgp_data_parallel_graph_segments(precision):
    """Verdict r3 item 6: the data-parallel training step is graph-replayed as three segments
    around its two all-reduces; the 2-rank losses equal the single-process ones."""
    import torch

    from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_train_worker, args=(2, _free_port(), out, precision), nprocs=2, join=True)
    X, y, Z = vgp_c3_data(n=24, m=4, half=4.0)
    N, B = len(X), 1024
    train_op, _, xb, yb = vgp_c3_graph(X, y, Z, B, precision=precision)
    rng = np.random.default_rng(3)
    Xd, yd = torch.as_tensor(X, device="cuda"), torch.as_tensor(y, device="cuda")
    idx = [torch.as_tensor(rng.integers(0, N, B), device="cuda") for _ in range(6)]
    ref = [float(train_op.run({xb: Xd[i], yb: yd[i]})) for i in idx]
    train_op.check()
    for r in range(2):
        losses, graph, nseg = out[r]
        assert graph and nseg == 3, (graph, nseg)
        np.testing.assert_allclose(losses, ref, rtol=1e-12)
    assert out[0][0] == out[1][0]

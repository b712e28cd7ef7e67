"""Synthetic workloads of BASELINE.json's configs, shared by bench.py and tools/.

* ``placement_split``: one 64 x 32 x 32 split (N = 65,536) of the greedy benchmark: a jittered
  grid (seed = rank, shifted along axis 0 by rank), EQ kernel, amp 1, ls = 2h, noise 1e-2 + 1e-6.
* ``c2_data``: config C2, the 32^3 grid for K assembly + potrf.
* ``vgp_c5_data``: config C5, 5-D uniform observations with a 4^5 inducing grid (M = 1,024).
* ``vgp_c3``: config C3.  N = 64^3 observations on a grid over [-7, 7]^3, M = 8^3 inducing points
  on the sub-grid (spacing 2, twice the initial length scale, so the unjittered Kzz whose log-det
  the KL term needs stays well conditioned).  Target y = sum_d exp(-x_d^2 / 20) sin(x_d) +
  N(0, 0.1^2), the 3-D form of variational_Gaussian_process_example.py:29-37.  Trainables
  initialised as the reference's (:51-64): softplus(0.54) amplitude and noise,
  1e-5 + softplus(0.54) length scale, the inducing points; Adam(0.01), minibatch B.
"""
from __future__ import annotations

import numpy as np

from .data_generation import grid_points, grid_spacing


def placement_split(shape=(64, 32, 32), rank=0):
    h = grid_spacing(shape)
    X = grid_points(shape, jitter=0.05, seed=rank)
    X[:, 0] += rank * shape[0] * h
    return X, 2.0 * h


def vgp_c3_data(n=64, m=8, half=7.0, seed=0):
    g = np.linspace(-half, half, n)
    X = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    rng = np.random.default_rng(seed)
    y = np.sum(np.exp(-X ** 2 / 20.0) * np.sin(X), axis=1) + rng.normal(0, 0.1, len(X))
    gz = np.linspace(-half, half, m)
    Z = np.stack(np.meshgrid(gz, gz, gz, indexing="ij"), -1).reshape(-1, 3)
    return X, y, Z


def vgp_c5_data(n=65536, m=4, d=5, half=2.0, seed=0):
    """Config C5: X ~ U[-2, 2]^5 (N = 65,536), M = 4^5 = 1,024 inducing points on a grid (spacing
    4/3 > the initial length scale, so the unjittered Kzz stays well conditioned), the d-dim form
    of the C3 target."""
    rng = np.random.default_rng(seed)
    X = rng.uniform(-half, half, (n, d))
    y = np.sum(np.exp(-X ** 2 / 20.0) * np.sin(X), axis=1) + rng.normal(0, 0.1, n)
    gz = np.linspace(-half, half, m)
    Z = np.stack(np.meshgrid(*([gz] * d), indexing="ij"), -1).reshape(-1, d)
    return X, y, Z


def c2_data(n=32, half=2.0):
    """Config C2: a 32^3 grid over linspace(-2, 2) per axis (N = 32,768), EQ amp 1, ls = 2h,
    noise 1e-2 + 1e-6."""
    shape = (n, n, n)
    X = grid_points(shape)
    return X, 2.0 * grid_spacing(shape)


def c4_grid(n=128, seed=0):
    """Config C4: the 128^3 jittered grid (N = 2,097,152) of the local-kernel greedy, EQ amp 1,
    ls = 2h -> (X, shape, ls)."""
    shape = (n, n, n)
    return grid_points(shape, jitter=0.05, seed=seed), shape, 2.0 * grid_spacing(shape)


def vgp_c3_graph(X, y, Z, B, lr=0.01, precision="fp64", group=None, n_total=None, kernel="eq",
                 **train_options):
    """The reference's training graph (variational_Gaussian_process_example.py:51-102) in this
    package's API -> (train_op, loss, x_batch placeholder, y_batch placeholder).  ``group``: the
    observations (X, y) are this rank's shard of ``n_total`` (data-parallel optimal posterior,
    two all-reduces per step); every rank feeds the same minibatch.  ``train_options``: the
    VGPTrainOp scheduling switches (graph, streams, fused_params, grouped)."""
    from . import distributions as tfd
    from . import psd_kernels as tfkern
    from .optimizers import AdamOptimizer
    from .variables import Softplus, Variable, placeholder
    amp = Softplus(Variable(0.54, name="amplitude"), offset=0.0)
    ls = Softplus(Variable(0.54, name="length_scale"), offset=1e-5)
    # C3 follows variational_Gaussian_process_example.py:55-57 (ExponentiatedQuadratic); C5 the
    # arch-2 VGP's MaternFiveHalves (main_architecture_2_sampledistribution.py:211)
    cls = {"eq": tfkern.ExponentiatedQuadratic, "matern52": tfkern.MaternFiveHalves,
           "matern32": tfkern.MaternThreeHalves, "matern12": tfkern.MaternOneHalf}[kernel]
    kernel = cls(amplitude=amp, length_scale=ls)
    noise = Softplus(Variable(0.54, name="observation_noise_variance"), offset=0.0)
    Zv = Variable(Z, name="inducing_index_points")
    loc, scale = tfd.VariationalGaussianProcess.optimal_variational_posterior(
        kernel=kernel, inducing_index_points=Zv, observation_index_points=X, observations=y,
        observation_noise_variance=noise)
    vgp = tfd.VariationalGaussianProcess(kernel, index_points=Z[:8], inducing_index_points=Zv,
                                         variational_inducing_observations_loc=loc,
                                         variational_inducing_observations_scale=scale,
                                         observation_noise_variance=noise)
    xb = placeholder(np.float64, [B, X.shape[1]], name="x_train_batch")
    yb = placeholder(np.float64, [B], name="y_train_batch")
    loss = vgp.variational_loss(observations=yb, observation_index_points=xb,
                                kl_weight=float(B) / float(n_total or len(X)))
    return (AdamOptimizer(learning_rate=lr).minimize(loss, group=group, precision=precision,
                                                     **train_options), loss, xb, yb)

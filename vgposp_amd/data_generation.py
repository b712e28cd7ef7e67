"""Synthetic inputs for the hot path (host side, numpy).

Mirrors the reference's generators:

* ``sinusoid``                  <- ``gp_functions.py:78-95``  (y = sum_d sin(2*pi*x_d), SIN_DENSITY=2)
* ``random_noise``              <- ``data_generation.py:76-79``
* ``generate_2D_data`` / ``generate_1D_data`` <- ``data_generation.py:24-50``
* ``generate_noisy_2Dsin_data`` / ``generate_noisy_1Dsin_data`` <- ``data_generation.py:53-73``
* ``create_random_cov``         <- ``data_generation.py:92-95``
* ``grid_points``               the C-order sensor grid of SURVEY §8(d): flat index
  ``i = i0*I1*I2 + i1*I2 + i2`` as in ``main.py:259-267`` / ``cache_plot_gen_idxs.py:22-30``.

Every generator takes an optional ``rng`` (``numpy.random.Generator``); with ``rng=None`` the
global ``np.random`` state is used exactly as the reference does.
"""
from __future__ import annotations

import numpy as np

SIN_DENSITY = 2


def _rng(rng):
    return np.random if rng is None else rng


def sinusoid(x, scale=1):
    """gp_functions.py:78-95 — sum over feature columns of sin(2*pi*x_d)."""
    x = np.asarray(x)
    s = 0
    if 1 < len(x.shape):
        for i in range(x.shape[1]):
            s += np.sin(SIN_DENSITY * np.pi * x[:, i])
    else:
        s += np.sin(SIN_DENSITY * np.pi * x[:])
    return s


def random_noise(loc, var, num, rng=None):
    """data_generation.py:76-79."""
    return _rng(rng).normal(loc=loc, scale=np.sqrt(var), size=(num))


def generate_2D_data(num_train_pts, coord_range, rng=None):
    """data_generation.py:24-38."""
    idx_pts = _rng(rng).uniform(0., 1., (num_train_pts, 2)).astype(np.float64)
    for d in range(2):
        scale = coord_range[d][1] - coord_range[d][0]
        idx_pts[:, d] *= scale
        idx_pts[:, d] += coord_range[d][0]
    return idx_pts


def generate_1D_data(num_train_pts, coord_range, rng=None):
    """data_generation.py:41-50."""
    idx_pts = _rng(rng).uniform(0., 1., (num_train_pts)).astype(np.float64)
    idx_pts *= coord_range[1] - coord_range[0]
    idx_pts += coord_range[0]
    return idx_pts


def generate_noisy_2Dsin_data(num_train_pts, obs_noise_variance, coord_range, rng=None):
    """data_generation.py:53-61."""
    idx_pts = generate_2D_data(num_train_pts, coord_range, rng)
    noise = random_noise(0, obs_noise_variance, num_train_pts, rng)
    return idx_pts, sinusoid(idx_pts) + noise


def generate_noisy_1Dsin_data(num_train_pts, obs_noise_variance, coord_range, rng=None):
    """data_generation.py:64-73."""
    idx_pts = generate_1D_data(num_train_pts, coord_range, rng)
    noise = random_noise(0, obs_noise_variance, num_train_pts, rng)
    return idx_pts, sinusoid(idx_pts) + noise


def generate_random_points(num_pts, range_val, rng=None):
    """data_generation.py:82-84 — (num_pts, 2) uniform points in [range_val[0], range_val[1])."""
    return _rng(rng).uniform(range_val[0], range_val[1], size=(num_pts, 2))


def create_line(u, v):
    """data_generation.py:87-89."""
    return np.asarray(u) - np.asarray(v)


def _polynomial_columns(degree, num=1200, rng=None):
    col = _rng(rng).uniform(size=(num, 1))
    return np.concatenate([col ** p for p in range(1, degree + 1)], axis=1).astype(np.float64)


def generate_6d_polinomials(rng=None):
    """data_generation.py:98-109 — rows (o, o^2, ..., o^6), o ~ U(0, 1), 1200 rows."""
    return _polynomial_columns(6, rng=rng)


def generate_4d_polinomials(rng=None):
    """data_generation.py:112-122 — rows (o, o^2, o^3, o^4), o ~ U(0, 1), 1200 rows."""
    return _polynomial_columns(4, rng=rng)


def create_random_cov(n, rng=None):
    """data_generation.py:92-95 — U U^T with U ~ U(0,1)^{n x n}."""
    m = _rng(rng).uniform(0, 1, n ** 2).reshape(-1, n)
    return np.dot(m, m.T)


def grid_spacing(shape, extent=4.0):
    """Uniform spacing h: the smallest axis with more than one point spans ``extent``
    (linspace(-2, 2, n) for a cube); ``extent`` for a single point."""
    n = min((int(s) for s in shape if int(s) > 1), default=2)
    return extent / (n - 1)


def grid_points(shape=(8, 8, 8), jitter=0.0, seed=0, extent=4.0):
    """SURVEY §8(d) sensor grid, flattened in C order (i0 slowest).

    Axis k has ``shape[k]`` points spaced ``h = grid_spacing(shape)`` and centred on 0, so a cube
    is ``linspace(-2, 2, n)`` per axis (``main_GP_fit.py:114``).  ``jitter`` > 0 adds
    ``U(-jitter, jitter) * h`` per coordinate from ``default_rng(seed)``; it breaks the grid's
    exact octant ties so that selected indices are decided by the data, not by rounding.
    """
    shape = tuple(int(s) for s in shape)
    h = grid_spacing(shape, extent)
    axes = [(np.arange(n, dtype=np.float64) - (n - 1) / 2.0) * h for n in shape]
    if all(n == shape[0] for n in shape):
        axes = [np.linspace(-extent / 2, extent / 2, n) for n in shape]
    X = np.stack(np.meshgrid(*axes, indexing="ij"), axis=-1).reshape(-1, len(shape))
    if jitter:
        rng = np.random.default_rng(seed)
        X = X + rng.uniform(-jitter, jitter, X.shape) * h
    return np.ascontiguousarray(X)


def grid_observations(X, noise_var=1e-3, seed=1):
    """Target of SURVEY §8(d): y = sinusoid(X) + N(0, noise_var) from default_rng(seed)."""
    rng = np.random.default_rng(seed)
    return sinusoid(X) + rng.normal(0.0, np.sqrt(noise_var), X.shape[0])


def flat_to_grid_index(i, shape):
    """Flat C-order index -> (i0, i1, i2) (cache_plot_gen_idxs.py:9-34)."""
    return np.unravel_index(np.asarray(i), shape)

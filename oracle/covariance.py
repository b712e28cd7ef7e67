"""Oracle (TEST INFRASTRUCTURE ONLY): numpy restatements of the reference's cov_vv builders.

* ``tfp_covariance(x, y)``: tfp.stats.covariance(x, y, sample_axis=0, event_axis=None) as called
  pair by pair at main.py:194-199 and main_architecture_2_sampledistribution.py:470-479:
  mean over samples of (x - mean x)(y - mean y) (biased).  TFP is absent: restated (unpinned).
* ``empirical_cov``: that, for every pair of locations, after the reference's standardisation
  t = (tracers - tr_mean) / tr_stdev (main.py:190-193).
* ``index_taper``: the beta-decay local kernel filter (main_architecture_2_sampledistribution.py:
  361-421): decay = exp(-(beta * delta)^2 / (2 pi)), entries with decay < 0.01 set to 0,
  delta = Euclidean distance of the grid indices (C-order flattening, main.py:259-267).
"""
from __future__ import annotations

import numpy as np


def tfp_covariance(x, y):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    return np.mean((x - x.mean()) * (y - y.mean()))


def empirical_cov(T, tr_mean=0.0, tr_stdev=1.0):
    t = (np.asarray(T, dtype=np.float64) - tr_mean) / tr_stdev
    tc = t - t.mean(axis=1, keepdims=True)
    return tc @ tc.T / t.shape[1]


def index_taper(C, cover, beta, threshold=0.01):
    I0, I1, I2 = cover
    n = I0 * I1 * I2
    idx = np.stack(np.unravel_index(np.arange(n), (I0, I1, I2)), axis=1).astype(np.float64)
    delta = np.sqrt(((idx[:, None, :] - idx[None, :, :]) ** 2).sum(-1))
    g = np.exp(-np.square(beta * delta) / (2 * np.pi))
    out = np.asarray(C, dtype=np.float64) * g
    out[g < threshold] = 0.0
    return out

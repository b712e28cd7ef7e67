"""PSD kernels with the ``tfp.positive_semidefinite_kernels`` surface the reference uses
(``from tensorflow_probability import positive_semidefinite_kernels as tfkern``):

* ``ExponentiatedQuadratic(amplitude, length_scale, feature_ndims=1)``
  (3D_sin_wave.py:158-159, main_tests.py:617-619, variational_Gaussian_process_example.py:55-57)
* ``MaternOneHalf`` (gp_functions.py:160-163, main.py:94)
* ``MaternThreeHalves``
* ``MaternFiveHalves`` (main_architecture_2_sampledistribution.py:211)

``amplitude`` / ``length_scale`` are floats, arrays (a shape-[B] value gives a batch of B kernels,
NOT ARD — as with the reference's shape-[2] AMPLITUDE_INIT, main_GP_fit.py:117-118), device
tensors, or trainable ``variables.Softplus`` views.  ``matrix(x1, x2)`` assembles K on the GPU
(libvgposp ``vgposp_kernel_matrix``) and returns a float64 device tensor [B, n, m]
(or [n, m] when the kernel is not batched).
"""
from __future__ import annotations

import numpy as np
import torch

from . import linalg
from .variables import batch_size, resolve


class PositiveSemidefiniteKernel:
    kind = None

    def __init__(self, amplitude=None, length_scale=None, feature_ndims=1, validate_args=False,
                 name=None):
        if feature_ndims != 1:
            raise NotImplementedError("only feature_ndims=1 (the reference's setting) is supported")
        self.amplitude = amplitude
        self.length_scale = length_scale
        self.feature_ndims = feature_ndims
        self.validate_args = validate_args
        self.name = name or type(self).__name__

    # -- parameters ---------------------------------------------------------------------------
    @property
    def batch_size(self):
        return batch_size(self.amplitude, self.length_scale)

    @property
    def batch_shape(self):
        B = self.batch_size
        shaped = any(hasattr(p, "shape") and tuple(getattr(p, "shape")) != ()
                     for p in (self.amplitude, self.length_scale) if p is not None)
        return (B,) if shaped else ()

    def params(self):
        B = self.batch_size
        amp = resolve(self.amplitude, B)
        ls = resolve(self.length_scale, B)
        if self.validate_args:
            if not bool((amp > 0).all()) or not bool((ls > 0).all()):
                raise ValueError("amplitude and length_scale must be positive")
        return amp, ls

    # -- evaluation ---------------------------------------------------------------------------
    def matrix(self, x1, x2, diag_shift=None, lower=False, keep_batch=None):
        amp, ls = self.params()
        K = linalg.kernel_matrix(self.kind, _pts(x1), _pts(x2), amp, ls, diag_shift=diag_shift,
                                 lower=lower)
        if keep_batch is None:
            keep_batch = self.batch_shape != ()
        return K if keep_batch else K[0]

    def apply(self, x1, x2):
        """k(x1_i, x2_i) for paired rows: the diagonal of matrix(x1, x2) (device tensor)."""
        K = self.matrix(x1, x2, keep_batch=True)
        out = torch.diagonal(K, dim1=-2, dim2=-1)
        return out if self.batch_shape != () else out[0]

    def __repr__(self):
        return f"{self.name}(amplitude={self.amplitude!r}, length_scale={self.length_scale!r})"


def _pts(x):
    if hasattr(x, "shape") and len(x.shape) == 1:
        return x.reshape(-1, 1) if hasattr(x, "reshape") else np.asarray(x).reshape(-1, 1)
    if hasattr(x, "shape") and len(x.shape) == 3:  # [batch=1, n, d] index points
        if x.shape[0] != 1:
            raise NotImplementedError("batched index points must have batch size 1")
        return x[0]
    return x


class ExponentiatedQuadratic(PositiveSemidefiniteKernel):
    kind = "eq"


class MaternOneHalf(PositiveSemidefiniteKernel):
    kind = "matern12"


class MaternThreeHalves(PositiveSemidefiniteKernel):
    kind = "matern32"


class MaternFiveHalves(PositiveSemidefiniteKernel):
    kind = "matern52"

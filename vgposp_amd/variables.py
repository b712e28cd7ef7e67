"""Trainable parameters (eager stand-ins for the reference's TF1 variables).

* ``Variable``  <- ``tf.Variable(initial_value=INIT, dtype=np.float64)`` (gp_functions.py:127-130):
  a float64 device tensor that optimizers update in place.
* ``Softplus``  <- the constrained view ``np.finfo(np.float64).tiny + tf.nn.softplus(var)``
  (gp_functions.py:131-134); ``offset`` covers the VGP example's ``1e-5 + softplus`` length
  scale and plain ``softplus`` (variational_Gaussian_process_example.py:47-61).
* ``assign_inverse_softplus`` <- ``invert_softplus`` (gp_functions.py:106-109): var <- log(e^x - 1).

The small elementwise transforms run as torch device ops (plumbing); every heavy computation that
consumes the values runs in libvgposp.
"""
from __future__ import annotations

import numpy as np
import torch

from . import linalg

TINY = float(np.finfo(np.float64).tiny)


class Variable:
    def __init__(self, initial_value, name=None, trainable=True, dtype=np.float64):
        if dtype not in (np.float64, torch.float64, "float64"):
            raise TypeError("vgposp_amd variables are float64 (the reference uses np.float64)")
        self.value = linalg.as_device(np.asarray(initial_value, dtype=np.float64))
        self.name = name
        self.trainable = trainable

    @property
    def shape(self):
        return tuple(self.value.shape)

    def numpy(self):
        return self.value.detach().cpu().numpy()

    def assign(self, value):
        self.value.copy_(linalg.as_device(np.asarray(value, dtype=np.float64)).reshape(self.value.shape))
        return self

    def _rebind(self, tensor):
        """Make this variable a view into an optimizer's flat parameter buffer."""
        tensor.copy_(self.value.reshape(tensor.shape))
        self.value = tensor.view(self.value.shape) if self.value.dim() else tensor.view(())

    def __repr__(self):
        return f"Variable({self.name!r}, {self.numpy()!r})"


class Softplus:
    """offset + softplus(var): a positive parameter backed by an unconstrained Variable."""

    def __init__(self, var, offset=TINY):
        self.var = var if isinstance(var, Variable) else Variable(var)
        self.offset = float(offset)

    def value(self):
        return self.offset + torch.nn.functional.softplus(self.var.value)

    def dvalue_dvar(self):
        return torch.sigmoid(self.var.value)

    def numpy(self):
        return self.value().detach().cpu().numpy()

    @property
    def shape(self):
        return self.var.shape

    def assign_inverse_softplus(self, x):
        """invert_softplus (gp_functions.py:106-109): var <- log(exp(x - offset) - 1)."""
        x = np.asarray(x, dtype=np.float64) - (self.offset if self.offset != TINY else 0.0)
        self.var.assign(np.log(np.exp(x) - 1.0))
        return self.numpy()

    def __repr__(self):
        return f"Softplus({self.numpy()!r})"


class Placeholder:
    """``tf.placeholder`` stand-in: a named slot filled from ``Session.run(..., feed_dict)``."""

    def __init__(self, shape=None, name=None, dtype=np.float64):
        self.shape = shape
        self.name = name
        self.dtype = dtype

    def __repr__(self):
        return f"Placeholder({self.name!r}, shape={self.shape})"


def placeholder(dtype=np.float64, shape=None, name=None):
    """tf.placeholder(DTYPE, shape, name) (variational_Gaussian_process_example.py:89-90)."""
    return Placeholder(shape, name, dtype)


def fed(x, feed):
    """Value of ``x``: looked up in ``feed`` when it is a Placeholder."""
    if isinstance(x, Placeholder):
        if feed is None or x not in feed:
            raise KeyError(f"feed_dict lacks a value for {x!r}")
        return feed[x]
    return x


def resolve(x, B=None):
    """Current value of a parameter-like as a 1-D float64 device tensor (optionally broadcast)."""
    if x is None:
        t = linalg.as_device([1.0])
    elif isinstance(x, Softplus):
        t = x.value().reshape(-1)
    elif isinstance(x, Variable):
        t = x.value.reshape(-1)
    elif isinstance(x, torch.Tensor):
        t = linalg.as_device(x).reshape(-1)
    else:
        t = linalg.as_device(np.atleast_1d(np.asarray(x, dtype=np.float64))).reshape(-1)
    if B is not None and t.numel() == 1 and B > 1:
        t = t.expand(B).contiguous()
    return t


def batch_size(*params):
    sizes = [int(np.prod(p.shape)) if hasattr(p, "shape") and p.shape != () else 1
             for p in params if p is not None and not isinstance(p, (int, float))]
    sizes = [s for s in sizes if s > 1]
    if not sizes:
        return 1
    if len(set(sizes)) != 1:
        raise ValueError(f"parameter batch shapes do not broadcast: {sizes}")
    return sizes[0]

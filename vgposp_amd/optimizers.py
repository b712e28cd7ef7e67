"""TF1 ``AdamOptimizer`` and training ops for the GP fit loop, device-resident.

Replaces ``tf.train.AdamOptimizer(lr).minimize(-log_likelihood)`` built by
``gp_functions.tf_train_gp_adam`` (gp_functions.py:179-182) and run by
``tf_optimize_model_params`` (gp_functions.py:228-259).

The trainable variables of a GP (softplus-constrained amplitude[B], length_scale[B] and the noise
variance) are re-bound as views into ONE flat device buffer; each step computes the LML and its
analytic gradient in libvgposp (Cholesky + inverse + gradient reduction), applies the chain rule
through softplus, and updates the buffer with the ``vgposp_adam_update`` HIP kernel.  Nothing is
copied to the host inside the loop.
"""
from __future__ import annotations

import ctypes

import torch

from . import linalg
from ._lib import call
from .variables import Softplus, Variable


class AdamOptimizer:
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 name="Adam"):
        self.lr = float(learning_rate)
        self.beta1 = float(beta1)
        self.beta2 = float(beta2)
        self.epsilon = float(epsilon)
        self.name = name

    def minimize(self, loss, var_list=None):
        """``loss``: a ``distributions.LogProb`` to MAXIMISE (the reference passes ``-feature``;
        see ``negate``) or a ``Negated`` LogProb.  Returns a ``GPTrainOp``."""
        if isinstance(loss, Negated):
            return GPTrainOp(loss.log_prob, self, var_list)
        raise TypeError("minimize() expects -log_prob (a Negated LogProb); "
                        "use gp_functions.tf_train_gp_adam(log_likelihood, lr)")


class Negated:
    def __init__(self, log_prob):
        self.log_prob = log_prob


def negate(log_prob):
    return Negated(log_prob)


class GPTrainOp:
    """One TF1-Adam step on -sum_b LML_b of an exact GaussianProcess; ``run()`` returns the
    pre-update LML [B] (device tensor), as sess.run([train_op, log_likelihood]) does."""

    def __init__(self, log_prob, opt, var_list=None):
        self.gp = log_prob.dist
        self.observations = log_prob.observations
        self.opt = opt
        k = self.gp.kernel
        self.views = {"amp": k.amplitude, "ls": k.length_scale,
                      "noise": self.gp.observation_noise_variance}
        self.trainable = [(name, v) for name, v in self.views.items()
                          if isinstance(v, Softplus) and v.var.trainable
                          and (var_list is None or v.var in var_list or v in var_list)]
        sizes = [v.var.value.numel() for _, v in self.trainable]
        n = max(sum(sizes), 1)
        dev = linalg.device()
        self.theta = torch.zeros(n, dtype=torch.float64, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float64, device=dev)
        self.m = torch.zeros(n, dtype=torch.float64, device=dev)
        self.v = torch.zeros(n, dtype=torch.float64, device=dev)
        self.step_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.slices = {}
        off = 0
        for (name, sp), sz in zip(self.trainable, sizes):
            sp.var._rebind(self.theta[off:off + sz])
            self.slices[name] = (off, sz, sp)
            off += sz

    def run(self, observations=None):
        obs = self.observations if observations is None else observations
        lml, ga, gl, gn = self.gp.log_prob_and_grads(obs)
        B = lml.numel()
        for name, g in (("amp", ga), ("ls", gl), ("noise", gn)):
            if name not in self.slices:
                continue
            off, sz, sp = self.slices[name]
            chain = sp.dvalue_dvar().reshape(-1)
            if sz == 1 and B > 1:
                self.grad[off:off + 1] = torch.sum(g) * chain
            else:
                self.grad[off:off + sz] = g.reshape(-1) * chain
        call("vgposp_adam_update", ctypes.c_void_p(self.theta.data_ptr()),
             ctypes.c_void_p(self.grad.data_ptr()), ctypes.c_void_p(self.m.data_ptr()),
             ctypes.c_void_p(self.v.data_ptr()), self.theta.numel(), self.opt.lr, self.opt.beta1,
             self.opt.beta2, self.opt.epsilon, ctypes.c_void_p(self.step_count.data_ptr()), -1.0,
             linalg._stream())
        return lml if self.gp.batch_shape != () else lml[0]

    def variables(self):
        return {name: sp for name, (_, _, sp) in self.slices.items()}


class Saver:
    """tf.train.Saver stand-in (gp_functions.py:257-258): saves trainable variables as .npz."""

    def __init__(self, var_dict=None):
        self.var_dict = dict(var_dict or {})

    def add(self, name, var):
        self.var_dict[name] = var

    def save(self, sess, save_path, global_step=None):
        import os

        import numpy as np
        path = f"{save_path}-{global_step}" if global_step is not None else save_path
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        arrays = {k: (v.var.numpy() if isinstance(v, Softplus) else
                      v.numpy() if hasattr(v, "numpy") else np.asarray(v))
                  for k, v in self.var_dict.items()}
        np.savez(path + ".npz", **arrays)
        return path

    def restore(self, sess, save_path):
        import numpy as np
        z = np.load(save_path if save_path.endswith(".npz") else save_path + ".npz")
        for k, v in self.var_dict.items():
            if k in z.files:
                (v.var if isinstance(v, Softplus) else v).assign(z[k])

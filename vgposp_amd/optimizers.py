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

from . import _lib, linalg
from ._lib import call
from .variables import Softplus, Variable, resolve


class AdamOptimizer:
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8,
                 name="Adam"):
        self.lr = float(learning_rate)
        self.beta1 = float(beta1)
        self.beta2 = float(beta2)
        self.epsilon = float(epsilon)
        self.name = name

    def minimize(self, loss, var_list=None, group=None, precision="fp64", **options):
        """``loss``: ``-log_prob`` of a GaussianProcess (a ``Negated`` LogProb, see ``negate``;
        gp_functions.tf_train_gp_adam) -> ``GPTrainOp``, or a VGP ``variational_loss``
        (variational_Gaussian_process_example.py:95-102) -> ``VGPTrainOp``.  ``group``: a
        torch.distributed group over which the VGP's observations are sharded.  ``precision``
        (VGP only): "mixed" factors the M x M matrices in fp32 with fp64 refinement (config C5).
        ``options`` (VGP only): the ``VGPTrainOp`` scheduling switches (graph, streams,
        fused_params, grouped)."""
        from .distributions import VariationalLoss
        if isinstance(loss, Negated):
            if options:
                raise TypeError(f"unexpected options for a GP train op: {sorted(options)}")
            return GPTrainOp(loss.log_prob, self, var_list)
        if isinstance(loss, VariationalLoss):
            return VGPTrainOp(loss, self, var_list, group, precision=precision, **options)
        raise TypeError("minimize() expects -log_prob (a Negated LogProb) or a VGP "
                        "variational_loss")


class Negated:
    def __init__(self, log_prob):
        self.log_prob = log_prob


def negate(log_prob):
    return Negated(log_prob)


class GPTrainOp:
    """One TF1-Adam step on -sum_b LML_b of an exact GaussianProcess; ``run()`` returns the
    pre-update LML [B] (device tensor), as sess.run([train_op, log_likelihood]) does."""

    def __init__(self, log_prob, opt, var_list=None):
        self.loss = log_prob
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


def _adam(theta, grad, m, v, step_count, opt, grad_scale):
    call("vgposp_adam_update", ctypes.c_void_p(theta.data_ptr()), ctypes.c_void_p(grad.data_ptr()),
         ctypes.c_void_p(m.data_ptr()), ctypes.c_void_p(v.data_ptr()), theta.numel(), opt.lr,
         opt.beta1, opt.beta2, opt.epsilon, ctypes.c_void_p(step_count.data_ptr()), grad_scale,
         linalg._stream())


class VGPTrainOp:
    """One TF1-Adam step on a VGP's variational_loss whose q(u) is optimal_variational_posterior
    (the reference's training graph, variational_Gaussian_process_example.py:51-102).  Trainables:
    the kernel's softplus amplitude / length_scale, the softplus observation noise variance and
    the inducing_index_points Variable, re-bound into one flat device buffer updated by the HIP
    Adam kernel.  ``run(feed)`` returns the pre-update loss (device scalar).  Call ``check()``
    after the last ``run`` of a training loop: a replayed step's factorization statuses are read
    behind the next step, so the last step's are checked only there.

    From the second run on, the whole step (posterior, ELBO, reverse pass, Adam: ~400 launches)
    is captured once into a HIP graph and replayed, with the feeds copied into static buffers —
    the same fixed graph a TF1 session runs.  A replayed step's Cholesky statuses are checked
    when the next step has been issued (or by ``check()``), so a non-PD factorization raises
    CholeskyError one ``run`` late.  With a data-parallel ``group`` the step is captured as
    three graph segments replayed around its two all-reduces.  Eager when ``graph=False`` or
    while the library's event timing is on.

    Scheduling switches (each measured, defaults = the faster setting): ``streams`` the VGP
    step's side-stream bitmask (``VGPObjective``), ``fused_params`` the softplus values in one
    launch and their chain rule inside the Adam launch, ``grouped`` one launch per dependency
    level of M x M products."""

    def __init__(self, loss, opt, var_list=None, group=None, graph=True, precision="fp64",
                 streams=None, fused_params=True, grouped=True):
        from .vgp_training import VGPObjective
        vgp = loss.vgp
        spec = getattr(vgp.variational_loc, "_vgposp_posterior", None)
        if spec is None:
            raise NotImplementedError(
                "VGP training is supported for q(u) = optimal_variational_posterior (the "
                "reference's graph); free variational loc / scale variables are not")
        kernel = vgp.kernel
        if spec["kernel"] is not kernel or kernel.batch_size != 1:
            raise NotImplementedError("VGP training needs one (non-batched) kernel shared by the "
                                      "posterior and the VGP")
        if spec["mean_fn"] is not None or vgp.mean_fn is not None:
            raise NotImplementedError("VGP training supports the zero mean function only")
        Z = vgp.inducing_index_points
        if spec["inducing_index_points"] is not Z:
            raise ValueError("the posterior and the VGP must share inducing_index_points")
        self.loss, self.vgp, self.opt = loss, vgp, opt
        self.params = {"amp": kernel.amplitude, "ls": kernel.length_scale,
                       "noise": vgp.observation_noise_variance}
        if spec["observation_noise_variance"] is not self.params["noise"]:
            raise ValueError("the posterior and the VGP must share observation_noise_variance")

        def chosen(var):
            return var.trainable and (var_list is None or var in var_list)
        self.trainable = [(k, p) for k, p in self.params.items()
                          if isinstance(p, Softplus) and chosen(p.var)]
        self.train_Z = isinstance(Z, Variable) and chosen(Z)
        self.Z = Z
        n = len(self.trainable) + (Z.value.numel() if self.train_Z else 0)
        dev = linalg.device()
        self.theta = torch.zeros(max(n, 1), dtype=torch.float64, device=dev)
        self.grad = torch.zeros_like(self.theta)
        self.m = torch.zeros_like(self.theta)
        self.v = torch.zeros_like(self.theta)
        self.step_count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.slot = {}
        for i, (k, p) in enumerate(self.trainable):
            p.var._rebind(self.theta[i:i + 1])
            self.slot[k] = i
        self.z_off = len(self.trainable)
        if self.train_Z:
            Z._rebind(self.theta[self.z_off:])
        self.objective = VGPObjective(kernel.kind, spec["observation_index_points"],
                                      spec["observations"], jitter=vgp.jitter,
                                      posterior_jitter=spec["jitter"],
                                      trace_adjoint=vgp.trace_adjoint, group=group,
                                      precision=precision, streams=streams, grouped=grouped)
        self.fused = bool(fused_params)
        # data parallel: the step is captured as graph segments between its two all-reduces
        self.graph = bool(graph)
        self._runs = 0
        self._g = None  # (graph, feed shapes, static X, static y, loss, statuses)
        self._hstat = None    # two pinned host buffers for the replayed steps' statuses
        self._pending = None  # (event, buffer) of the last replayed step, not yet checked
        self._pv = None       # the three softplus parameter values (one launch per step)

    def _value(self, p):
        return resolve(p).reshape(())

    def _step(self, Xb, yb, infos=None):
        Zv = self.Z.value if isinstance(self.Z, Variable) else linalg.as_device(self.Z)
        names = ("amp", "ls", "noise")
        fused = self.fused
        if fused and all(k in self.slot for k in names):
            # all three are trainable softplus parameters in theta: their values in one launch,
            # their softplus chain rule inside the Adam launch
            if self._pv is None:
                self._pv = torch.empty(3, dtype=torch.float64, device=self.theta.device)
            slots = (ctypes.c_int * 3)(*[self.slot[k] for k in names])
            call("vgposp_softplus_values", ctypes.c_void_p(self.theta.data_ptr()),
                 self.theta.numel(), 3, slots,
                 (ctypes.c_double * 3)(*[float(self.params[k].offset) for k in names]),
                 ctypes.c_void_p(self._pv.data_ptr()), linalg._stream())
            vals = [self._pv[i] for i in range(3)]
        else:
            vals = [self._value(self.params[k]) for k in names]
        zbar = self.grad[self.z_off:].view_as(Zv) if self.train_Z else None
        loss, ga, gl, gn, gZ = self.objective.loss_and_grads(
            Zv, *vals, Xb, yb, self.loss.kl_weight, infos=infos, zbar_out=zbar)
        chain = [(self.slot[k], g) for k, g in zip(names, (ga, gl, gn)) if k in self.slot]
        if not fused:  # the chain rule as elementwise launches (A/B reference)
            for i, g in chain:
                k = names[[self.slot.get(n) for n in names].index(i)]
                self.grad[i:i + 1] = g * self.params[k].dvalue_dvar().reshape(-1)
            chain = []
        if self.train_Z and gZ is not zbar:
            self.grad[self.z_off:] = gZ.reshape(-1)
        call("vgposp_adam_update_softplus", ctypes.c_void_p(self.theta.data_ptr()),
             ctypes.c_void_p(self.grad.data_ptr()), ctypes.c_void_p(self.m.data_ptr()),
             ctypes.c_void_p(self.v.data_ptr()), self.theta.numel(), self.opt.lr, self.opt.beta1,
             self.opt.beta2, self.opt.epsilon, ctypes.c_void_p(self.step_count.data_ptr()), 1.0,
             len(chain), (ctypes.c_int * 4)(*[i for i, _ in chain]),
             (ctypes.c_void_p * 4)(*[g.data_ptr() for _, g in chain]), linalg._stream())
        return loss

    def _capture(self, sX, sy):
        """Capture the step into HIP graph segments: ONE graph on a single GPU; with a
        data-parallel group a new segment starts at each of the step's two all-reduces (the
        [P0, c] partials, the Kzx VJP's), which run between the segment replays — RCCL on the
        current stream without a host synchronisation, gloo through the host.  The segments share
        one memory pool and are replayed in capture order.  -> (segments [(graph, tensor to
        all-reduce after it or None)], loss, status)."""
        obj = self.objective
        pool = torch.cuda.graph_pool_handle()
        segs, infos = [], []
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        cur = [torch.cuda.CUDAGraph()]

        def boundary(t):
            obj.join_side_streams()
            cur[0].capture_end()
            segs.append((cur[0], t))
            cur[0] = torch.cuda.CUDAGraph()
            cur[0].capture_begin(pool=pool)
            return t

        with torch.cuda.stream(cap):
            cur[0].capture_begin(pool=pool)
            obj._capture_hook = boundary if obj.group is not None else None
            try:
                loss = self._step(sX, sy, infos)
                status = torch.cat(infos)
                obj.join_side_streams()
            finally:
                obj._capture_hook = None
            cur[0].capture_end()
            segs.append((cur[0], None))
        torch.cuda.current_stream().wait_stream(cap)
        return segs, loss, status

    def _replay(self, Xb, yb):
        key = (tuple(Xb.shape), tuple(yb.shape))
        if self._g is None or self._g[1] != key:
            sX, sy = Xb.clone(), yb.clone()
            segs, loss, status = self._capture(sX, sy)
            self._g = (segs, key, sX, sy, loss, status)
        segs, _, sX, sy, loss, status = self._g
        sX.copy_(Xb)
        sy.copy_(yb)
        for g, t in segs:
            g.replay()
            if t is not None:
                self.objective.allreduce_now(t)
        out = loss.clone()
        # The step's Cholesky statuses go to pinned host memory behind the replay and are checked
        # when the NEXT step has been issued (or by check()): waiting then costs nothing, the GPU
        # already holds that step, so the host never drains the queue between steps.  The
        # captured step holds only kernel nodes (the library's fills / 2-D copies are kernels,
        # common.h vg_memset / vg_memcpy2d), which removed the stale-status reads round 2 saw
        # when memset / memcpy nodes were replayed back to back.
        if self._hstat is None or self._hstat[0].numel() != status.numel():
            self._hstat = [torch.empty(status.numel(), dtype=status.dtype, pin_memory=True)
                           for _ in range(2)]
        buf = self._hstat[self._runs & 1]
        prev = self._pending
        if prev is not None and prev[1] is buf:
            self.check()
            prev = None
        buf.copy_(status, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._pending = (ev, buf)
        if prev is not None:
            prev[0].synchronize()
            linalg.check_info(prev[1])
        return out

    def check(self):
        """Check the statuses of the last replayed step (its factorizations were PD); ``run``
        checks each step's when the next one has been issued."""
        if self._pending is not None:
            ev, buf = self._pending
            self._pending = None
            ev.synchronize()
            linalg.check_info(buf)

    def run(self, feed=None):
        yb, Xb = self.loss.inputs(feed)
        if Xb is None:
            Xb = self.vgp.index_points
        Xb = linalg.as_device(Xb)
        Xb = Xb[:, None] if Xb.dim() == 1 else Xb
        yb = linalg.as_device(yb).reshape(-1)
        if self.graph and self._runs > 0 and not _lib.prof_on():
            loss = self._replay(Xb, yb)
        else:
            self.check()
            loss = self._step(Xb, yb)
        self._runs += 1
        self.loss.value = loss
        return loss


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

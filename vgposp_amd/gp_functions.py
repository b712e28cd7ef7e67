"""Drop-in counterpart of the reference's ``gp_functions`` hot-path functions
(``/root/reference/gp_functions.py``), eager and GPU-backed.

Same names, argument order and meaning; TF1-only plumbing arguments (``sess``, ``summ``,
``writer``, placeholders) are accepted and handled by a small eager ``Session`` so the reference's
call sequences (main_GP_fit.py:191-267, main_tests.py:598-750, main.py:68-123) run unchanged in
shape:

  sess = reset_session()
  amp, amp_assign, amp_p, lensc, lensc_assign, lensc_p, emb, emb_assign, emb_p, noise = \\
      tf_Placeholder_assign_test(AMPLITUDE_INIT, LENGTHSCALE_INIT, INIT_OBSNOISEVAR)
  kernel = create_cov_kernel(amp, lensc)
  gp = fit_gp(kernel, obs_idx_pts, noise)
  log_likelihood = gp.log_prob(obs)
  train_op = tf_train_gp_adam(log_likelihood, LEARNING_RATE)
  summ, writer, saver = tf_summary_writer_saver(sess, LOGDIR)
  lls = tf_optimize_model_params(sess, NUM_ITERS, train_op, log_likelihood, summ, writer, saver,
                                 LOGDIR, LOGCHECKPT, obs, None)
  gprm = tf_gp_regression_model(kernel, pred_idx_pts, obs_idx_pts, obs, noise, 0.)
  samples = sess.run(gprm.sample(NUM_SAMPLES))
  H = calc_H(XEDGES, YEDGES, lensc, lensc_assign, lensc_p, amp, amp_assign, amp_p,
             log_likelihood, sess, None, obs)

Reference functions outside the hot path (VAE, section-cut geometry, CFD covariance builders,
the buggy legacy greedy at gp_functions.py:576-701) are intentionally absent; see DESIGN.md.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import linalg
from .data_generation import sinusoid  # noqa: F401  (gp_functions.py:78-95)
from .distributions import (GaussianProcess, GaussianProcessRegressionModel, LogProb,
                            VariationalLoss)
from .optimizers import AdamOptimizer, GPTrainOp, Saver, VGPTrainOp, negate
from .psd_kernels import MaternOneHalf
from .variables import TINY, Placeholder, Softplus, Variable, placeholder  # noqa: F401

TEST_FN_PARAM = 1


def sinusoid_(x, scale=TEST_FN_PARAM):
    """gp_functions.py:98-103."""
    a = np.dot(x, scale)
    return np.sin(a)


# ---------------------------------------------------------------------------------------------
# Eager session / placeholder shim
# ---------------------------------------------------------------------------------------------
class AssignOp:
    """The eager form of ``invert_softplus(placeholder, variable)`` (gp_functions.py:106-109)."""

    def __init__(self, view, placeholder):
        self.view = view
        self.placeholder = placeholder

    def __call__(self, value):
        return self.view.assign_inverse_softplus(value)


class Session:
    """Minimal ``tf.Session``: ``run(fetches, feed_dict)`` evaluates this package's objects."""

    def run(self, fetches, feed_dict=None):
        feed = feed_dict or {}
        if isinstance(fetches, (list, tuple)):
            # assignments first (TF runs them before reads that depend on them); a train op's
            # loss fetched in the same run is the value the step was computed from (pre-update),
            # as in a TF graph where the loss tensor feeds both the fetch and the gradients
            for f in fetches:
                if isinstance(f, AssignOp):
                    self._eval(f, feed)
            memo = {}
            for f in fetches:
                if isinstance(f, (GPTrainOp, VGPTrainOp)):
                    memo[id(f)] = self._eval(f, feed)
                    src = getattr(f, "loss", None)
                    if src is not None:
                        memo[id(src)] = memo[id(f)]
            return [memo[id(f)] if id(f) in memo else self._eval(f, feed, assigned=True)
                    for f in fetches]
        return self._eval(fetches, feed)

    def _eval(self, f, feed, assigned=False):
        if isinstance(f, AssignOp):
            if assigned:
                return f.view.numpy()
            if f.placeholder not in feed:
                raise KeyError("feed_dict lacks the assign placeholder")
            return f(feed[f.placeholder])
        if isinstance(f, GPTrainOp):
            obs = _feed_obs(feed)
            return f.run(obs).detach().cpu().numpy()
        if isinstance(f, VGPTrainOp):
            return f.run(feed).detach().cpu().numpy()
        if isinstance(f, VariationalLoss):
            return f.evaluate(feed).detach().cpu().numpy()
        if isinstance(f, LogProb):
            obs = _feed_obs(feed)
            if obs is None:
                obs = f.observations
            return f.dist.log_prob(obs).numpy()
        if isinstance(f, (Softplus, Variable)):
            return f.numpy()
        if isinstance(f, torch.Tensor):
            return f.detach().cpu().numpy()
        if f is None:
            return None
        return f

    def close(self):
        pass


def _feed_obs(feed):
    for k, v in feed.items():
        if isinstance(k, Placeholder) and k.name in ("input_values", "obs_values", None):
            return v
    return None


_SESSION = None


def reset_session():
    """gp_functions.py:112-121 (an eager session; nothing to reset)."""
    global _SESSION
    _SESSION = Session()
    return _SESSION


# ---------------------------------------------------------------------------------------------
# Variables (gp_functions.py:48-65, 106-109, 124-157)
# ---------------------------------------------------------------------------------------------
def invert_softplus(place_holder, variable, name="assign_op"):
    """Returns an AssignOp; calling it (or sess.run with a feed) sets var = log(exp(x) - 1)."""
    view = variable if isinstance(variable, Softplus) else Softplus(variable)
    return AssignOp(view, place_holder)


def tf_Variable(FEATURE_s, FEATURE_n, INIT):
    """-> (feature_var, feature) with feature = tiny + softplus(feature_var)."""
    var = Variable(np.asarray(INIT, dtype=np.float64), name=FEATURE_n)
    return var, Softplus(var, TINY)


def tf_Placeholder_assignments(feature_var, FEATUREPLH_s, FEATUREPLH_n, INIT):
    plh = Placeholder(np.shape(INIT), FEATUREPLH_n)
    return plh, invert_softplus(plh, feature_var)


def tf_Placeholder_assign_test(AMPLITUDE_INIT, LENGTHSCALE_INIT, INIT_OBSNOISEVAR):
    AMPLITUDE_INIT = np.asarray(AMPLITUDE_INIT, dtype=np.float64)
    LENGTHSCALE_INIT = np.asarray(LENGTHSCALE_INIT, dtype=np.float64)
    amp_var, amp = tf_Variable("amplitude", "amplitude", AMPLITUDE_INIT)
    amp_plh = Placeholder(AMPLITUDE_INIT.shape, "amplitude_assign")
    amp_assign = AssignOp(amp, amp_plh)
    lensc_var, lensc = tf_Variable("lengthscale", "lengthscale", LENGTHSCALE_INIT)
    lensc_plh = Placeholder(LENGTHSCALE_INIT.shape, "lengthscale_assign")
    lensc_assign = AssignOp(lensc, lensc_plh)
    _, obs_noise_var = tf_Variable("observation_noise_variance", "observation_noise_variance",
                                   INIT_OBSNOISEVAR)
    emb_var, emb = tf_Variable("log_probability_embedding", "log_probability_embedding",
                               LENGTHSCALE_INIT)
    emb_plh = Placeholder(LENGTHSCALE_INIT.shape, "log_probability_embedding_assign")
    emb_assign = AssignOp(emb, emb_plh)
    assert amp.shape == AMPLITUDE_INIT.shape
    assert lensc.shape == LENGTHSCALE_INIT.shape
    return (amp, amp_assign, amp_plh, lensc, lensc_assign, lensc_plh, emb, emb_assign, emb_plh,
            obs_noise_var)


def do_assign(sess, feature, feature_assign, feature_plh, feature_arr):
    """gp_functions.py:222-225 -> the assigned (constrained) value."""
    return feature_assign(feature_arr)


# ---------------------------------------------------------------------------------------------
# GP model, training, prediction (gp_functions.py:160-297)
# ---------------------------------------------------------------------------------------------
def create_cov_kernel(amp, lensc):
    """gp_functions.py:160-163: MaternOneHalf(amp, lensc)."""
    return MaternOneHalf(amp, lensc)


def fit_gp(kernel, obs_idx_pts, obs_noise_var):
    """gp_functions.py:166-172."""
    return GaussianProcess(kernel=kernel, index_points=obs_idx_pts,
                           observation_noise_variance=obs_noise_var, validate_args=True)


def tf_train_gp_adam(feature, LEARNING_RATE):
    """gp_functions.py:179-182: AdamOptimizer(lr).minimize(-feature)."""
    return AdamOptimizer(learning_rate=LEARNING_RATE).minimize(negate(feature))


def tf_summary_writer_saver(sess, LOGDIR):
    """gp_functions.py:211-218 -> (summ, writer, saver); summaries are not recorded."""
    return None, None, Saver()


tf_summary_writer_projector_saver = tf_summary_writer_saver


def tf_optimize_model_params(sess, num_iters, train_op, log_likelihood=None, summ=None,
                             writer=None, saver=None, LOGDIR=None, LOGCHECKPT=None,
                             obs_train_dataset=None, obs_value_placeholder=None):
    """gp_functions.py:228-259: one warm-up step, then num_iters+1 steps; lls[i] is the LML before
    update i; checkpoint every 200 steps.  Returns lls [num_iters + 1, B] (numpy)."""
    if not isinstance(train_op, GPTrainOp):
        raise TypeError("train_op must come from tf_train_gp_adam")
    obs = obs_train_dataset
    if saver is not None and not saver.var_dict:
        for name, sp in train_op.variables().items():
            saver.add(name, sp)
    train_op.run(obs)  # the initial run (gp_functions.py:248-250)
    B = max(train_op.gp.kernel.batch_size, 1)
    lls = torch.empty((num_iters + 1, B), dtype=torch.float64, device=train_op.theta.device)
    for i in range(num_iters + 1):
        lls[i] = train_op.run(obs).reshape(-1)
        if saver is not None and LOGDIR is not None and i % 200 == 0:
            saver.save(sess, os.path.join(LOGDIR, LOGCHECKPT or "model.ckpt"), i)
    return lls.cpu().numpy()


def create_meshgrid(pred_x, pred_y):
    """gp_functions.py:262-280 -> [len(pred_y) * len(pred_x), 2] prediction points."""
    h = np.array(np.meshgrid(pred_x, pred_y, sparse=False))
    return h.swapaxes(0, -1).reshape(-1, 2)


def tf_gp_regression_model(kernel, pred_idx_pts, obs_idx_pts, obs, obs_noise_var, pred_noise_var):
    """gp_functions.py:283-297."""
    return GaussianProcessRegressionModel(
        kernel=kernel, index_points=np.asarray(pred_idx_pts, dtype=np.float64),
        observation_index_points=np.asarray(obs_idx_pts, dtype=np.float64),
        observations=np.asarray(obs, dtype=np.float64).reshape(-1),
        observation_noise_variance=obs_noise_var, predictive_noise_variance=pred_noise_var)


# ---------------------------------------------------------------------------------------------
# Log-marginal-likelihood surface (gp_functions.py:864-889), batched on the GPU
# ---------------------------------------------------------------------------------------------
def lml_surface(kind, X, y, ls_values, amp_values, noise, jitter=1e-6):
    """LML for every (ls_i, amp_j) pair in ONE batched evaluation -> [len(ls), len(amp)]."""
    ls_values = np.asarray(ls_values, dtype=np.float64)
    amp_values = np.asarray(amp_values, dtype=np.float64)
    LS, AMP = np.meshgrid(ls_values, amp_values, indexing="ij")
    from .psd_kernels import PositiveSemidefiniteKernel
    k = PositiveSemidefiniteKernel(AMP.reshape(-1), LS.reshape(-1))
    k.kind = kind
    gp = GaussianProcess(k, np.asarray(X, dtype=np.float64), observation_noise_variance=noise,
                         jitter=jitter)
    return gp.log_prob(y).numpy().reshape(LS.shape)


def calc_H(XEDGES, YEDGES, lensc, lensc_assign, lensc_p, amp, amp_assign, amp_p, log_likelihood,
           sess, obs_values_placeholder=None, obs_train_dataset=None):
    """gp_functions.py:864-876: H[i, j] = LML[0] at ls = 40 (1+i)/XEDGES, amp = 40 (1+j)/YEDGES.
    All XEDGES*YEDGES likelihoods are one batched GPU evaluation; like the reference, the
    variables are left at the last assigned pair."""
    gp = log_likelihood.dist
    obs = log_likelihood.observations if obs_train_dataset is None else obs_train_dataset
    ls_vals = 40 * np.double((1 + np.arange(XEDGES)) / XEDGES)
    amp_vals = 40 * np.double((1 + np.arange(YEDGES)) / YEDGES)
    noise = gp._noise()[0:1]
    H = lml_surface(gp.kernel.kind, gp.index_points, obs, ls_vals, amp_vals, noise, gp.jitter)
    shape_l = lensc.shape if hasattr(lensc, "shape") else ()
    shape_a = amp.shape if hasattr(amp, "shape") else ()
    lensc_assign(np.full(shape_l, ls_vals[-1]))
    amp_assign(np.full(shape_a, amp_vals[-1]))
    return H


def calc_H_1d(XEDGES, YEDGES, lensc, lensc_assign, lensc_p, amp, amp_assign, amp_p,
              log_likelihood, sess):
    """gp_functions.py:879-889: the same surface on (2 (1+i)/XEDGES, 2 (1+j)/YEDGES)."""
    gp = log_likelihood.dist
    ls_vals = 2 * np.double((1 + np.arange(XEDGES)) / XEDGES)
    amp_vals = 2 * np.double((1 + np.arange(YEDGES)) / YEDGES)
    noise = gp._noise()[0:1]
    return lml_surface(gp.kernel.kind, gp.index_points, log_likelihood.observations, ls_vals,
                       amp_vals, noise, gp.jitter)


# ---------------------------------------------------------------------------------------------
# Index -> coordinate helpers (gp_functions.py:1226-1248)
# ---------------------------------------------------------------------------------------------
def py_get_coord_idxs(sel_idx, xyz_idxs):
    """Rows of xyz_idxs for the selected flat indices (the reference hard-codes 7 sensors)."""
    sel_idx = [int(i) for i in sel_idx]
    return np.vstack([np.reshape(np.asarray(xyz_idxs)[i, :], [1, 3]) for i in sel_idx])


def denormalize_coord(sel_norm_coord):
    """gp_functions.py:1239-1248 (constants of the reference's normalisation)."""
    stdev_var = 0.0007434639347162126 * 3000000
    mean_var = 0.0018159087825037148
    return np.asarray(sel_norm_coord, dtype=np.float64) * stdev_var + mean_var

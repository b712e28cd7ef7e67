"""Generate golden placement vectors by running the REFERENCE's own numpy greedy.

Run in the build container only (``/root/reference`` is absent on the GPU box):

    python tests/golden/make_golden.py

It imports ``/root/reference/placement_algorithm2.py`` with inert stand-ins for the modules the
file imports but this path never calls (tensorflow, tensorflow_probability, tensorboard, seaborn:
absent from the image), captures the reference's per-evaluation prints (``:188``, ``:205``) by
injecting a ``print`` into the module namespace, and writes small fixtures:

    tests/golden/placement_<case>.npz   inputs (cov_vv, or grid points + kernel params)
    tests/golden/placement_golden.json  expected indices (Alg. 1 / Alg. 2) + delta trace

Only data is committed (inputs and outputs); no reference source is copied.
"""
from __future__ import annotations

import json
import os
import sys
import types
from unittest import mock

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import gp as ogp  # noqa: E402
from vgposp_amd.data_generation import grid_points, grid_spacing  # noqa: E402


class _Stub(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        m = mock.MagicMock(name=f"{self.__name__}.{name}")
        setattr(self, name, m)
        return m


def _import_reference():
    for name in ["tensorflow", "tensorflow.compat", "tensorflow.compat.v1",
                 "tensorflow_probability", "tensorboard", "tensorboard.plugins",
                 "tensorboard.plugins.projector", "seaborn"]:
        sys.modules[name] = _Stub(name)
    sys.modules["tensorflow"].__version__ = "1.15.0"
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, "/root/reference")
    import placement_algorithm2 as alg2  # the reference module
    return alg2


def grid_cov(shape, kind="eq", jitter=0.05, seed=0, amp=1.0, ls_h=2.0, noise=1e-2, gp_jitter=1e-6):
    X = grid_points(shape, jitter=jitter, seed=seed)
    ls = ls_h * grid_spacing(shape)
    K = ogp.kernel_matrix(kind, X, X, amp, ls)[0] + (noise + gp_jitter) * np.eye(X.shape[0])
    return X, K, dict(shape=list(shape), kind=kind, jitter=jitter, seed=seed, amp=amp, ls=ls,
                      noise=noise, gp_jitter=gp_jitter)


def main():
    alg2 = _import_reference()
    trace = []

    def capture(*args, **kw):
        if len(args) >= 4 and args[0] == "delta_y=":
            trace.append([int(args[3]), float(np.asarray(args[1]).reshape(-1)[0])])
        elif len(args) >= 2 and args[0] == "y*=":
            trace.append(["select", int(args[1])])

    alg2.print = capture

    cases = {}
    # 1. the reference's own fixture (placement_algorithm2.py:473-479)
    cases["cov4x4"] = dict(cov=alg2.cov_vv_4x4(), k=4, alg1=True, params={"source": "cov_vv_4x4"})
    # 2. random covariance as in dg_create_random_cov (placement_algorithm2.py:441-444)
    rng = np.random.default_rng(11)
    m = rng.uniform(0, 1, 11 ** 2).reshape(-1, 11)
    cases["randcov11"] = dict(cov=m @ m.T, k=5, alg1=True, params={"source": "UU^T, U~U(0,1), rng 11"})
    # 3. SPD as in snippets_save.test_save_cov_vv (snippets_save.py:36-39)
    for n, k, seed in [(11, 5, 7), (40, 8, 8)]:
        rng = np.random.default_rng(seed)
        U = rng.normal(1, 1, size=(n, n))
        cases[f"spd{n}"] = dict(cov=U @ U.T + 0.001 * np.eye(n), k=k, alg1=True,
                                params={"source": f"UU^T+1e-3 I, U~N(1,1), rng {seed}"})
    # 4. jittered sensor grids, EQ / Matern kernels, noise 1e-2 + jitter 1e-6
    for name, shape, kind, k, alg1 in [("grid4", (4, 4, 4), "eq", 8, True),
                                       ("grid5", (5, 5, 5), "eq", 8, False),
                                       ("grid654", (6, 5, 4), "eq", 6, False),
                                       ("grid5m12", (5, 5, 5), "matern12", 6, False),
                                       ("grid5m52", (5, 5, 5), "matern52", 6, False),
                                       ("grid8", (8, 8, 8), "eq", 5, False)]:
        X, K, p = grid_cov(shape, kind)
        cases[name] = dict(cov=K, X=X, k=k, alg1=alg1, params=p)

    golden = {}
    for name, c in cases.items():
        cov = np.asarray(c["cov"], dtype=np.float64)
        trace.clear()
        A2 = [int(a) for a in alg2.placement_algorithm_2(cov, c["k"])]
        entry = dict(k=c["k"], N=int(cov.shape[0]), alg2=A2, trace=list(trace), params=c["params"])
        if c["alg1"]:
            entry["alg1"] = [int(a) for a in alg2.placement_algorithm_1(cov, c["k"])]
        golden[name] = entry
        arrays = {"cov": cov} if cov.shape[0] <= 216 else {}
        if "X" in c:
            arrays["X"] = c["X"]
        np.savez_compressed(os.path.join(HERE, f"placement_{name}.npz"), **arrays)
        print(name, "alg2", A2, "alg1", entry.get("alg1"), "evals", sum(1 for t in trace if t[0] != "select"),
              flush=True)
    with open(os.path.join(HERE, "placement_golden.json"), "w") as f:
        json.dump(golden, f, indent=1)


if __name__ == "__main__":
    main()

"""Golden vectors for the GP regression model from the REFERENCE itself.

Run in the build container only (``/root/reference`` is absent on the GPU box):

    python tests/golden/make_golden_gprm.py

``plot_confidence_interval.py`` is the reference's one pure-numpy GP posterior: 5 noiseless
training points Xtrain = [-4, -3, -2, -1, 1], ytrain = sin(Xtrain), the kernel
``exp(-0.5 * sqdist / 0.3)`` (EQ, amplitude 1, length scale sqrt(0.3)), K + 5e-5 I, and at 700 test
points in [-15, 15] the posterior mean ``mu`` and variance ``s2 = diag(K_ss) - sum(Lk**2)``
(plot_confidence_interval.py:38-51).  This script executes that file as it lies (matplotlib on the
Agg backend, ``pyplot.show`` a no-op, numpy's global RNG seeded — the draws only feed the plotted
samples, never ``mu`` / ``s2``) and records the module's own ``Xtrain``, ``ytrain``, ``Xtest``,
``mu`` and ``s2`` in ``tests/golden/gprm_confidence.npz``.  Only data is committed.

The first of the file's three ``np.linalg.cholesky`` calls, the prior factor of K_ss + 1e-15 I at
:26 (700 points 0.04 apart at length scale 0.55), is not numerically positive definite with this
numpy/LAPACK and raises; it only feeds the plotted prior samples.  ``np.linalg.cholesky`` is therefore wrapped for the run: a call that raises
``LinAlgError`` is retried with a diagonal jitter growing from 1e-12 × mean diag, and the
number of such retries is printed.  The call that matters, chol(K + 5e-5 I) at :43, must
succeed unmodified — the script asserts it.
"""
from __future__ import annotations

import os
import runpy

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/plot_confidence_interval.py"


def main():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as pl
    pl.show = lambda *a, **kw: None
    np.random.seed(0)
    chol = np.linalg.cholesky
    calls = []

    def cholesky(a, *args, **kw):
        try:
            L = chol(a, *args, **kw)
            calls.append((a.shape[0], 0.0))
            return L
        except np.linalg.LinAlgError:
            eps = 1e-12 * float(np.mean(np.diag(a)))
            while True:
                try:
                    L = chol(a + eps * np.eye(a.shape[0]), *args, **kw)
                    calls.append((a.shape[0], eps))
                    return L
                except np.linalg.LinAlgError:
                    eps *= 10.0

    np.linalg.cholesky = cholesky
    try:
        g = runpy.run_path(REF, run_name="reference_plot_confidence_interval")
    finally:
        np.linalg.cholesky = chol
        pl.close("all")
    # the training factor chol(K + 5e-5 I) (the only one mu / s2 depend on) ran unmodified
    assert [c for c in calls if c[0] == 5] == [(5, 0.0)], calls
    print("cholesky calls (size, added jitter):", calls)
    out = {k: np.asarray(g[k], dtype=np.float64) for k in ("Xtrain", "ytrain", "Xtest", "mu", "s2")}
    out["param"] = np.float64(g["param"])
    out["diag_shift"] = np.float64(5e-5)  # plot_confidence_interval.py:43
    np.savez_compressed(os.path.join(HERE, "gprm_confidence.npz"), **out)
    print("mu[:4]", out["mu"][:4], "s2 range", out["s2"].min(), out["s2"].max())


if __name__ == "__main__":
    main()

"""CPU oracle for the vgposp_amd hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline.  The product path
(``vgposp_amd``) never imports it and fails loudly when its HIP library is missing.

Contents
--------
``placement``  numpy restatement of ``placement_algorithm2.py`` (lazy greedy MI, Krause Alg. 2,
               and the full greedy Alg. 1), pinv-faithful: same ``np.linalg.pinv`` calls on the same
               slices, so it reproduces the reference bit for bit.  Pinned against golden vectors
               produced by running the reference's own ``placement_algorithm2.py`` in the build
               container (``tests/golden/make_golden.py``).
               Also a Cholesky/precision restatement (same lazy policy) for sizes where pinv per
               candidate is too slow; it is pinned against the pinv restatement.
``gp``         numpy restatement of the TFP (~0.7) semantics the reference reaches through
               ``gp_functions.py``: PSD kernels, ``GaussianProcess.log_prob`` (jitter 1e-6 on top of
               the noise), its gradient, TF1 Adam, ``GaussianProcessRegressionModel`` and
               ``VariationalGaussianProcess``.  TF/TFP are absent from this container and no
               reference test pins numbers at that boundary, so these are **parity unpinned**
               except the exact-GP LML, which is cross-checked against scikit-learn.
"""

"""Oracle (TEST INFRASTRUCTURE ONLY): ctypes binding of oracle/c4_exact.c, the plain-C restatement
of config C4's exact algorithm 3 (snippets_a3.py:43-364 on the beta-decay tapered covariance,
main_architecture_2_sampledistribution.py:355-421) in the bounded-lazy form, for CPU checks of the
GPU picks at sizes the dense oracle (oracle.placement.placement_window_precision) cannot reach.

The restatement itself is pinned to the dense oracle on small grids (tests/test_c4_oracle.py), and
the dense oracle to the reference's golden vectors; at 128^3 it is the CPU side of "selected indices
bit-exact vs CPU".  Built by oracle/Makefile into oracle/_build/libc4oracle.so (build() in
__graft_entry__ runs it); imported only by tests/, smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import math
import os
import time

import numpy as np

from .taper import TF_JITTER, TF_SMALL, taper_support

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "libc4oracle.so")
KINDS = {"eq": 0, "matern12": 1, "matern32": 2, "matern52": 3}
_lib = None


def build():
    """make -C oracle (gcc -O3 -fopenmp)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, I32, F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_double
        L.c4o_coef.argtypes = [P, I64, I64, I64, I32, F, F, F, F, P, I32, P, I32, P, P]
        L.c4o_coef.restype = I32
        L.c4o_run.argtypes = [P, I64, I64, I64, I32, F, F, F, F, F, P, I32, P, I32, P, P, P, P, I32,
                              I32, F, I32, F, I32, I32, P, P, P]
        L.c4o_run.restype = I32
        L.c4o_threads.restype = I32
        L.c4o_set_threads.argtypes = [I32]
        L.c4o_set_threads.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def reach(offsets, K):
    """Offsets within K stencil steps, sorted by step count then C order (node itself first):
    (tab [T, 3], cnt [K + 1], nb [T, m-1] = row of tab[i] + off_o or -1)."""
    offs = [tuple(int(v) for v in o) for o in np.asarray(offsets).reshape(-1, 3)]
    dist, front = {(0, 0, 0): 0}, [(0, 0, 0)]
    for d in range(1, K + 1):
        nxt = []
        for v in front:
            for o in offs:
                w = (v[0] + o[0], v[1] + o[1], v[2] + o[2])
                if w not in dist:
                    dist[w] = d
                    nxt.append(w)
        front = nxt
    items = sorted(dist.items(), key=lambda kv: (kv[1], kv[0]))
    pos = {k: i for i, (k, _) in enumerate(items)}
    tab = np.array([k for k, _ in items], dtype=np.int32).reshape(-1, 3)
    cnt = np.array([sum(1 for _, s in items if s <= d) for d in range(K + 1)], dtype=np.int32)
    nb = np.array([[pos.get((k[0] + o[0], k[1] + o[1], k[2] + o[2]), -1) for o in offs]
                   for k, _ in items], dtype=np.int32).reshape(len(items), len(offs))
    return tab, cnt, nb


def steps_for(lam_min, lam_max, target=1e-6, kmax=8):
    """(K, hi_scale): the fewest CG steps whose bracket width 4 rho^2K is <= target (kmax at most);
    Q_yy <= g_K (1 + 1e-12) / (1 - 4 rho^2K)."""
    if not lam_min > 0.0:
        return None
    kappa = lam_max / lam_min
    rho = (math.sqrt(kappa) - 1.0) / (math.sqrt(kappa) + 1.0)
    for K in range(1, kmax + 1):
        w = 4.0 * rho ** (2 * K)
        if w < 0.5 and (w <= target or K == kmax):
            return K, (1.0 + 1e-12) / (1.0 - w)
    return None


def cg_iterations(lam_min, lam_max, tol):
    kappa = lam_max / lam_min
    rho = (math.sqrt(kappa) - 1) / (math.sqrt(kappa) + 1)
    if rho <= 0:
        return 1
    return int(min(400, math.ceil(math.log(tol / 2) / math.log(rho)) + 4))


def exact_alg3(X, shape, k, cutoff, beta=4.0, kind="eq", amp=1.0, ls=1.0, diag_shift=0.0,
               jitter=TF_JITTER, threshold=TF_SMALL, cg_tol=1e-16, K=None, stats=None,
               threads=None):
    """Algorithm 3 on the tapered covariance of the grid points X (C order) -> (picks [k] int64,
    pick deltas [k]).  ``K`` overrides the bracket's CG steps (any K gives the same picks);
    ``stats`` (dict) receives refinements, K, cg_iters, the Gershgorin bounds and seconds;
    ``threads``: the OpenMP team size (default: OMP_NUM_THREADS / the runtime's)."""
    I0, I1, I2 = (int(s) for s in shape)
    n = I0 * I1 * I2
    X = np.ascontiguousarray(X, dtype=np.float64).reshape(n, 3)
    offs, tau = taper_support(beta)
    offs = np.ascontiguousarray(offs, dtype=np.int32).reshape(-1, 3)
    tau = np.ascontiguousarray(tau, dtype=np.float64)
    m1 = len(offs)
    L = lib()
    if threads:
        L.c4o_set_threads(int(threads))
    t0 = time.perf_counter()
    coef = np.empty((n, m1 + 1))
    lam = np.zeros(2)
    L.c4o_coef(_ptr(X), I0, I1, I2, KINDS[kind], amp, ls, diag_shift, jitter, _ptr(offs), m1,
               _ptr(tau), len(tau), _ptr(coef), _ptr(lam))
    st = steps_for(lam[0], lam[1], kmax=K or 8)
    if st is None:
        raise ValueError("Sigma + eps I is not diagonally dominant: the CG bracket does not hold")
    Ks, scale = (K, st[1]) if K else st
    if K:
        kappa = lam[1] / lam[0]
        rho = (math.sqrt(kappa) - 1.0) / (math.sqrt(kappa) + 1.0)
        scale = (1.0 + 1e-12) / (1.0 - 4.0 * rho ** (2 * K))
    tab, cnt, nb = reach(offs, Ks)
    nbf = np.ascontiguousarray(nb if nb.size else np.full((len(tab), 1), -1, np.int32))
    its = cg_iterations(lam[0], lam[1], cg_tol)
    picks = np.full(k, -1, dtype=np.int64)
    deltas = np.zeros(k)
    sts = np.zeros(2, dtype=np.int64)
    rc = L.c4o_run(_ptr(X), I0, I1, I2, KINDS[kind], amp, ls, diag_shift, jitter, threshold,
                   _ptr(offs), m1, _ptr(tau), len(tau), _ptr(coef), _ptr(tab), _ptr(nbf), _ptr(cnt),
                   len(tab), Ks, scale, its, cg_tol, k, cutoff, _ptr(picks), _ptr(deltas),
                   _ptr(sts))
    if rc:
        raise RuntimeError(f"c4o_run failed ({rc}): out of column storage after {sts[0]} "
                           "refinements")
    if stats is not None:
        stats.update(refinements=int(sts[0]), rounds=int(sts[1]), K=Ks, cg_iters=its,
                     lam=(float(lam[0]), float(lam[1])), seconds=time.perf_counter() - t0,
                     threads=int(L.c4o_threads()))
    return picks, deltas

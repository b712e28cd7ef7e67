"""Golden vectors for placement algorithm 3 (config C4's semantics) from the REFERENCE's own arithmetic.

Run in the build container only (``/root/reference`` is absent on the GPU box):

    python tests/golden/make_golden_alg3.py [--jobs J] [case ...]

The reference's algorithm 3 (``snippets_a3.sparse_placement_algorithm_3``, snippets_a3.py:43-364)
is a TF1 graph and TF is absent here.  Its per-delta arithmetic is not TF-specific: with
``S = cov_vv + eps I`` (eps = 1e-6, snippets_a2.py:161-163)

    tf_nominator(y, A, cov_vv)     = placement_algorithm2.nominator(y, A \\ {y}, S) - eps
    tf_denominator(y, Abar, cov_vv) = placement_algorithm2.denominator(y, Abar, S) - eps

because the jitter is added to the diagonal of Sigma_AA only and y is never in the conditioning
set.  So this script imports the reference's ``placement_algorithm2`` (same inert module stubs as
make_golden.py) and drives ITS ``nominator`` / ``denominator`` (placement_algorithm2.py:371-413,
``make_slice`` / ``call_pinv`` included) and ITS ``argmax_cache_linear`` (:53-67, lowest index
wins ties) through the window loop of snippets_a3.py:

* round 0 scores every candidate against A = {} and Abar = V (:77-124);
* the threshold of ``if_denom_is_near_zero`` (snippets_a2.py:480): |nom| or |denom| < 1e-7 -> 0;
* each of the k - 1 rounds picks the cache arg-max over V \\ A (:143), zeroes its entry (:162-168),
  re-scores the index window [i - c, i + c) per axis (upper bound exclusive, :205-303), leaving
  entries of A at 0 (:252-254), zeroes the pick again and snapshots the cache as column i + 1 of
  delta_cached_iters (:318-332);
* the last pick is the arg-max of the final cache (:360-362).

The tapered covariance is the beta-decay filter of main_architecture_2_sampledistribution.py:361-421
(oracle/covariance.index_taper) over an EQ / Matern kernel matrix of a jittered grid; it is INPUT
data, stored in each fixture.  Output: tests/golden/alg3_<case>.npz (cov, X, order, dci, cache)
and tests/golden/alg3_golden.json (parameters + picks).  Only data is committed.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import _import_reference  # noqa: E402
from oracle import taper as lpo  # noqa: E402
from vgposp_amd.data_generation import grid_points, grid_spacing  # noqa: E402

EPS = 1e-6     # snippets_a2.py:161-163
SMALL = 1e-7   # snippets_a2.py:480
SHIFT = 0.01 + 1e-6  # noise 1e-2 + GP jitter 1e-6, as the C4 tests and bench

# (name, shape, kernel, beta, cutoff, k, seed)
CASES = [
    ("g555_eq_b4_c1", (5, 5, 5), "eq", 4.0, 1, 8, 11),
    ("g555_eq_b4_c2", (5, 5, 5), "eq", 4.0, 2, 8, 12),
    ("g555_m32_b4_c3", (5, 5, 5), "matern32", 4.0, 3, 8, 13),
    ("g654_m52_b4_c3", (6, 5, 4), "matern52", 4.0, 3, 8, 14),
    ("g565_eq_b25_c2", (5, 6, 5), "eq", 2.5, 2, 8, 15),
    ("g666_eq_b25_c3", (6, 6, 6), "eq", 2.5, 3, 8, 16),
    ("g666_m52_b4_c1", (6, 6, 6), "matern52", 4.0, 1, 10, 17),
    ("g777_eq_b4_c2", (7, 7, 7), "eq", 4.0, 2, 6, 18),
    # config C4's own parameters (bench.py c4_line, main_architecture_2_sampledistribution.py:973):
    # EQ, beta 4, window cutoff 3, noise 1e-2 + 1e-6, ls 2h; k = 24 so the bounded-lazy form
    # refines over several batches (about 20 CPU-minutes of reference arithmetic; --jobs 8)
    ("g888_eq_b4_c3", (8, 8, 8), "eq", 4.0, 3, 24, 19),
]


def window(y, shape, cutoff):
    I0, I1, I2 = shape
    s0, s1 = I1 * I2, I2
    i0 = y // s0
    i1 = (y - i0 * s0) // s1
    i2 = y - i0 * s0 - i1 * s1
    for j0 in range(max(i0 - cutoff, 0), min(i0 + cutoff, I0)):
        for j1 in range(max(i1 - cutoff, 0), min(i1 + cutoff, I1)):
            for j2 in range(max(i2 - cutoff, 0), min(i2 + cutoff, I2)):
                yield s0 * j0 + s1 * j1 + j2


_W = {}  # worker state: the reference module and the jittered matrix (inherited through fork)


def _delta(args):
    y, A, Abar = args
    alg2, S = _W["alg2"], _W["S"]
    # tf.sets keep their values sorted: A \ {y} and Abar \ {y} in ascending order
    Ay = sorted(set(A) - {y})
    nom = float(np.asarray(alg2.nominator(y, Ay, S)).reshape(-1)[0]) - EPS
    den = float(np.asarray(alg2.denominator(y, sorted(set(Abar) - {y}), S)).reshape(-1)[0]) - EPS
    return 0.0 if (abs(den) < SMALL or abs(nom) < SMALL) else nom / den


def _worker_init():
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)


def alg3_reference_arithmetic(alg2, cov, k, shape, cutoff, jobs=1):
    """The window loop of snippets_a3.py over the reference's own per-delta arithmetic.  The deltas
    of one round are independent evaluations, so with ``jobs`` > 1 they run in forked worker
    processes (one BLAS thread each): the same calls on the same inputs."""
    N = cov.shape[0]
    _W["alg2"], _W["S"] = alg2, cov + EPS * np.eye(N)
    V = list(range(N))
    A, Abar = [], list(range(N))
    pool = None
    if jobs > 1:
        import multiprocessing as mp
        pool = mp.get_context("fork").Pool(jobs, initializer=_worker_init)

    def deltas(ys):
        work = [(y, list(A), list(Abar)) for y in ys]
        return pool.map(_delta, work, chunksize=1) if pool else [_delta(w) for w in work]

    cache = np.full(N, 1e8)
    dci = np.zeros((N, k))
    cache[:] = deltas(range(N))
    dci[:, 0] = cache
    for i in range(k - 1):
        y = int(alg2.argmax_cache_linear(cache, A, V))
        A.append(y)
        Abar.remove(y)
        cache[y] = 0.0
        win = list(window(y, shape, cutoff))
        todo = [yj for yj in win if yj not in A]
        vals = dict(zip(todo, deltas(todo)))
        for yj in win:
            cache[yj] = 0.0 if yj in A else vals[yj]
        cache[y] = 0.0
        dci[:, i + 1] = cache
        print(f"  round {i + 1}: pick {y}", flush=True)
    A.append(int(alg2.argmax_cache_linear(cache, A, V)))
    if pool:
        pool.close()
        pool.join()
    return A, cache, dci


def main(only=(), jobs=1):
    """``only``: case names to (re)generate; the others keep their committed entries."""
    alg2 = _import_reference()
    alg2.print = lambda *a, **kw: None
    path = os.path.join(HERE, "alg3_golden.json")
    golden = {}
    if only and os.path.exists(path):
        with open(path) as f:
            golden = json.load(f)
    for name, shape, kind, beta, cutoff, k, seed in CASES:
        if only and name not in only:
            continue
        t0 = time.time()
        X = grid_points(shape, jitter=0.05, seed=seed)
        ls = 2.0 * grid_spacing(shape)
        cov = lpo.tapered_cov(X, shape, beta, kind=kind, ls=ls, diag_shift=SHIFT)
        order, cache, dci = alg3_reference_arithmetic(alg2, cov, k, list(shape), cutoff, jobs)
        np.savez_compressed(os.path.join(HERE, f"alg3_{name}.npz"), cov=cov, X=X,
                            order=np.asarray(order, dtype=np.int64), dci=dci, cache=cache)
        golden[name] = dict(shape=list(shape), kernel=kind, beta=beta, cutoff=cutoff, k=k,
                            seed=seed, ls=float(ls), diag_shift=SHIFT, jitter=0.05, order=order,
                            pick_deltas=[float(dci[a, i]) for i, a in enumerate(order)])
        print(name, order, f"{time.time() - t0:.1f} s", flush=True)
    with open(path, "w") as f:
        json.dump(golden, f, indent=1)


if __name__ == "__main__":
    argv = sys.argv[1:]
    jobs = 1
    if argv[:1] == ["--jobs"]:
        jobs, argv = int(argv[1]), argv[2:]
    main(tuple(argv), jobs)

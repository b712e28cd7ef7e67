"""CPU fixture for the headline's own 50 picks at N = 65,536 (verdict r5, item 1).

Run in the build container (62 GB of RAM, no GPU; ~25 min on 8 cores):

    OMP_NUM_THREADS=8 python tests/golden/make_golden_65k.py

The workload is bench.py's main line exactly: ``workloads.placement_split((64, 32, 32), 0)`` (a
jittered 64 x 32 x 32 grid, seed 0), EQ kernel, amplitude 1, length scale 2h, diagonal shift
1e-2 + 1e-6, k = 50 lazy-greedy placements (placement_algorithm2.py:151-219) with no extra jitter.

Nothing N x N is copied: Sigma's lower triangle is assembled straight into ONE Fortran-ordered
buffer (34.4 GB) and replaced in place by L, then by M = L^-1 (a blocked Cholesky and a blocked
triangular inverse driven from here, every LAPACK / BLAS call on at most N x 4096 operands:
LAPACK's own dpotrf on the whole buffer segfaulted inside OpenBLAS, LP64 and ILP64 builds alike).
Q_yy = |M e_y|^2 and Q e_a = M^T (M e_a) are read from that triangle.  The rounds are the oracle's
incremental lazy greedy (``oracle.placement.placement_lazy_columns``, the core of
``placement_lazy_incremental``, which test_oracle.py pins to the reference-executed goldens), with
Sigma e_y rebuilt from the points.  This is an independent route to the GPU's numbers: different
blocking, different summation orders, OpenBLAS instead of the HIP kernels.  The two agree to rounding, so the picks must be
equal unless two candidates' deltas tie to ~1e-12; the fixture stores each round's margin (the
pick's delta minus the best other cache entry) so a divergence can be judged.

Output: tests/golden/bench65k_cpu_picks.json (picks, deltas, per-round margins, wall times, BLAS
threads).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def assemble_lower_fortran(X, ls, shift, block=512):
    """Sigma's lower triangle (incl. diagonal) into a Fortran-ordered N x N buffer: column block
    [j0, j1) gets rows j0..N-1.  K = exp(-0.5 |x_i - x_j|^2 / ls^2), + shift on the diagonal
    (the GPU's kernel_matrix.hip forms the same sum of squared differences)."""
    N = X.shape[0]
    F = np.empty((N, N), dtype=np.float64, order="F")
    inv_ls2 = 1.0 / (ls * ls)
    for j0 in range(0, N, block):
        j1 = min(N, j0 + block)
        d2 = np.zeros((N - j0, j1 - j0))
        for k in range(X.shape[1]):
            e = X[j0:, k][:, None] - X[j0:j1, k][None, :]
            d2 += e * e
        blk = np.exp(-0.5 * d2 * inv_ls2)
        blk[np.arange(j1 - j0), np.arange(j1 - j0)] += shift
        F[j0:, j0:j1] = blk
    return F


def blocked_cholesky_inverse(F, nb=4096, log=print):
    """In place on the lower triangle of the Fortran-ordered N x N buffer F: F <- L, then
    F <- M = L^-1 (Sigma = L L^T).  Blocked right-looking Cholesky and a right-to-left blocked
    triangular inverse, every LAPACK / BLAS call on at most N x nb operands (LAPACK's dpotrf on the
    whole 65,536 x 65,536 buffer segfaulted inside OpenBLAS, LP64 and ILP64 builds alike).  The
    strictly upper triangle is never read (it holds whatever the buffer held)."""
    from scipy.linalg import lapack

    N = F.shape[0]
    nbk = (N + nb - 1) // nb
    for kb in range(nbk):
        k0, k1 = kb * nb, min(N, (kb + 1) * nb)
        D = np.asfortranarray(np.tril(F[k0:k1, k0:k1]))
        Dc, info = lapack.dpotrf(D, lower=1, clean=1)
        assert info == 0, f"dpotrf info {info} at block {kb}"
        F[k0:k1, k0:k1] = Dc
        if k1 == N:
            break
        # panel: P = A21 L11^-T
        P = np.asfortranarray(F[k1:, k0:k1])
        Li = lapack.dtrtri(Dc, lower=1)[0]
        P = P @ np.tril(Li).T
        F[k1:, k0:k1] = P
        # trailing lower triangle: A22 -= P P^T, one nb-wide column block at a time
        for jb in range(kb + 1, nbk):
            j0, j1 = jb * nb, min(N, (jb + 1) * nb)
            F[j0:, j0:j1] -= P[j0 - k1:] @ P[j0 - k1:j1 - k1].T
        log(f"cholesky block {kb + 1}/{nbk}")
    for jb in reversed(range(nbk)):
        j0, j1 = jb * nb, min(N, (jb + 1) * nb)
        Xjj = np.tril(lapack.dtrtri(np.asfortranarray(np.tril(F[j0:j1, j0:j1])), lower=1)[0])
        if j1 < N:
            # X21 = -X22 L21 X11 with X22 = L22^-1 already in place (columns >= j1)
            Lcol = np.asfortranarray(F[j1:, j0:j1])
            out = np.empty_like(Lcol)
            for ib in range(jb + 1, nbk):
                i0, i1 = ib * nb, min(N, (ib + 1) * nb)
                acc = np.tril(F[i0:i1, i0:i1]) @ Lcol[i0 - j1:i1 - j1]
                if i0 > j1:
                    acc += F[i0:i1, j1:i0] @ Lcol[:i0 - j1]
                out[i0 - j1:i1 - j1] = acc
            F[j1:, j0:j1] = -(out @ Xjj)
        F[j0:j1, j0:j1] = Xjj
        log(f"inverse block {nbk - jb}/{nbk}")


def lower_colnorms2(F, nb=4096):
    """diag(M^T M) = squared column norms of the lower triangle of F."""
    N = F.shape[0]
    d = np.empty(N)
    for j0 in range(0, N, nb):
        j1 = min(N, j0 + nb)
        d[j0:j1] = (np.tril(F[j0:j1, j0:j1]) ** 2).sum(0) + (F[j1:, j0:j1] ** 2).sum(0)
    return d


def lower_mtm_col(F, a, nb=4096):
    """M^T (M e_a) for the lower-triangular M held in F's lower triangle."""
    N = F.shape[0]
    v = np.zeros(N)
    v[a:] = F[a:, a]
    u = np.empty(N)
    for j0 in range(0, N, nb):
        j1 = min(N, j0 + nb)
        u[j0:j1] = np.tril(F[j0:j1, j0:j1]).T @ v[j0:j1] + F[j1:, j0:j1].T @ v[j1:]
    return u


def main():
    import argparse

    from oracle.placement import placement_lazy_columns
    from vgposp_amd.workloads import placement_split

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs=3, default=[64, 32, 32])
    ap.add_argument("--k", type=int, default=50)
    ap.add_argument("--out", default=os.path.join(HERE, "bench65k_cpu_picks.json"))
    ap.add_argument("--nb", type=int, default=4096)
    args = ap.parse_args()
    shape, k, shift = tuple(args.shape), args.k, 1e-2 + 1e-6
    X, ls = placement_split(shape, 0)
    N = X.shape[0]
    out_path = args.out
    t = {}

    def mark(name, t0):
        t[name] = round(time.perf_counter() - t0, 2)
        print(f"[65k] {name}: {t[name]} s", flush=True)

    t0 = time.perf_counter()
    F = assemble_lower_fortran(X, ls, shift)
    mark("assemble_s", t0)
    t0 = time.perf_counter()
    blocked_cholesky_inverse(F, nb=args.nb, log=lambda m: print(f"[65k] {m} "
                             f"({time.perf_counter() - t0:.0f} s)", flush=True))
    mark("cholesky_inverse_s", t0)
    t0 = time.perf_counter()
    q_diag = lower_colnorms2(F, args.nb)
    mark("diag_q_s", t0)
    sigma_diag = np.full(N, 1.0 + shift)
    inv_ls2 = 1.0 / (ls * ls)

    def sigma_row(y):
        d = X - X[y]
        r = np.exp(-0.5 * np.einsum("ij,ij->i", d, d) * inv_ls2)
        r[y] += shift
        return r

    def q_col(y):          # Q e_y = M^T (M e_y)
        return lower_mtm_col(F, y, args.nb)

    deltas, margins = [], []

    def log(r, y, d):
        print(f"[65k] round {r}: pick {y} delta {d!r} margin {margins[-1]!r}", flush=True)

    t0 = time.perf_counter()
    picks = placement_lazy_columns(sigma_diag, sigma_row, q_diag, q_col, k, deltas_out=deltas,
                                   margins_out=margins, log=log)
    mark("rounds_s", t0)
    rec = {
        "workload": "bench.py main line: 64x32x32 jittered grid seed 0, EQ amp 1 ls 2h noise "
                    "1e-2+1e-6, k=50 lazy greedy (placement_algorithm2.py:151-219)",
        "generator": "tests/golden/make_golden_65k.py: LAPACK dpotrf + dpotri in place (one "
                     "Fortran buffer), oracle.placement.placement_lazy_columns",
        "shape": list(shape), "N": N, "k": k, "picks": [int(v) for v in picks], "deltas": deltas,
        "margins": margins, "times": t,
        "blas_threads": os.environ.get("OMP_NUM_THREADS"),
        "numpy": np.__version__,
    }
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)
    print(f"[65k] wrote {out_path}", flush=True)


if __name__ == "__main__":
    main()

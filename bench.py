"""Benchmark of the hot path: greedy MI sensor placement on an N = 65,536-point 3-D grid
(64 x 32 x 32, EQ kernel) — BASELINE.json's metric "greedy sensor placements/sec + fp64 Cholesky
GF/s on N=65k 3D grid".

One step = the whole job for ONE placement problem, with the grid points already resident in HBM:
  assemble Sigma = K(X, X) + (noise + jitter) I  (kernel_matrix, HBM-write-bound)
  -> fused Cholesky + inverse of Sigma             (potrf sweep, fp64 MFMA-bound, 2N^3/3 flops)
  -> k = 50 lazy-greedy selections                 (per round one HBM-bound triangular mat-vec)
value = placements per second of that job.  With --gpus N the SAME problem is candidate-sharded
over the N ranks (vgposp_amd.sharded_placement over RCCL): the ranks factor Sigma together
(vgposp_amd.dist_cholesky: each large node of the recursive Cholesky has its panel TRSM and SYRK
split over the ranks, shares all-gathered), each rank forms L^-1 only in its own candidate columns
(1/N of the inverse), and per round all-reduces the pick's column of L^-1, all-gathers the delta
slabs and all-reduces the pivot row.  Strong scaling.  The timed loop runs with the library's event timing OFF;
the roofline numbers come from one more, profiled, step.

Also reported: fp64 Cholesky GF/s (plain potrf of the same Sigma, N^3/3 flops); config C4 (the
128^3 local-kernel greedy, candidates sharded over the same ranks: where sharding pays); at N > 1
the independent-splits throughput (one 64x32x32 split per rank) as a labelled extra; at N = 1 the
C2 / C3 / C5 lines and a CPU baseline (the oracle timed on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense fp64 matrix peak (spec)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (spec), MI355X_MICROARCH.md
METRIC = "greedy sensor placements/sec + fp64 Cholesky GF/s on N=65k 3D grid"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--shape", type=int, nargs=3, default=[64, 32, 32])
    p.add_argument("--k", type=int, default=50)
    p.add_argument("--kernel", default="eq")
    p.add_argument("--noise", type=float, default=1e-2)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    p.add_argument("--cpu-shape", type=int, nargs=3, default=[8, 8, 8])
    p.add_argument("--cpu-k", type=int, default=2)
    p.add_argument("--no-potrf", action="store_true", help="skip the separate potrf GF/s run")
    p.add_argument("--no-vgp", action="store_true", help="skip the C3 / C5 VGP training lines")
    p.add_argument("--no-c2", action="store_true", help="skip the C2 assembly + potrf line")
    p.add_argument("--vgp-steps", type=int, default=10)
    p.add_argument("--no-vgp-mixed", action="store_true",
                   help="skip C5 as named (the fp32 factor + fp64 refinement; slower than fp64 at "
                        "M = 1,024 on MI355X, DESIGN.md §8)")
    p.add_argument("--no-c4", action="store_true", help="skip the C4 (128^3 exact algorithm 3) line")
    p.add_argument("--c4-steps", type=int, default=10)
    p.add_argument("--no-sweep", action="store_true",
                   help="skip the 32^3 / 64^3 / 128^3 grid sweep")
    p.add_argument("--no-c4-selinv", action="store_true",
                   help="skip the C4 selected-inverse cross-check run")
    p.add_argument("--no-splits", action="store_true",
                   help="skip the N > 1 independent-splits extra")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                        "the multi-rank path on one GPU with VGPOSP_BENCH_DEVICE=0)")
    p.add_argument("--c4-pmc", default=os.path.join(ROOT, "profiles", "pmc_c4_r6.json"),
                   help="per-run C4 kernel bytes from rocprofv3 PMC passes (tools/pmc_c4.py)")
    p.add_argument("--rank-check", action="store_true",
                   help="(tests) every rank prints its rank / world size and exits before any GPU call")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_r6.json"),
                   help="per-launch HBM bytes from a rocprofv3 PMC pass of this command")
    return p.parse_args()


def cpu_threads():
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"]
        if n:
            return int(max(n))
    except Exception:
        pass
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, N):
    """The same algorithm on the host: the oracle's incremental-precision lazy greedy
    (oracle.placement.placement_lazy_incremental: LAPACK dpotrf + dpotri once, O(N^2) numpy per
    round — the maths the HIP path runs) on a jittered 16x16x32 grid (N = 8,192), k = 50, all BLAS
    threads; plus the reference's own algorithm (the pinv-faithful restatement of
    placement_algorithm2.py, one SVD per delta evaluation) on an 8^3 grid with k = 2, and an
    OpenBLAS Cholesky of the same kernel family."""
    from oracle import gp as ogp
    from oracle import placement as op
    from vgposp_amd.data_generation import grid_points, grid_spacing

    def sigma(shape):
        X = grid_points(shape, jitter=0.05, seed=0)
        S = ogp.kernel_matrix(args.kernel, X, X, 1.0, 2 * grid_spacing(shape))[0]
        S[np.diag_indices(len(X))] += args.noise + 1e-6
        return S

    shape = (16, 16, 32)
    S = sigma(shape)
    # the host's CPUs, capped at 64: numpy / scipy's OpenBLAS is built for at most 64 threads
    # (MAX_THREADS=64), so asking it for the box's 256 runs no faster.  ONE thread count for the
    # whole leg: changing OpenBLAS's count back up inside the process (64 -> 16 -> 64) segfaulted
    # it in round 6 (tools/cpu_blas_probe.py runs each count in its own process without a fault)
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:  # pragma: no cover
        threadpool_limits = None
    ncpu = os.cpu_count() or 1
    try:
        naff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        naff = ncpu
    th_main = min(naff, 64)
    # (set once here and never restored inside the leg: the pinv sample and the Cholesky below
    # run at the same count)
    if threadpool_limits is not None:
        threadpool_limits(limits=th_main, user_api="blas")
    parts = {}
    t0 = time.perf_counter()
    op.placement_lazy_incremental(S, args.k, timings=parts)
    t_inc = time.perf_counter() - t0
    del S
    if threadpool_limits is None:  # pragma: no cover
        th_main = cpu_threads()
    runs = {th_main: t_inc}
    ps = tuple(args.cpu_shape)
    Sp = sigma(ps)
    trace = []
    t0 = time.perf_counter()
    op.placement_algorithm_2(Sp, args.cpu_k, trace=trace)
    t_pinv = time.perf_counter() - t0
    nevals = sum(1 for e in trace if e[0] != "select")
    # the GPU on the SAME samples (so the two can be read side by side)
    gpu_same = gpu_on_sample(S_keep := sigma(shape), args.k)
    gpu_ref = gpu_on_sample(Sp, args.cpu_k)
    del S_keep
    nc = 6144
    Sc = sigma((24, 16, 16))
    t0 = time.perf_counter()
    np.linalg.cholesky(Sc)
    tc = time.perf_counter() - t0
    n_inc = int(np.prod(shape))
    # the sample's two parts scaled by their own orders: the O(n^3) factor + inverse by (N / n)^3,
    # the O(k n^2) rounds (and the sample's fixed costs) by (N / n)^2
    f3, f2 = (N / n_inc) ** 3, (N / n_inc) ** 2
    t_fit = parts["factor_inverse"] * f3 + (t_inc - parts["factor_inverse"]) * f2
    return {
        "value": args.k / t_inc,
        "unit": "placements/s",
        "cores": th_main,
        "os_cpu_count": ncpu,
        "affinity_cpus": naff,
        "by_threads": {str(t): args.k / v for t, v in runs.items()},
        "kind": "port",
        "sample": (f"oracle placement_lazy_incremental (same algorithm as the GPU path) on a "
                   f"jittered {shape[0]}x{shape[1]}x{shape[2]} grid (N={n_inc}), k={args.k}: "
                   f"{t_inc:.1f} s; the GPU line is at N={N}, where the O(N^3) init alone is "
                   f"{(N / n_inc) ** 3:.0f}x this sample's"),
        "gpu_same_sample": gpu_same,
        # the headline's own config is N = 65,536 (timing it there takes most of an hour of host
        # time).  Scaling the WHOLE sample time by (N / n)^3 over-scales its O(n^2) rounds and
        # fixed costs, and BLAS runs faster at large n, so that time is too long and its rate a
        # LOWER bound of the CPU's rate at the config; the estimate scales each part by its order
        "at_config_lower_bound": {
            "value": args.k / (t_inc * (N / n_inc) ** 3), "unit": "placements/s", "N": N,
            "model": f"whole sample time x (N / {n_inc})^3 (a lower bound of the rate)"},
        "at_config_estimate": {
            "value": args.k / t_fit, "unit": "placements/s", "N": N,
            "model": (f"factor + inverse {parts['factor_inverse']:.2f} s x (N / {n_inc})^3 + rounds "
                      f"and the rest {t_inc - parts['factor_inverse']:.2f} s x (N / {n_inc})^2 = "
                      f"{t_fit:.0f} s")},
        # measured at the config itself, on another host: the oracle's algorithm on the bench's
        # exact workload, in the build container (tests/golden/bench65k_cpu_picks.json)
        "at_config_measured": _cpu_fixture_rate(),
        "reference_algorithm": {
            "value": args.cpu_k / t_pinv, "unit": "placements/s",
            "sample": (f"pinv restatement of placement_algorithm2.placement_algorithm_2 on a "
                       f"jittered {ps[0]}x{ps[1]}x{ps[2]} grid (N={len(Sp)}), k={args.cpu_k}: "
                       f"{nevals} delta evaluations (one SVD each) in {t_pinv:.1f} s"),
            "gpu_same_sample": gpu_ref},
        "cholesky_gflops": nc ** 3 / 3 / tc / 1e9,
        "cholesky_sample": f"numpy.linalg.cholesky at N={nc}",
        "cpu_model": cpu_model(),
    }


def _cpu_fixture_rate():
    """placements/s of the host run that made tests/golden/bench65k_cpu_picks.json (the bench's
    own N = 65,536 workload, the oracle's algorithm; the build container, not the GPU box)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench65k_cpu_picks.json")) as f:
            fx = json.load(f)
    except (OSError, ValueError):
        return None
    t = fx["times"]
    secs = t["cholesky_inverse_s"] + t["diag_q_s"] + t["rounds_s"]
    return {"value": fx["k"] / secs, "unit": "placements/s", "N": fx["N"], "seconds": secs,
            "host": f"the build container, {fx.get('blas_threads')} OpenBLAS threads (blocked "
                    "Cholesky + inverse, then the incremental lazy rounds; Sigma's assembly "
                    f"({t['assemble_s']} s) excluded); its picks are the ones the main line's "
                    "matches_committed_picks compares with"}


def gpu_on_sample(S, k, reps=5):
    """placements/s of the HIP path on the host covariance S (device-resident before timing:
    Sigma copied in, factored in place, k lazy rounds; best of `reps`), with its picks."""
    import torch

    from vgposp_amd.placement_algorithm2 import GreedyPlacement
    Sd = torch.as_tensor(S, device="cuda")
    work = torch.empty_like(Sd)
    g = GreedyPlacement(work, k)
    best = None
    for _ in range(reps + 1):
        work.copy_(Sd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.run(k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    g.check()
    picks = [int(v) for v in g.selected[:k].cpu()]
    del g, work, Sd
    torch.cuda.empty_cache()
    return {"value": k / best, "unit": "placements/s", "N": int(S.shape[0]), "k": k,
            "picks_head": picks[:6]}


def load_traffic(path, kernel, N, shape, k):
    """Per-launch HBM bytes of `kernel` measured by a rocprofv3 PMC pass of this same workload
    (tools/pmc_traffic.py writes the file; (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 per the gfx950
    correction in MI355X_MICROARCH.md).  None when absent, measured on another workload, or
    measured on a build whose kernel sources differ from this one's (source_sha256)."""
    from vgposp_amd._lib import source_hash
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    w = t.get("workload", {})
    if w.get("N") != N or list(w.get("shape", [])) != list(shape) or w.get("k") != k:
        return None
    kern = t.get("kernels", {}).get(kernel)
    if not kern:
        return None
    if kern.get("source_sha256") != source_hash(kernel):
        return {"stale": True, "source": os.path.relpath(path, ROOT),
                "recorded_sha256": kern.get("source_sha256"), "build_sha256": source_hash(kernel)}
    return {"bytes_per_launch": kern["hbm_bytes_per_launch"], "source": os.path.relpath(path, ROOT)}


def _committed(name, picks):
    """Whether `picks` equal the selection committed in tests/golden/<name> (the headline's:
    a CPU run of the same workload; C4's: the C oracle's; at N > 1 the sharded path must
    reproduce it), None if absent."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", name)) as f:
            want = json.load(f).get("picks")
    except (OSError, ValueError):
        return None
    return None if want is None else [int(a) for a in picks] == [int(a) for a in want]


def vgp_line(args, which="c3", precision="fp64", world=1, rank=0, barrier=None, maxtime=None):
    """Config C3 or C5: VGP training steps/s — optimal posterior over all N +
    minibatch ELBO + analytic gradient + Adam(0.01), minibatch N / 8.
      C3: N = 64^3 observations over [-7, 7]^3, M = 8^3, 3-D.
      C5: N = 65,536 uniform over [-2, 2]^5, M = 4^5 = 1,024, 5-D (fp64, or the fp32 factor +
          fp64 refinement the config names).
    With world > 1 the N observations are sharded over the ranks (data parallel):
    each rank assembles its Kzx slab and its share of Kzx Kzx^T / Kzx y, two all-reduces per step
    (M^2 + M, then 2 + M d doubles), the same minibatch on every rank; strong scaling."""
    import torch
    import torch.distributed as dist

    from vgposp_amd import _lib
    from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph, vgp_c5_data
    X, y, Z = vgp_c3_data() if which == "c3" else vgp_c5_data()
    N, M = len(X), len(Z)
    B = N // 8
    shard = np.array_split(np.arange(N), world)[rank]
    group = dist.group.WORLD if world > 1 else None
    kernel = "eq" if which == "c3" else "matern52"
    train_op, loss, xb, yb = vgp_c3_graph(X[shard], y[shard], Z, B, precision=precision,
                                          group=group, n_total=N, kernel=kernel)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    rng = np.random.default_rng(1)
    idx = [torch.as_tensor(rng.integers(0, N, B), device="cuda") for _ in range(args.vgp_steps + 2)]
    first = float(train_op.run({xb: Xd[idx[0]], yb: yd[idx[0]]}))
    train_op.run({xb: Xd[idx[1]], yb: yd[idx[1]]})  # captures the step's HIP graph (1 rank)
    torch.cuda.synchronize()
    if barrier:
        barrier()
    t0 = time.perf_counter()
    for i in range(2, args.vgp_steps + 2):
        last = train_op.run({xb: Xd[idx[i]], yb: yd[idx[i]]})
    torch.cuda.synchronize()
    if barrier:
        barrier()
    dt = (maxtime(time.perf_counter() - t0) if maxtime else time.perf_counter() - t0) / args.vgp_steps
    train_op.check()  # the last step's Cholesky statuses (each earlier one: at the next run)
    # GEMM share from one more step run eagerly with the library's event timing on
    _lib.prof_enable(True)
    train_op.run({xb: Xd[idx[1]], yb: yd[idx[1]]})
    torch.cuda.synchronize()
    ms, n, fl, _ = _lib.prof_query("gemm_f64")
    _lib.prof_enable(False)
    desc = ("C3: 64^3 observations over [-7,7]^3, 8^3 inducing points" if which == "c3" else
            "C5: 65,536 observations U[-2,2]^5, 4^5 inducing points, " +
            ("fp64" if precision == "fp64" else
             f"M x M Cholesky in fp32 (f32 MFMA) + {precision.partition(':')[2] or 3} fp64 "
             "refinement steps (ELBO within 1e-5 of fp64), the rest fp64"))
    # roofline of the step's dominant kernel, the fp64 MFMA GEMM: its launches' algorithmic flops
    # (the library's counters: 2 m n k per launch, triangles at their true flops) over their summed
    # HIP-event time.  Beside it the step's own algorithmic flops over the whole step time:
    # 2 M^2 N (the products over all N observations) + 2 M^2 B (the minibatch products) + M^3 / 3
    # (one M x M Cholesky)
    alg = 2.0 * M * M * N + 2.0 * M * M * B + M ** 3 / 3.0
    roof = None
    if ms:
        ach = fl / (ms * 1e-3) / 1e12
        roof = {"kernel": "gemm_f64", "bound": "mfma", "unit": "TFLOP/s", "achieved": ach,
                "peak": FP64_MFMA_PEAK_TFLOPS, "frac": ach / FP64_MFMA_PEAK_TFLOPS,
                "launches_per_step": n, "avg_launch_ms": ms / max(n, 1),
                "share_of_step": ms / (dt * 1e3), "traffic": None,
                "step_algorithmic_flops": alg,
                "step_algorithmic_tflops": alg / dt / 1e12,
                "step_frac": alg / dt / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                "measured": "HIP events around every GEMM launch of one eager step (rank 0)"}
    out = {"metric": "VGP ELBO Adam steps/sec", "value": 1.0 / dt, "ms_per_step": dt * 1e3,
           "n_gpus": world, "scaling": "strong" if world > 1 else None,
           "config": {"workload": desc + (", EQ" if kernel == "eq" else ", MaternFiveHalves") +
                                  ", optimal posterior over all N + minibatch ELBO + grads + "
                                  "Adam(0.01)", "N": N, "M": M, "d": X.shape[1],
                      "batch": B,
                      "parallelism": "single" if world == 1 else f"observations sharded x{world}"},
           "loss_first": first, "loss_last": float(last),
           "graph": bool(train_op.graph),
           "gemm": {"ms_per_step": ms, "tflops": fl / (ms * 1e-3) / 1e12 if ms else None,
                    "launches_per_step": n, "note": "one eager step with event timing (rank 0)"},
           "roofline": roof}
    if world > 1:
        out["allreduce_doubles_per_step"] = M * M + M + 2 + M * X.shape[1]
    return out


def c2_line(reps=5):
    """Config C2: N = 32,768 (32^3 grid) K assembly (lower triangle + noise on the
    diagonal, GB/s of algorithmic bytes 4 n (n + 1) + 8 d n) and the fp64 Cholesky (GF/s of
    n^3 / 3), each the best of ``reps`` runs after a warm-up.  The kernel parameters are device
    tensors made once, so no host-to-device copy sits inside the timed region."""
    import torch

    from vgposp_amd import linalg
    from vgposp_amd.workloads import c2_data
    X, ls = c2_data()
    n, d = X.shape
    Xd = linalg.as_device(X)
    A = torch.empty((1, n, n), dtype=torch.float64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    amp_d, ls_d, sh_d = (linalg.as_device([v]) for v in (1.0, ls, 0.01 + 1e-6))

    def assemble():
        linalg.kernel_matrix("eq", Xd, None, amp_d, ls_d, diag_shift=sh_d, lower=True, out=A)

    def timed(fn, reps=reps):
        best = None
        for _ in range(reps):
            assemble()
            torch.cuda.synchronize()
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            t = ev[0].elapsed_time(ev[1]) * 1e-3
            best = t if best is None else min(best, t)
        return best

    assemble()
    linalg.cholesky_(A[0], check=True)  # warm-up (and the PD check)
    t_k = timed(assemble)
    t_c = timed(lambda: linalg.cholesky_(A[0], check=False), reps=2)
    del A
    torch.cuda.empty_cache()
    return {"config": {"workload": "C2: 32^3 grid over [-2,2]^3, EQ amp 1 ls 2h, noise 1e-2+1e-6",
                       "N": n},
            "assembly_ms": t_k * 1e3, "assembly_gbps": (4.0 * n * (n + 1) + 8.0 * d * n) / t_k / 1e9,
            "potrf_ms": t_c * 1e3, "potrf_gflops": n ** 3 / 3.0 / t_c / 1e9}


def c4_line(args, world, rank, barrier, maxtime):
    """Config C4: 128^3 = 2,097,152 candidates, k = 50, the reference's algorithm 3
    (snippets_a3.py:43-364) on the beta = 4 tapered covariance, window cutoff 3, exact
    (vgposp_amd.sparse_placement).  One step = the bounded-lazy form end to end: stencil
    coefficients, upper bounds of every Q_yy from K CG steps per candidate (Gauss-Radau bounds,
    K = 4 at beta = 4; sharded over the ranks, one all-gather), then the k rounds (refining a candidate by its CG column whenever the
    arg-max lands on a bounded one; replicated on every rank).  The multifrontal selected inverse
    (exact diag(Q) on fp64 MFMA fronts, subtree-to-subcube over the ranks) runs once beside it as
    the cross-check of the picks and reports its own rate."""
    import torch

    from vgposp_amd import _lib
    from vgposp_amd.sparse_placement import ExactTaperPlacement
    from vgposp_amd.workloads import c4_grid
    X, shape, ls = c4_grid()
    k, beta, cutoff = args.k, 4.0, 3
    run = ExactTaperPlacement(X, shape, k, cutoff, beta, ls=ls, diag_shift=args.noise + 1e-6,
                              method="bounds")
    run.run()
    torch.cuda.synchronize()
    ref = run.greedy.picks[:k].clone()
    reps = args.c4_steps
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run.run()
    torch.cuda.synchronize()
    barrier()
    dt = maxtime(time.perf_counter() - t0) / reps
    same = bool(torch.equal(ref, run.greedy.picks[:k]))
    picks = [int(v) for v in ref.cpu()]
    # one profiled step: the bounds pass and the rounds separately
    g = run.greedy
    _lib.prof_enable(True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    barrier()
    ev[0].record()
    c0, c1 = (0, run.prob.n)
    if world > 1:
        from vgposp_amd.sparse_placement import slab_of
        c0, c1 = slab_of(run.prob.n, world, rank)
    K, scale, width = g.bound_qdiag(run.qdiag, c0, c1)
    ev[1].record()
    if world > 1:
        from vgposp_amd.sparse_placement import allgather_slabs
        allgather_slabs(run.qdiag, run.group)
    ev[2].record()
    g.run_bounded(run.qdiag, k)
    ev[3].record()
    torch.cuda.synchronize()
    prof = _lib.prof_fold(_lib.prof_dump())
    _lib.prof_enable(False)
    bounds_ms, gather_ms, rounds_ms = (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]),
                                       ev[2].elapsed_time(ev[3]))
    nb = c1 - c0
    out = {"metric": "greedy sensor placements/sec", "value": k / dt, "unit": "placements/s",
           "ms_per_step": dt * 1e3, "n_gpus": world, "scaling": "strong",
           "config": {"workload": "C4: 128^3 jittered grid (N=2,097,152), EQ amp 1 ls 2h, "
                                  f"noise {args.noise}+1e-6, beta-decay taper beta={beta} "
                                  f"(support {run.prob.m} points), window cutoff {cutoff}, k={k}, "
                                  "exact algorithm 3 (dense-equivalent deltas, TF constants)",
                      "N": int(np.prod(shape)), "k": k,
                      "parallelism": "single" if world == 1 else
                      f"bounds sharded over {world} ranks (one all-gather), rounds replicated "
                      "(profiles/r6_c4_shard_model.json)"},
           "method": "bounded-lazy (K-step CG brackets of Q_yy, refinement by CG columns)",
           "picks_head": picks[:6],
           "deterministic_selection": same,
           "matches_committed_picks": (_committed("c4_picks.json", picks)
                                       if k == 50 and args.noise == 1e-2 else None),
           "bounds": {"ms": bounds_ms, "cg_steps": K, "bracket_rel_width": width,
                      "form": "gauss-radau" if g.bound_mu > 0 else "chebyshev",
                      "mu": g.bound_mu,
                      "candidates_this_rank": nb,
                      "mcandidates_per_s": nb / (bounds_ms * 1e-3) / 1e6},
           "allgather_ms": gather_ms if world > 1 else None,
           "exchanged_gb_per_step": (8.0 * (-(-run.prob.n // world)) * (world - 1) / 1e9
                                     if world > 1 else 0.0),
           "rounds_ms": rounds_ms, "refinements": g.refinements,
           "refine_batches": g.refine_batches, "host_reads": getattr(g, "host_reads", None),
           "roofline": c4_roofline(run, prof, nb, args.c4_pmc),
           "cg_iterations_per_column": g.cg_iters,
           "breakdown_ms": {n: v[0] for n, v in prof.items()}}
    # the selected-inverse form once: the same picks, and the fp64-MFMA rate of its fronts
    if not args.no_c4_selinv:
        sel = ExactTaperPlacement(X, shape, k, cutoff, beta, ls=ls, diag_shift=args.noise + 1e-6,
                                  method="selinv")
        sel.run()
        torch.cuda.synchronize()
        sel.check()
        comm = sel.sel.comm
        b0 = comm.bytes if comm is not None else 0
        _lib.prof_enable(True)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        barrier()
        e[0].record()
        sel.sel.run(out=sel.qdiag)
        e[1].record()
        sel.greedy.run(sel.qdiag, k)
        e[2].record()
        torch.cuda.synchronize()
        sprof = _lib.prof_fold(_lib.prof_dump())
        _lib.prof_enable(False)
        sel.check()
        sel_ms = e[0].elapsed_time(e[1])
        fl_alg = sel.sel.tree.flops(padded=False)
        gms, gl, gfl, _ = sprof.get("gemm_f64", (0.0, 0, 0.0, 0.0))
        gemm_tf = gfl / (gms * 1e-3) / 1e12 if gms else None
        out["selected_inverse"] = {
            "picks_equal": [int(v) for v in sel.greedy.picks[:k].cpu()] == picks,
            "ms": sel_ms, "rounds_ms": e[1].elapsed_time(e[2]),
            "placements_per_s": k / ((sel_ms + e[1].elapsed_time(e[2])) * 1e-3),
            "flops_algorithmic": fl_alg, "flops_this_rank_padded": sel.sel.flops(),
            "tflops_algorithmic": fl_alg / (sel_ms * 1e-3) / 1e12,
            "mfma_frac_algorithmic": fl_alg / (sel_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "gemm_tflops": gemm_tf,
            "gemm_frac": gemm_tf / FP64_MFMA_PEAK_TFLOPS if gemm_tf else None,
            "gemm_ms": gms, "gemm_launches": gl,
            "fronts": len(sel.sel.tree.fronts), "levels": len(sel.sel.lay.levels),
            "groups_this_rank": len(sel.sel.lay.groups), "plan_s": sel.sel.plan_s,
            "exchanged_gb": ((comm.bytes - b0) / 1e9) if comm is not None else 0.0,
            "breakdown_ms": {n: v[0] for n, v in sprof.items()},
            "note": "nested-dissection multifrontal Cholesky + Takahashi recurrences on batched "
                    "fp64 MFMA fronts, then the plain rounds; one profiled run"}
        del sel
        torch.cuda.empty_cache()
    # the CPU side: the plain-C restatement (oracle/c4_exact.c, OpenMP) on the whole workload —
    # its picks are the "bit-exact vs CPU" check at full size, its time the C4 CPU baseline
    if world == 1 and rank == 0 and not args.no_cpu:
        from oracle import c4_exact as oc4
        # at the runtime's default team (OMP_NUM_THREADS: 16 on the GPU box) and at every
        # logical CPU of the host; the value is the faster of the two
        runs = {}
        for th in sorted({oc4.lib().c4o_threads(), os.cpu_count() or 1}):
            st = {}
            cp, _ = oc4.exact_alg3(X, shape, k, cutoff, beta, ls=ls, diag_shift=args.noise + 1e-6,
                                   stats=st, threads=th)
            runs[th] = (st["seconds"], [int(v) for v in cp] == picks, st["refinements"])
        best = min(runs, key=lambda t: runs[t][0])
        out["cpu_baseline"] = {
            "value": k / runs[best][0], "unit": "placements/s", "cores": best,
            "os_cpu_count": os.cpu_count(),
            "by_threads": {str(t): k / v[0] for t, v in runs.items()},
            "kind": "port", "sample": f"the whole workload (128^3, k={k}), one run per team size",
            "picks_equal": all(v[1] for v in runs.values()), "seconds": runs[best][0],
            "refinements": runs[best][2],
            "note": "oracle/c4_exact.c: the same bounded-lazy algorithm 3 in C (OpenMP bounds, "
                    "sequential rounds)"}
    return out


L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: aggregate L2 bandwidth (4 MiB per XCD, 8 XCDs)


def c4_roofline(run, prof, ncand, pmc_path=None):
    """Rooflines of config C4's two dominant phases from one profiled run (`prof`: prof_fold'ed
    vgposp_prof_dump), with their algorithmic bytes:
      exact_bounds: each candidate y reads the coefficient rows of the nodes within K stencil
        steps (T rows of m doubles: its K-step Krylov space) and writes qdiag[y].  Unique bytes
        (the coefficient table once + qdiag) against HBM; the per-candidate operand bytes
        (T m 8 + 8) against the L2, where the neighbouring candidates' shared rows are served.
      exact_cg: per column and iteration the active region of (it + 1) stencil radii around the
        column's centre — the Manhattan ball (2R + 1)(2R^2 + 2R + 3) / 3 nodes for the 7-point
        stencil, whose CG walk skips the rest of the cube; the cube otherwise — at 8 (m + 9) bytes
        per node (coefficient row, r / p / q / x reads and writes), every column counted for the
        iteration cap (columns that converge earlier exit early, so this over-counts).
    `traffic`: FETCH + WRITE bytes per run from a rocprofv3 PMC pass (profiles/pmc_c4_*.json) when
    it was measured on this build's sources.  The block returned leads with whichever of the two
    took more time in the profiled run and nests the other ("cg" or "bounds")."""
    from vgposp_amd._lib import source_hash
    from vgposp_amd.sparse_placement import reach_table
    g = run.greedy
    pr = run.prob
    m = pr.m
    K = g.bound[0] if g.bound else None
    T = len(reach_table(pr.offs_np, K)[0]) if K else 0
    stride = (m + 1) & ~1
    b_ms = prof.get("exact_bounds", (0.0,))[0]
    uniq = pr.n * 8.0 * stride + ncand * 8.0
    oper = ncand * (8.0 * T * m + 8.0)
    out = {"kernel": "exact_bounds", "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "achieved": uniq / (b_ms * 1e-3) / 1e9 if b_ms else None, "traffic": None,
           "algorithmic_bytes": uniq, "candidates": ncand, "K": K, "reach_nodes": T,
           "l2_operand_bytes": oper, "ms_per_run": b_ms,
           "l2_achieved": oper / (b_ms * 1e-3) / 1e9 if b_ms else None, "l2_peak": L2_PEAK_GBS}
    if out["achieved"]:
        out["frac"] = out["achieved"] / HBM_PEAK_GBS
        out["l2_frac"] = out["l2_achieved"] / L2_PEAK_GBS
    cg_ms = prof.get("exact_cg", (0.0,))[0]
    box = 2 * g.radius * g.cg_iters + 1
    if m == 7 and g.radius == 1:  # the 7-point walk covers the diamond |d0| + |d1| + |d2| <= R
        node_its = sum((2 * R + 1) * (2 * R * R + 2 * R + 3) // 3
                       for R in (min(it + 1, g.cg_iters) for it in range(g.cg_iters)))
    else:
        node_its = sum(min(2 * (it + 1) * g.radius + 1, box) ** 3 for it in range(g.cg_iters))
    cg_bytes = g.refinements * node_its * 8.0 * (m + 9)
    out["cg"] = {"kernel": "exact_cg_a/b", "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                 "columns": g.refinements, "iterations": g.cg_iters, "batches": g.refine_batches,
                 "node_iterations_per_column": node_its, "algorithmic_bytes": cg_bytes,
                 "ms_per_run": cg_ms, "traffic": None,
                 "achieved": cg_bytes / (cg_ms * 1e-3) / 1e9 if cg_ms else None,
                 "launch_bound_floor_ms": g.refine_batches * (2 * g.cg_iters + 2) * 6.5e-3}
    if out["cg"]["achieved"]:
        out["cg"]["frac"] = out["cg"]["achieved"] / HBM_PEAK_GBS
    if pmc_path and os.path.exists(pmc_path):
        t = json.load(open(pmc_path))
        if t.get("source_sha256") == source_hash("exact") and t.get("workload", {}).get("N") == pr.n:
            kb = t["kernels"]
            bnd = [v for kk, v in kb.items() if kk.startswith("exact_bounds")]
            if bnd:
                out["traffic"] = sum(v["fetch_bytes_per_run"] + v["write_bytes_per_run"] for v in bnd)
                out["l2_hit_rate"] = bnd[0].get("l2_hit_rate")
            cgk = [v for kk, v in kb.items() if kk.startswith("exact_cg")]
            if cgk:
                out["cg"]["traffic"] = sum(v["fetch_bytes_per_run"] + v["write_bytes_per_run"]
                                           for v in cgk)
            out["traffic_source"] = os.path.relpath(pmc_path, ROOT)
        else:
            out["traffic_note"] = "null: the PMC file was measured on other kernel sources"
    if cg_ms > b_ms:  # lead with the dominant phase
        cg = out.pop("cg")
        cg["bounds"] = out
        return cg
    return out


def grid_sweep(args, world, rank, barrier, maxtime):
    """north_star's grid sizes: placements/s of k = 50 on 32^3, 64^3 and 128^3 at
    this run's GPU count.  32^3 (N = 32,768): the dense exact lazy greedy of the headline
    (placement_algorithm_2; sharded at N > 1) with its GEMM's fraction of the fp64 MFMA peak;
    64^3 and 128^3: the exact algorithm 3 on the beta = 4 tapered covariance (config C4's form: no
    dense cov_vv fits, 64^3 dense would be 550 GB), latency-bound, so no roofline fraction."""
    import torch

    from vgposp_amd import _lib, linalg
    from vgposp_amd.placement_algorithm2 import GreedyPlacement
    from vgposp_amd.sharded_placement import HipGreedyBackend, ShardedGreedyPlacement
    from vgposp_amd.sparse_placement import ExactTaperPlacement
    from vgposp_amd.workloads import c4_grid, placement_split
    k = 50
    out = {}
    # 32^3 dense
    shape = (32, 32, 32)
    X, ls = placement_split(shape, 0)
    N = len(X)
    Xd = linalg.as_device(X)
    amp_d, ls_d, sh_d = (linalg.as_device([v]) for v in (1.0, ls, args.noise + 1e-6))
    S = torch.empty((N, N), dtype=torch.float64, device="cuda")
    if world == 1:
        g = GreedyPlacement(S, k)

        def rounds():
            g.init()
            for _ in range(k):
                g.step(lazy=True)
    else:
        sh = ShardedGreedyPlacement(HipGreedyBackend(S, k), partition_inverse=True)
        g = sh.b.g

        def rounds():
            sh.run(k)

    def step():
        linalg.kernel_matrix("eq", Xd, None, amp_d, ls_d, diag_shift=sh_d, out=S[None])
        rounds()

    step()
    torch.cuda.synchronize()
    g.check()
    reps = 3
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    barrier()
    dt = maxtime(time.perf_counter() - t0) / reps
    g.check()
    _lib.prof_enable(True)
    step()
    torch.cuda.synchronize()
    gms, _, gfl, _ = _lib.prof_query("gemm_f64")
    _lib.prof_enable(False)
    gtf = gfl / (gms * 1e-3) / 1e12 if gms else None
    out["32^3_dense_alg2"] = {"N": N, "placements_per_s": k / dt, "ms_per_problem": dt * 1e3,
                              "gemm_tflops": gtf,
                              "gemm_frac_of_fp64_mfma": gtf / FP64_MFMA_PEAK_TFLOPS if gtf else None,
                              "selected_head": [int(v) for v in g.selected[:6].cpu()]}
    del S, g
    torch.cuda.empty_cache()
    # 64^3 and 128^3 tapered exact algorithm 3
    for n in (64, 128):
        Xc, shp, lsc = c4_grid(n)
        run = ExactTaperPlacement(Xc, shp, k, 3, 4.0, ls=lsc, diag_shift=args.noise + 1e-6,
                                  method="bounds")
        run.run()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(5):
            run.run()
        torch.cuda.synchronize()
        barrier()
        dt = maxtime(time.perf_counter() - t0) / 5
        _lib.prof_enable(True)
        run.run()
        torch.cuda.synchronize()
        sprof = _lib.prof_fold(_lib.prof_dump())
        _lib.prof_enable(False)
        picks = [int(v) for v in run.greedy.picks[:k].cpu()]
        ent = {"N": n ** 3, "placements_per_s": k / dt, "ms_per_problem": dt * 1e3,
               "picks_head": picks[:6],
               "roofline": c4_roofline(run, sprof, run.prob.n // world, None)}
        if world == 1 and rank == 0 and not args.no_cpu:
            from oracle import c4_exact as oc4
            st = {}
            th = os.cpu_count() or 1
            cp, _ = oc4.exact_alg3(Xc, shp, k, 3, 4.0, ls=lsc, diag_shift=args.noise + 1e-6,
                                   stats=st, threads=th)
            ent["cpu_baseline"] = {"value": k / st["seconds"], "unit": "placements/s",
                                   "cores": th, "kind": "port", "sample": "the whole problem",
                                   "picks_equal": [int(v) for v in cp] == picks}
        out[f"{n}^3_tapered_alg3"] = ent
        del run
        torch.cuda.empty_cache()
    out["note"] = ("k = 50 each; 32^3: jittered grid, EQ ls 2h, noise 1e-2 + 1e-6 (the headline's "
                   "workload at N = 32,768); 64^3 / 128^3: config C4's taper (beta 4, cutoff 3)")
    return out


def splits_line(args, world, barrier, maxtime, rank):
    """N > 1 extra: one independent 64x32x32 split per rank (weak scaling, no collective)."""
    import torch

    from vgposp_amd import linalg
    from vgposp_amd.placement_algorithm2 import GreedyPlacement
    from vgposp_amd.workloads import placement_split
    X, ls = placement_split(tuple(args.shape), rank)
    N = len(X)
    Xd = linalg.as_device(X)
    Sigma = torch.empty((N, N), dtype=torch.float64, device="cuda")
    g = GreedyPlacement(Sigma, args.k)

    def step():
        linalg.kernel_matrix(args.kernel, Xd, None, 1.0, ls, diag_shift=args.noise + 1e-6,
                             out=Sigma[None])
        g.run(args.k)

    step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    barrier()
    dt = maxtime(time.perf_counter() - t0)
    del Sigma, g
    torch.cuda.empty_cache()
    return {"metric": "greedy sensor placements/sec (independent splits)",
            "value": world * args.k / dt, "unit": "placements/s", "scaling": "weak",
            "config": {"workload": f"one jittered {args.shape} split per rank (seed = rank), "
                                   "dense-exact, no collective", "splits": world}}


def launch_ranks(args):
    """``python bench.py --gpus N`` (N > 1) outside a launcher: start the N ranks ourselves.

    The parent makes no GPU call (torch is not even imported here): it runs
    ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1`` on this
    same command line as a CHILD process (never an exec), streams the children's stdout through —
    rank 0 prints the one JSON line — and returns the launcher's exit status, non-zero if any rank
    failed."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
    print(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd[1:6])}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: rank launcher exited with status {rc}", file=sys.stderr, flush=True)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: the ranks must equal --gpus")
    if args.rank_check:
        print(json.dumps({"rank": rank, "local_rank": local, "n_gpus": world}), flush=True)
        return
    # VGPOSP_BENCH_DEVICE pins every rank to one device (rehearsing N > 1 on a one-GPU box)
    dev = int(os.environ.get("VGPOSP_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.backend)

    from vgposp_amd import _lib, linalg
    from vgposp_amd.placement_algorithm2 import GreedyPlacement
    from vgposp_amd.sharded_placement import HipGreedyBackend, ShardedGreedyPlacement
    from vgposp_amd.workloads import placement_split

    def barrier():
        if world > 1:
            dist.barrier()

    def maxtime(t):
        if world == 1:
            return t
        v = torch.tensor([t], dtype=torch.float64,
                         device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v.item())

    shape = tuple(args.shape)
    # ONE problem on every rank: a jittered grid (seed 0) so the selections are decided by the
    # data, not by the exact octant ties of a regular grid
    X, ls = placement_split(shape, 0)
    N = X.shape[0]
    k = args.k
    Xd = linalg.as_device(X)
    amp_d = linalg.as_device([1.0])
    ls_d = linalg.as_device([ls])
    shift_d = linalg.as_device([args.noise + 1e-6])
    Sigma = torch.empty((N, N), dtype=torch.float64, device="cuda")
    if world == 1:
        g = GreedyPlacement(Sigma, k)  # Sigma is factored in place every step

        def run_rounds():
            g.init()
            for _ in range(k):
                g.step(lazy=True)
        selected = g.selected
    else:
        sh = ShardedGreedyPlacement(HipGreedyBackend(Sigma, k), partition_inverse=True)
        g = sh.b.g

        def run_rounds():
            sh.run(k)
        selected = g.selected

    def step():
        linalg.kernel_matrix(args.kernel, Xd, None, amp_d, ls_d, diag_shift=shift_d, out=Sigma[None])
        run_rounds()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    g.check()
    ref_sel = selected.clone()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = maxtime(time.perf_counter() - t0)
    g.check()
    deterministic = bool(torch.equal(ref_sel, selected))

    # one more step with the library's per-launch event timing on: the roofline numbers
    _lib.prof_enable(True)
    step()
    torch.cuda.synchronize()
    prof = {name: _lib.prof_query(name) for name in
            ["kernel_matrix", "gemm_f64", "potrf_diag", "greedy_colsq", "greedy_trmv", "greedy_update"]}
    # the GEMM launches by layout class (NT / NN / TN, triangular operands, narrow = < 512
    # workgroups): per-flop rates of the step's own shapes
    gemm_classes = {name[len("gemm_f64"):]: {
        "ms_per_step": v[0], "launches": v[1], "tflops": v[2] / (v[0] * 1e-3) / 1e12 if v[0] else None,
        "frac": v[2] / (v[0] * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS if v[0] else None,
        "share_of_gemm_flops": v[2] / prof["gemm_f64"][2] if prof["gemm_f64"][2] else None}
        for name, v in sorted(_lib.prof_dump().items()) if name.startswith("gemm_f64[")}
    _lib.prof_enable(False)
    # exact algorithmic bytes of the triangular mat-vec: rows >= a of the lower triangle of L^-1
    # over this rank's candidate columns (the library only knows the full-triangle upper bound at
    # launch time; a lives on device)
    sel = [int(v) for v in selected.cpu()]
    tri = lambda x: x * (x + 1) / 2.0  # noqa: E731
    trmv_bytes = 8.0 * sum(tri(N) - tri(a) + 2 * N for a in sel[:-1])
    ms_t, n_t, _, _ = prof["greedy_trmv"]
    prof["greedy_trmv"] = (ms_t, n_t, 0.0, trmv_bytes if world == 1 else 0.0)

    # separate plain potrf (N^3/3) for the Cholesky GF/s figure
    chol_gflops = None
    dist_exchanged_gb = None
    if not args.no_potrf:
        linalg.kernel_matrix(args.kernel, Xd, None, amp_d, ls_d, diag_shift=shift_d, lower=True,
                             out=Sigma[None])
        if world == 1:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            linalg.cholesky_(Sigma, invert=False, check=False)
            ev1.record()
            torch.cuda.synchronize()
            chol_gflops = N ** 3 / 3 / (ev0.elapsed_time(ev1) * 1e-3) / 1e9
        else:
            # the distributed factorization the sharded step runs, over all ranks
            from vgposp_amd.dist_cholesky import DistCholesky, greedy_cholesky_ops
            dc = DistCholesky(greedy_cholesky_ops(g))
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dc.factor()
            torch.cuda.synchronize()
            barrier()
            chol_gflops = N ** 3 / 3 / maxtime(time.perf_counter() - t0) / 1e9
            dist_exchanged_gb = 8.0 * dc.exchanged / 1e9
    del Sigma
    torch.cuda.empty_cache()

    c4 = None if args.no_c4 else c4_line(args, world, rank, barrier, maxtime)
    sweep = None if args.no_sweep else grid_sweep(args, world, rank, barrier, maxtime)
    vgp = None
    if not args.no_vgp:
        kw = dict(world=world, rank=rank, barrier=barrier, maxtime=maxtime)
        vgp = {"vgp_c3": vgp_line(args, "c3", **kw), "vgp_c5": vgp_line(args, "c5", **kw)}
        if not args.no_vgp_mixed:  # BASELINE configs[4] as named: the fp32 mixed-precision factor
            vgp["vgp_c5_mixed"] = vgp_line(args, "c5", precision="mixed:2", **kw)
    splits = splits_line(args, world, barrier, maxtime, rank) if world > 1 and not args.no_splits \
        else None

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1e3
    value = k * args.steps / elapsed
    # dominant kernel by time in the profiled step
    dom = max(prof, key=lambda n: prof[n][0])
    ms, launches, flops, nbytes = prof[dom]
    if flops > 0 and dom == "gemm_f64":
        achieved = flops / (ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP64_MFMA_PEAK_TFLOPS, "traffic": None}
    else:
        achieved = nbytes / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None}
    roof.update({"kernel": dom, "launches": launches, "avg_launch_ms": ms / max(launches, 1),
                 "share_of_step": ms / ms_per_step,
                 "measured": "HIP events around every launch on the library's stream, in one extra "
                             "profiled step after the timed loop"})
    tr = load_traffic(args.traffic, dom, N, shape, k)
    if tr is not None and tr.get("stale"):
        roof["traffic_note"] = (f"null: {tr['source']} was measured on kernel sources "
                                f"{tr['recorded_sha256']}, this build is {tr['build_sha256']}")
        tr = None
    if tr is not None:
        roof["traffic"] = tr["bytes_per_launch"]
        roof["traffic_vs_algorithmic"] = tr["bytes_per_launch"] / (nbytes / max(launches, 1))
        roof["traffic_source"] = tr["source"]
    elif dom == "gemm_f64":
        roof["traffic_note"] = (
            "null: no PMC pass of this build in " + os.path.relpath(args.traffic, ROOT) +
            " (tools/step65k.cpp + tools/pmc_traffic.py measure one: DESIGN.md §5)")
    # the HBM-bound kernel of the placement rounds, with its PMC-measured traffic
    ms_t, n_t, _, by_t = prof["greedy_trmv"]
    hbm = {"kernel": "greedy_trmv", "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
           "achieved": by_t / (ms_t * 1e-3) / 1e9 if ms_t and by_t else None, "launches": n_t,
           "avg_launch_ms": ms_t / max(n_t, 1), "traffic": None}
    if hbm["achieved"] is not None:
        hbm["frac"] = hbm["achieved"] / HBM_PEAK_GBS
    trm = load_traffic(args.traffic, "greedy_trmv", N, shape, k)
    if trm is not None and trm.get("stale"):
        hbm["traffic_note"] = (f"null: {trm['source']} was measured on kernel sources "
                               f"{trm['recorded_sha256']}, this build is {trm['build_sha256']}")
        trm = None
    if trm is not None and n_t and by_t:
        hbm["traffic"] = trm["bytes_per_launch"]
        hbm["traffic_vs_algorithmic"] = trm["bytes_per_launch"] / (by_t / n_t)
        hbm["traffic_source"] = trm["source"]
    breakdown = {n: {"ms_per_step": v[0], "launches_per_step": v[1],
                     "achieved": (v[2] / (v[0] * 1e-3) / 1e12 if v[2] and n == "gemm_f64" else
                                  v[3] / max(v[0], 1e-9) / 1e6),
                     "unit": "TFLOP/s" if n == "gemm_f64" else "GB/s"}
                 for n, v in prof.items() if v[1]}
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"{shape[0]}x{shape[1]}x{shape[2]} jittered grid (N={N}), "
                               f"{args.kernel.upper()} kernel amp=1 ls=2h noise={args.noise}+1e-6, "
                               f"k={k} lazy-greedy MI placements, dense-exact, one problem"
                               + (f" candidate-sharded over {world} ranks "
                                  f"({'RCCL' if args.backend == 'nccl' else args.backend}), Cholesky "
                                  "distributed (panel / SYRK shares all-gathered), inverse "
                                  "partitioned" if world > 1 else ""),
                   "N": N, "k": k, "parallelism": f"candidates{world}" if world > 1 else "single",
                   "rccl_world_size": world if world > 1 and args.backend == "nccl" else None,
                   "backend": args.backend if world > 1 else None},
        "cholesky_gflops": chol_gflops,
        "cholesky_note": ("plain single-GPU potrf of the same Sigma" if world == 1 else
                          f"distributed potrf over {world} ranks (max-over-ranks time), "
                          f"{dist_exchanged_gb} GB all-gathered"),
        "roofline": roof,
        "roofline_hbm": hbm,
        "breakdown": breakdown,
        "gemm_classes": gemm_classes,
        "deterministic_selection": deterministic,
        "selected_head": sel[:8],
        "selected": sel,
        # the CPU run of this exact workload (tests/golden/make_golden_65k.py: host LAPACK + the
        # oracle's incremental lazy greedy at N = 65,536), not a GPU self-pin
        "matches_committed_picks": (_committed("bench65k_cpu_picks.json", sel)
                                    if (shape == (64, 32, 32) and k == 50 and args.kernel == "eq"
                                        and args.noise == 1e-2) else None),
    }
    if c4 is not None:
        out["c4"] = c4
    if sweep is not None:
        out["grid_sweep"] = sweep
    if splits is not None:
        out["independent_splits"] = splits
    if vgp is not None:
        out.update(vgp)
    if world == 1 and not args.no_c2:
        out["c2"] = c2_line()
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args, N)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""C4 (128^3, k = 50, beta 4, cutoff 3) end-to-end run time, as bench.py's c4 line measures it:
python tools/c4_time.py [--reps R] [--one-level] [--cheb] [batch ...] -> one JSON line per refinement batch size: mean ms
over R (10) runs, picks vs tests/golden/c4_picks.json, refinements / batches / host reads, and a profiled run's
per-phase event times.  --one-level: one bound level for all candidates (no tightening)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.sparse_placement import ExactTaperPlacement  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
want = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_picks.json")))["picks"]
args = sys.argv[1:]
REPS = 10
if args[:1] == ["--reps"]:
    REPS, args = int(args[1]), args[2:]
ONE = "--one-level" in args  # (the default is two bound levels)
CHEB = "--cheb" in args  # the Chebyshev bounds (K + 1 steps) instead of Gauss-Radau
TARGET = None
if "--target" in args:  # the one-level bracket target (Chebyshev width), e.g. 3e-5 -> K = 3 Radau
    i = args.index("--target")
    TARGET = float(args[i + 1])
    args = args[:i] + args[i + 2:]
PT = LOT = None
if "--pt" in args:  # two levels: candidates pre-tightened before the rounds
    i = args.index("--pt")
    PT = int(args[i + 1])
    args = args[:i] + args[i + 2:]
if "--lo-target" in args:  # two levels: the first level's bracket target (Chebyshev width)
    i = args.index("--lo-target")
    LOT = float(args[i + 1])
    args = args[:i] + args[i + 2:]
args = [a for a in args if a not in ("--one-level", "--two-level", "--cheb")]
X, shape, ls = c4_grid()
run = ExactTaperPlacement(X, shape, 50, 3, 4.0, ls=ls, diag_shift=0.01 + 1e-6, method="bounds")
g = run.greedy
g.two_level = not ONE
g.radau = not CHEB
if TARGET is not None:
    g.bound_target = TARGET
if PT is not None:
    g.pretighten = PT
if LOT is not None:
    g.lo_target = LOT
for B in [int(v) for v in args] or [8]:
    orig = g.run_bounded
    g.run_bounded = lambda q, k, _o=orig, _b=B: _o(q, k, batch=_b)
    run.run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    picks = [int(v) for v in g.picks[:50].cpu()]
    _lib.prof_enable(True)
    run.run()
    torch.cuda.synchronize()
    prof = _lib.prof_dump()
    _lib.prof_enable(False)
    g.run_bounded = orig
    print(json.dumps({"batch": B, "levels": 1 if ONE else 2, "radau": g.radau, "pretighten": g.pretighten, "bound": g.bound, "tight": g.tight,
                      "tightened": g.tightened, "ms_mean": 1e3 * sum(ts) / len(ts), "ms_min": 1e3 * min(ts),
                      "picks_equal": picks == want, "refinements": g.refinements,
                      "batches": g.refine_batches, "host_reads": getattr(g, "host_reads", None),
                      "prof_ms": {k: round(v[0], 3) for k, v in prof.items()},
                      "prof_launches": {k: v[1] for k, v in prof.items()}}), flush=True)

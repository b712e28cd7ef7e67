"""C4 bounded-lazy form, phase timing at 128^3 (or n^3): python tools/bench_bounds.py [n] [k] [K...]
-> one JSON line per bracket width K: bounds ms, rounds ms, refinements, picks == fixture."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.sparse_placement import ExactTaperPlacement, bound_steps  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
Ks = [int(v) for v in sys.argv[3:]] or [0]
BATCH = int(os.environ.get("C4_BATCH", "8"))
X, shape, ls = c4_grid(n)
run = ExactTaperPlacement(X, shape, k, 3, 4.0, ls=ls, diag_shift=0.01 + 1e-6, method="bounds")
g = run.greedy
want = None
fx = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                  "c4_picks.json")
if n == 128 and k == 50:
    want = json.load(open(fx))["picks"]
lo, hi = g.gershgorin(run.qdiag)
for K in Ks:
    steps = bound_steps(run.prob.offs_np, lo, hi, kmax=K) if K else None
    for rep in range(2 if K == 0 or K >= 5 else 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b = g.bound_qdiag(run.qdiag, steps=steps)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        picks = g.run_bounded(run.qdiag, k, batch=BATCH)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    _lib.prof_enable(True)
    g.bound_qdiag(run.qdiag, steps=steps)
    g.run_bounded(run.qdiag, k, batch=BATCH)
    torch.cuda.synchronize()
    prof = _lib.prof_dump()
    _lib.prof_enable(False)
    p = [int(v) for v in picks.cpu()]
    print(json.dumps({"n": n, "k": k, "K": b[0], "width": b[2], "gersh": [lo, hi],
                      "bounds_ms": (t1 - t0) * 1e3, "rounds_ms": (t2 - t1) * 1e3,
                      "total_ms": (t2 - t0) * 1e3, "placements_per_s": k / (t2 - t0),
                      "refinements": g.refinements, "batches": g.refine_batches,
                      "matches_fixture": (p == want) if want else None,
                      "picks_head": p[:6],
                      "prof_ms": {kk: round(v[0], 3) for kk, v in prof.items()}}), flush=True)

"""Time the exact C4 path (vgposp_amd.sparse_placement) phase by phase on one GPU.

python tools/bench_exact.py [n] [k] [leaf]  -> one JSON line: plan time, selected inverse (with the
per-group breakdown from the library's event timing), rounds, CG iterations, picks head."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.sparse_placement import ExactTaperPlacement  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    leaf = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    reps = int(os.environ.get("REPS", "2"))
    X, shape, ls = c4_grid(n)
    t0 = time.perf_counter()
    run = ExactTaperPlacement(X, shape, k, 3, ls=ls, diag_shift=0.01 + 1e-6, leaf=leaf)
    t_setup = time.perf_counter() - t0
    run.run()
    torch.cuda.synchronize()
    run.check()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record()
        run.sel.run(out=run.qdiag)
        ev[1].record()
        picks = run.greedy.run(run.qdiag, k)
        ev[2].record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        r = (wall, ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]))
        best = r if best is None or r[0] < best[0] else best
    evs = []

    def tick(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        evs.append((tag, e))
    run.sel.run(out=run.qdiag, timer=tick)
    torch.cuda.synchronize()
    phases = {}
    for (t0_, e0), (t1_, e1) in zip(evs[:-1], evs[1:]):
        phases[f"{t1_[0]}{run.sel.tree.levels[t1_[1]]['depth']}"] = round(e0.elapsed_time(e1), 3)
    _lib.prof_enable(True)
    run.sel.run(out=run.qdiag)
    run.greedy.run(run.qdiag, k)
    torch.cuda.synchronize()
    prof = _lib.prof_dump()
    _lib.prof_enable(False)
    gemm = _lib.prof_fold(prof).get("gemm_f64", (0, 0, 0, 0))
    out = {"n": n, "N": n ** 3, "k": k, "leaf": leaf, "setup_s": t_setup, "plan_s": run.sel.plan_s,
           "wall_ms": best[0] * 1e3, "selinv_ms": best[1], "rounds_ms": best[2],
           "placements_per_s": k / best[0], "flops_padded": run.sel.flops(),
           "flops_unpadded": run.sel.tree.flops(False),
           "selinv_tflops": run.sel.flops() / (best[1] * 1e-3) / 1e12,
           "gemm_ms": gemm[0], "gemm_launches": gemm[1],
           "gemm_tflops": gemm[2] / (gemm[0] * 1e-3) / 1e12 if gemm[0] else None,
           "cg_iters": run.greedy.cg_iters, "cg_used_last": run.greedy.cg_iterations_used(),
           "picks_head": [int(v) for v in picks[:8].cpu()],
           "prof": {kname: [round(v[0], 3), v[1]] for kname, v in prof.items()},
           "phases_ms": phases, "groups": run.sel.tree.summary()}
    if os.environ.get("PICKS_OUT"):
        with open(os.environ["PICKS_OUT"], "w") as f:
            json.dump({"workload": f"c4_grid({n}) EQ ls 2h noise 1e-2+1e-6 beta 4 cutoff 3",
                       "k": k, "picks": [int(v) for v in picks.cpu()]}, f)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""How many candidates would a truly lazy GPU round have to re-score?

  python tools/lazy_superset.py [--shapes 16,16,32 16,32,32] [--out profiles/r6_lazy_superset.json]

The device rounds keep every candidate's (nom, P_yy) current: one HBM pass over L^-1 per round
(greedy_trmv, 99 ms of the 65k step).  The reference's lazy loop (placement_algorithm2.py:183-208)
re-scores only the entries it pops.  A round that re-scored only those would have to know, before
scoring, a superset of them: every stale entry whose key is >= the final pick's key.  A valid lower
bound of that key is the fresh value of an entry the loop really pops; under submodularity (fresh <=
stale) the fresh value of ANY re-scored entry is one.  This script replays the oracle's lazy loop
(oracle.placement.placement_lazy_incremental on the bench's jittered grid, noise 1e-2 + 1e-6) and
records per round: the loop's own evaluations, the superset sizes for the bound taken from its
first p pops (p = 1, 4, 16), and how many unevaluated entries violate fresh <= stale."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import placement as op  # noqa: E402  (test infrastructure: a CPU analysis)
from vgposp_amd.workloads import placement_split  # noqa: E402

POPS = (1, 4, 16)


def run(shape, k=50):
    rows = []
    orig = op._lazy_select_np

    def lazy_sel(cache, fresh, selected):
        c0 = np.where(selected | np.isnan(cache), -np.inf, cache).copy()
        y, ev = orig(cache, fresh, selected)
        row = {"evals": len(ev)}
        for p in POPS:
            f = max(fresh[e] for e in ev[:p]) if ev else -np.inf
            row[f"superset_p{p}"] = int(np.sum(c0 >= f))
        up = np.zeros(len(cache), dtype=bool)
        up[ev] = True
        nonev = ~up & ~selected & np.isfinite(c0)
        row["fresh_above_stale"] = int(np.sum(fresh[nonev] > c0[nonev] * (1 + 1e-12)))
        rows.append(row)
        return y, ev

    op._lazy_select_np = lazy_sel
    try:
        X, ls = placement_split(shape, 0)
        d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
        S = np.exp(-0.5 * d2 / ls ** 2) + (1e-2 + 1e-6) * np.eye(len(X))
        del d2
        t0 = time.perf_counter()
        op.placement_lazy_incremental(S, k)
        secs = time.perf_counter() - t0
    finally:
        op._lazy_select_np = orig
    later = rows[1:]   # round 0 scores every candidate (cache = +inf)
    keys = list(later[0].keys())
    return {"shape": list(shape), "N": int(np.prod(shape)), "k": k, "seconds": secs,
            "mean": {kk: float(np.mean([r[kk] for r in later])) for kk in keys},
            "max": {kk: int(max(r[kk] for r in later)) for kk in keys},
            "per_round": later}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["16,16,32", "16,32,32"])
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6_lazy_superset.json"))
    a = ap.parse_args()
    out = {"what": __doc__.strip().splitlines()[0], "runs": []}
    for s in a.shapes:
        shape = tuple(int(v) for v in s.split(","))
        r = run(shape)
        print(json.dumps({kk: r[kk] for kk in ("shape", "N", "seconds", "mean", "max")}), flush=True)
        out["runs"].append(r)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

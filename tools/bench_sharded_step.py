"""Per-rank work of the WHOLE sharded 65k placement step (bench.py --gpus R) on ONE GPU, for
R = 1, 2, 4, 8 and every rank r: rank r's distributed Cholesky share (tools/bench_dist_chol.py's
LocalDist: the collectives replaced by the packs / unpacks around them), its slab of L^-1
(vgposp_greedy_finish_slab), and its 50 rounds (column extract, the mat-vec and update over its
own candidate columns, the select), the picks forced to the committed CPU fixture's so every
round's rows are the real ones.  The numbers computed are garbage; the launches, shapes and
bytes are exactly rank r's.  The collectives are only counted (bytes and count per step):

  python tools/bench_sharded_step.py [--out profiles/r6_sharded_step_per_rank.json]

max over ranks of the per-rank time is what R GPUs cannot go below; the driver's SCALE run adds
the RCCL time (25 GB all-gathered in the factorization, three collectives per round)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from bench_dist_chol import LocalDist  # noqa: E402
from vgposp_amd import linalg  # noqa: E402
from vgposp_amd.dist_cholesky import DIST_MIN  # noqa: E402
from vgposp_amd.sharded_placement import HipGreedyBackend, inverse_slabs  # noqa: E402
from vgposp_amd.workloads import placement_split  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", nargs="+", type=int, default=[1, 2, 4, 8])
    ap.add_argument("--dist-min", type=int, default=DIST_MIN,
                    help="smallest node whose panel / SYRK are split over the ranks")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6_sharded_step_per_rank.json"))
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "bench65k_cpu_picks.json")) as f:
        fx = json.load(f)
    shape, k, picks = tuple(fx["shape"]), fx["k"], fx["picks"]
    X, ls = placement_split(shape, 0)
    N = len(X)
    Xd = linalg.as_device(X)
    S = torch.empty((N, N), dtype=torch.float64, device="cuda")
    b = HipGreedyBackend(S, k)
    g = b.g
    forced = torch.tensor(picks, dtype=torch.int64, device="cuda")

    def assemble():
        linalg.kernel_matrix("eq", Xd, None, 1.0, ls, diag_shift=0.01 + 1e-6, lower=False,
                             out=S[None])

    def rounds(c0, c1, partitioned):
        for rnd in range(k):
            if partitioned and rnd > 0:
                b.extract(rnd, c0, c1)
                b.update(rnd, c0, c1, extract=False)
            else:
                b.update(rnd, c0, c1)
            b.select(rnd, True, c0, c1)
            g.selected[rnd:rnd + 1].copy_(forced[rnd:rnd + 1])   # the real pick's rows next round

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    out = {"N": N, "k": k, "dist_min": a.dist_min, "per_R": {}}
    for R in a.ranks:
        ranks = []
        slabs = inverse_slabs(N, R)
        for r in range(R):
            c0, c1 = slabs[r]
            assemble()
            rec = {"rank": r, "slab": [c0, c1]}
            if R == 1:
                rec["factor_and_inverse_s"] = timed(b.init)
                rec["exchanged_GB"] = 0.0
            else:
                b.prepare()
                dc = LocalDist(b.chol_ops(), r, R, a.dist_min)
                rec["factor_s"] = timed(dc.factor)
                rec["inverse_slab_s"] = timed(lambda: b.finish_slab(c0, c1))
                rec["exchanged_GB"] = 8 * dc.exchanged / 1e9
                rec["all_gathers"] = getattr(dc, "n_exchanges", 0)
            rec["rounds_s"] = timed(lambda: rounds(c0, c1, R > 1))
            rec["total_s"] = sum(v for kk, v in rec.items() if kk.endswith("_s"))
            ranks.append(rec)
            print(json.dumps({"R": R, **rec}), flush=True)
        worst = max(x["total_s"] for x in ranks)
        out["per_R"][R] = {
            "ranks": ranks, "max_total_s": worst,
            "placements_per_s_before_collectives": k / worst,
            "collectives_per_step": {
                "factor_allgather_GB": ranks[0]["exchanged_GB"],
                "per_round": "sum all-reduce of the pick's L^-1 column (8 N B), all-gather of the "
                             "delta slabs (8 N B), all-reduce of the pivot row (16 + 16 round B)",
                "rounds_GB": (k - 1) * 2 * 8 * N / 1e9 if R > 1 else 0.0}}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({R: round(v["placements_per_s_before_collectives"], 2)
                      for R, v in out["per_R"].items()}))


if __name__ == "__main__":
    main()

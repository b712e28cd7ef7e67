"""Config C4 at R ranks: does sharding the ROUNDS by candidate slab pay, against the replicated
rounds bench.py runs (verdict r5 item 7)?

  python tools/c4_shard_model.py [--reps 2000] [--out profiles/r6_c4_shard_model.json]

Two measured inputs and the committed 128^3 picks (tests/golden/c4_picks.json):
* where each round's work lands under the bounds pass's slab split (rank r owns candidates
  [r ceil(N/R), (r+1) ceil(N/R)): 128^2 / R ... planes of axis 0): the window re-score of round t
  covers the cube [i - c, i + c) around pick t-1 (snippets_a3.py:196-308, cutoff c = 3: 216
  candidates), the CG column of a refined candidate its Krylov box of half-width 29;
* the latency of the one collective a sharded round adds, a 16-byte (delta, -index) MAX all-reduce
  (snippets_a3.py:143's arg-max across ranks), timed here with 2 gloo ranks.
A sharded round costs max over ranks of (its window share + its slab's arg-max) + the all-reduce.
The round's kernels are latency-bound single-workgroup chains (exact_step 11.3 us, exact_window
10.2 us per round, profiles/r5_c4_kernel_stats_final.txt) whose time does not shrink with the
candidate count, and the window lies in ONE rank's slab in most rounds, so sharding leaves the
per-round chain where it is and adds the collective."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def window_split(picks, n, R, cutoff=3, half_box=29):
    per = -(-n ** 3 // R)
    planes_per_rank = per / (n * n)
    touched_w, touched_cg, share = [], [], []
    for a in picks:
        i0 = a // (n * n)
        lo, hi = max(0, i0 - cutoff), min(n, i0 + cutoff)   # window planes [lo, hi)
        ranks = {int(p // planes_per_rank) for p in range(lo, hi)}
        touched_w.append(len(ranks))
        counts = np.bincount([int(p // planes_per_rank) for p in range(lo, hi)], minlength=R)
        share.append(counts.max() / max(1, counts.sum()))
        blo, bhi = max(0, i0 - half_box), min(n, i0 + half_box + 1)
        touched_cg.append(len({int(p // planes_per_rank) for p in range(blo, bhi)}))
    return {"R": R, "planes_per_rank": planes_per_rank,
            "rounds_window_on_one_rank": int(sum(1 for t in touched_w if t == 1)),
            "rounds": len(picks),
            "mean_ranks_touched_by_window": float(np.mean(touched_w)),
            "mean_max_rank_share_of_window": float(np.mean(share)),
            "mean_ranks_touched_by_cg_box": float(np.mean(touched_cg))}


def _gloo_worker(rank, world, port, reps, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = torch.zeros(2, dtype=torch.float64)
    for _ in range(50):
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(reps):
        x[0] = float(rank + i)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
    dt = (time.perf_counter() - t0) / reps
    if rank == 0:
        q.put(dt)
    dist.destroy_process_group()


def gloo_allreduce_us(reps, world=2, port=29533):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, reps, q)) for r in range(world)]
    for p in ps:
        p.start()
    dt = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
    return dt * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r6_c4_shard_model.json"))
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "c4_picks.json")) as f:
        picks = json.load(f)["picks"]
    split = {R: window_split(picks[:-1], 128, R) for R in (2, 4, 8)}
    ar_us = gloo_allreduce_us(a.reps)
    step_us, window_us = 11.3, 10.2   # profiles/r5_c4_kernel_stats_final.txt, per round
    replicated = step_us + window_us
    out = {"picks": "tests/golden/c4_picks.json (128^3, k = 50)",
           "window_and_cg_split": split,
           "allreduce_16B_us": {"gloo_2_ranks_cpu": ar_us},
           "per_round_us": {"replicated (step + window kernels)": replicated,
                            "sharded, lower bound (the same chain on the window's rank + the "
                            "16-B all-reduce)": {"gloo": replicated + ar_us}},
           "host": {"cpu_count": os.cpu_count(), "python": sys.version.split()[0]}}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""A/B of VGP step settings in ONE process: python tools/vgp_ab.py [--c5] [--mixed] VAR=a,b ...
Each variant sets the environment, builds a fresh training op (new HIP graph) and times 10
graph-replayed steps after 2 warmups; variants interleave over 3 repeats.  One JSON line per run."""
import itertools
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph, vgp_c5_data  # noqa: E402


def main():
    c5 = "--c5" in sys.argv
    mixed = "--mixed" in sys.argv
    specs = [a.split("=", 1) for a in sys.argv[1:] if "=" in a]
    names = [k for k, _ in specs]
    variants = list(itertools.product(*[v.split(",") for _, v in specs]))
    torch.cuda.set_device(0)
    if c5:
        X, y, Z = vgp_c5_data()
        B, kernel = 8192, "matern52"
    else:
        X, y, Z = vgp_c3_data(64, 8)
        B, kernel = 32768, "eq"
    if mixed:
        os.environ["VGPOSP_MIXED_ITERS"] = "2"
    rng = np.random.default_rng(1)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    batches = [torch.as_tensor(rng.integers(0, len(X), B), device="cuda") for _ in range(12)]
    for rep in range(3):
        for var in variants:
            for k, v in zip(names, var):
                os.environ[k] = v
            train_op, _, xb, yb = vgp_c3_graph(X, y, Z, B, precision="mixed" if mixed else "fp64",
                                               kernel=kernel)
            losses = [float(train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]}))
                      for i in range(2)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(2, 12):
                lo = train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]})
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            train_op.check()
            print(json.dumps({"rep": rep, "c5": c5, "mixed": mixed, **dict(zip(names, var)),
                              "ms_per_step": dt * 1e3, "loss0": losses[0],
                              "loss_last": float(lo)}), flush=True)
            del train_op


if __name__ == "__main__":
    main()

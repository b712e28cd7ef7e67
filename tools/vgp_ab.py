"""A/B of VGP step settings in ONE process: python tools/vgp_ab.py [--c5] [--mixed] OPT=a,b ...

OPT is one of
  streams  the step's side-stream bitmask (VGPObjective streams: 1 Kzb, 2 vector chain, 4 VJPs)
  split    the short-K split depth (vgposp_gemm_set_split_depth)
  grouped  1 / 0: one launch per level of M x M products, or one per product
  fused    1 / 0: softplus values + chain rule in the Adam launch, or elementwise launches
Every setting is passed explicitly (constructor arguments, the ABI setter); nothing is read from
or written to the environment.  Each variant builds a fresh training op (new HIP graph) and times
10 graph-replayed steps after 2 warmups; variants interleave over 3 repeats.  One JSON line per
run.  --mixed runs the C5 mixed path with 2 refinement steps ("mixed:2", the bench's)."""
import itertools
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph, vgp_c5_data  # noqa: E402

OPTS = ("streams", "split", "grouped", "fused")


def main():
    c5 = "--c5" in sys.argv
    mixed = "--mixed" in sys.argv
    specs = [a.split("=", 1) for a in sys.argv[1:] if "=" in a]
    for k, _ in specs:
        if k not in OPTS:
            raise SystemExit(f"unknown option {k!r}; expected one of {OPTS}")
    names = [k for k, _ in specs]
    variants = list(itertools.product(*[[int(x) for x in v.split(",")] for _, v in specs]))
    torch.cuda.set_device(0)
    if c5:
        X, y, Z = vgp_c5_data()
        B, kernel = 8192, "matern52"
    else:
        X, y, Z = vgp_c3_data(64, 8)
        B, kernel = 32768, "eq"
    rng = np.random.default_rng(1)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    batches = [torch.as_tensor(rng.integers(0, len(X), B), device="cuda") for _ in range(12)]
    lib = _lib.load()
    for rep in range(3):
        for var in variants:
            o = dict(zip(names, var))
            _lib.call("vgposp_gemm_set_split_depth", o.get("split", 16))
            opts = {}
            if "streams" in o:
                opts["streams"] = o["streams"]
            if "grouped" in o:
                opts["grouped"] = bool(o["grouped"])
            if "fused" in o:
                opts["fused_params"] = bool(o["fused"])
            train_op, _, xb, yb = vgp_c3_graph(X, y, Z, B, precision="mixed:2" if mixed else "fp64",
                                               kernel=kernel, **opts)
            losses = [float(train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]}))
                      for i in range(2)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(2, 12):
                lo = train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]})
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 10
            train_op.check()
            print(json.dumps({"rep": rep, "c5": c5, "mixed": mixed, **o,
                              "split_depth": int(lib.vgposp_gemm_split_depth()),
                              "ms_per_step": dt * 1e3, "loss0": losses[0],
                              "loss_last": float(lo)}), flush=True)
            del train_op
    _lib.call("vgposp_gemm_set_split_depth", 16)


if __name__ == "__main__":
    main()

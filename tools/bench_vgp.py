"""Time the VGP training step on one GPU, with a per-kernel breakdown.

Workload: N = 64^3 observations on a grid over [-7, 7]^3, M = 8^3 inducing points on the
sub-grid (spacing 2 = twice the initial length scale, so the unjittered Kzz the KL term factors
stays well conditioned), EQ kernel with the reference's initial values (softplus(0.54) amp /
noise, 1e-5 + softplus(0.54) ls), minibatch B, Adam(0.01).  One step = optimal posterior over
all N + minibatch variational loss + full analytic gradient + Adam update.
"""
import argparse
import json
import os
import sys

import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vgposp_amd import _lib
from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph, vgp_c5_data


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--c5", action="store_true", help="config C5: 65,536 x 5-D, M = 4^5, B = 8192")
    ap.add_argument("--mixed", action="store_true", help="fp32 Cholesky + fp64 refinement")
    ap.add_argument("--kernel", default="eq")
    ap.add_argument("--mixed-iters", type=int, default=None,
                    help="fp64 refinement steps of the mixed factor (precision 'mixed:<n>')")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    if args.c5:
        X, y, Z = vgp_c5_data()
        args.batch = 8192
    else:
        X, y, Z = vgp_c3_data(args.n, args.m)
    N, B = len(X), args.batch
    train_op, loss, xb, yb = vgp_c3_graph(X, y, Z, B,
                                          precision=("fp64" if not args.mixed else "mixed" if
                                                     args.mixed_iters is None else
                                                     f"mixed:{args.mixed_iters}"),
                                          kernel=args.kernel)
    rng = np.random.default_rng(1)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    batches = [torch.as_tensor(rng.integers(0, N, B), device="cuda")
               for _ in range(args.warmup + args.steps)]
    losses = []
    for i in range(args.warmup):
        losses.append(float(train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]})))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        l_ = train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]})
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    train_op.check()
    losses.append(float(l_))
    # per-kernel breakdown from eager steps with the library's event timing on (no graph)
    _lib.prof_enable(True)
    t1 = time.perf_counter()
    for i in range(args.warmup, args.warmup + args.steps):
        train_op.run({xb: Xd[batches[i]], yb: yd[batches[i]]})
    torch.cuda.synchronize()
    dt_eager = (time.perf_counter() - t1) / args.steps
    prof = {}
    for name in ("kernel_matrix", "gemm_f64", "gemv_f64", "kernel_vjp", "potrf_diag", "gemm_f32",
                 "potrf_diag_f32"):
        ms, launches, flops, nbytes = _lib.prof_query(name)
        if launches:
            prof[name] = {"ms_per_step": ms / args.steps, "launches_per_step": launches / args.steps,
                          "TFLOP/s": flops / (ms * 1e-3) / 1e12 if flops else None,
                          "GB/s": nbytes / (ms * 1e-3) / 1e9}
    _lib.prof_enable(False)
    M = Z.shape[0]
    print(json.dumps({"N": N, "M": M, "batch": B, "kernel": args.kernel, "mixed": args.mixed,
                      "mixed_iters": args.mixed_iters, "losses": losses[:3],
                      "ms_per_step": dt * 1e3, "graph": train_op.graph,
                      "eager_profiled_ms_per_step": dt_eager * 1e3,
                      "elbo_steps_per_s": 1.0 / dt, "loss_first": losses[0], "loss_last": losses[-1],
                      "flops_2M2N_x2": 4.0 * M * M * N, "breakdown": prof}))


if __name__ == "__main__":
    main()

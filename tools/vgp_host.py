"""Is the graph-replayed VGP step bound by the host's node dispatch?  Times g.replay()'s return
(host enqueue of every node) against the following synchronize (GPU done), C3 or C5."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vgposp_amd.workloads import vgp_c3_data, vgp_c3_graph, vgp_c5_data


def main():
    c5 = "--c5" in sys.argv
    torch.cuda.set_device(0)
    X, y, Z = vgp_c5_data() if c5 else vgp_c3_data()
    N = len(X)
    B = N // 8
    train_op, loss, xb, yb = vgp_c3_graph(X, y, Z, B)
    Xd = torch.as_tensor(X, device="cuda")
    yd = torch.as_tensor(y, device="cuda")
    idx = torch.as_tensor(np.random.default_rng(1).integers(0, N, B), device="cuda")
    for _ in range(3):
        train_op.run({xb: Xd[idx], yb: yd[idx]})
    torch.cuda.synchronize()
    g = train_op._g[0]
    host, total = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(t1 - t0)
        total.append(t2 - t0)
    print(f"{'C5' if c5 else 'C3'}: replay host enqueue {1e3 * np.median(host):.3f} ms, "
          f"replay to GPU idle {1e3 * np.median(total):.3f} ms")


if __name__ == "__main__":
    main()

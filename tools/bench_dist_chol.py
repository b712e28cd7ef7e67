"""Per-rank work of the distributed Cholesky (vgposp_amd.dist_cholesky) at N = 65,536 on ONE GPU:
for R = 1, 2, 4, 8 and each rank r, run rank r's share of every node (panel rows, SYRK band,
replicated small blocks) plus the pack / unpack of every all-gather, with the collective itself
replaced by nothing (the other ranks' shares are unpacked from an unfilled buffer, so the numbers
are garbage but the launches and shapes are exactly rank r's).  max over ranks + the measured
all-gather volume / RCCL bandwidth predicts the N-GPU factorization."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vgposp_amd import linalg  # noqa: E402
from vgposp_amd._lib import query  # noqa: E402
from vgposp_amd.dist_cholesky import DistCholesky, HipCholeskyOps  # noqa: E402
from vgposp_amd.workloads import placement_split  # noqa: E402


class LocalDist(DistCholesky):
    def __init__(self, ops, rank, world, dist_min):
        super().__init__(ops, dist_min=dist_min)
        self.rank, self.world = rank, world

    def _exchange(self, pieces, defer=None, depth=0):
        """DistCholesky._exchange without the collective: rank r's pack, the same buffers, and the
        unpack of the (unfilled) receive buffer at the same point — right away, or, for a
        deferred exchange, at the _flush that the real code waits in."""
        ops = self.ops
        sizes = [ops.pack_elems(*p) for p in pieces]
        S = max(sizes)
        if S == 0:
            return
        keys = ("send", "recv") if defer is None else (("dsend", depth), ("drecv", depth))
        send = self._buf(keys[0], S, ops.device)
        recv = self._buf(keys[1], self.world * S, ops.device)
        if sizes[self.rank]:
            ops.pack(*pieces[self.rank], send, False)
        entry = (defer, None, send, recv, None, pieces, sizes, S)
        self.exchanged += sum(sizes)
        self.n_exchanges = getattr(self, "n_exchanges", 0) + 1
        if defer is None:
            self._unpack(entry)
        else:
            self._pending.append(entry)


def main():
    shape = tuple(int(v) for v in (sys.argv[1:4] or (64, 32, 32)))
    dist_min = int(os.environ.get("DIST_MIN", "4096"))
    X, ls = placement_split(shape, 0)
    N = len(X)
    Xd = linalg.as_device(X)
    A = torch.empty((N, N), dtype=torch.float64, device="cuda")
    ws = linalg.workspace(query("vgposp_potrf_workspace_bytes", N))
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    ops = HipCholeskyOps(A, ws.data_ptr(), ws.numel(), info)

    def assemble():
        linalg.kernel_matrix("eq", Xd, None, 1.0, ls, diag_shift=0.01 + 1e-6, lower=True, out=A[None])

    for R in (1, 2, 4, 8):
        times = []
        ex = 0
        for r in range(R):
            assemble()
            dc = LocalDist(ops, r, R, dist_min)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            dc.factor()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            ex = dc.exchanged
        t = max(times)
        print(f"R={R}: per-rank factor+pack (s) {[round(x, 3) for x in times]} -> max {t:.3f} s, "
              f"{N ** 3 / 3 / t / 1e12:.1f} TF/s aggregate before collectives; all-gathered "
              f"{8 * ex / 1e9:.1f} GB", flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic for the round-4 rocprofv3 --pmc SIGSEGV (verdict r4 item 2): run the placement
init (fused Cholesky + inverse, vgposp_greedy_init_ex — the call the crash was inside) at growing
N under the counter pass, with tools/segv_maps.c's handler installed AFTER the GPU runtime and the
profiler tool are up, so that a fault writes its address, PC and /proc/self/maps first.

usage (from the repo root):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/x -o p -- \
      python3 tools/pmc_segv_probe.py gpurun_out/segv_maps.txt 4096 16384 65536
"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

out = sys.argv[1]
sizes = [int(v) for v in sys.argv[2:]] or [4096, 16384, 65536]
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")  # HIP / HSA and the profiler's tool are initialised here
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libsegvmaps.so"))
assert lib.segv_maps_install(os.path.abspath(out).encode()) == 0
from vgposp_amd import linalg  # noqa: E402
from vgposp_amd.placement_algorithm2 import GreedyPlacement  # noqa: E402
from vgposp_amd.workloads import placement_split  # noqa: E402

with open(out + ".maps_at_start", "w") as f:
    f.write(open("/proc/self/maps").read())
for n in sizes:
    shape = {4096: (16, 16, 16), 16384: (32, 32, 16), 32768: (32, 32, 32), 65536: (64, 32, 32)}[n]
    X, ls = placement_split(shape, 0)
    Sigma = torch.empty((n, n), dtype=torch.float64, device="cuda")
    linalg.kernel_matrix("eq", linalg.as_device(X), None, 1.0, ls, diag_shift=0.01 + 1e-6,
                         out=Sigma[None])
    g = GreedyPlacement(Sigma, 4)
    t0 = time.time()
    print(f"N={n}: init ...", flush=True)
    g.init()
    torch.cuda.synchronize()
    g.step(lazy=True)
    torch.cuda.synchronize()
    g.check()
    print(f"N={n}: init + 1 round ok in {time.time() - t0:.1f} s", flush=True)
    del g, Sigma
    torch.cuda.empty_cache()
print("probe done", flush=True)

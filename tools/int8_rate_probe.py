"""How fast is a plain int8 x int8 -> int32 GEMM on this part (torch._int_mm, hipBLASLt)?  The
input to the fp64-emulation estimate of DESIGN.md §8 item 2 (Ozaki scheme II needs ~16 of them
per fp64 product)."""
import json
import time

import torch

out = {}
for n in (4096, 8192, 16384):
    a = torch.randint(-128, 128, (n, n), dtype=torch.int8, device="cuda")
    b = torch.randint(-128, 128, (n, n), dtype=torch.int8, device="cuda")
    for lay, fn in (("nt", lambda: torch._int_mm(a, b.t())), ("nn", lambda: torch._int_mm(a, b))):
        try:
            c = fn()
            torch.cuda.synchronize()
            reps = 20 if n < 16384 else 5
            t = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / reps
            out[f"{lay}_{n}"] = {"ms": dt * 1e3, "tops": 2 * n ** 3 / dt / 1e12}
            if n == 4096 and lay == "nt":   # exactness spot check against an fp64 product
                ref = (a[:256].double() @ b[:256].double().t())
                out["exact_4096_block"] = bool(torch.equal(c[:256, :256].double(), ref))
        except Exception as e:  # noqa: BLE001 (a probe: record what the library refuses)
            out[f"{lay}_{n}"] = {"error": str(e)[:200]}
        print(json.dumps({k: v for k, v in out.items() if str(n) in k}), flush=True)
    del a, b
print(json.dumps(out))

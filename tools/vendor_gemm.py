import torch, time, json, sys
sys.path.insert(0, "/root/repo")
from vgposp_amd import linalg
res = {}
for n in (4096, 8192, 16384):
    a = torch.randn(n, n, dtype=torch.float64, device="cuda"); b = torch.randn(n, n, dtype=torch.float64, device="cuda")
    for name, fn in (("torch", lambda: a @ b.t()), ("vgposp", lambda: linalg.gemm(a, b, transb=True, splitk=False))):
        fn(); torch.cuda.synchronize()
        reps = 5 if n < 16384 else 2
        t = time.perf_counter()
        for _ in range(reps): fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        res[f"{name}_{n}"] = 2 * n**3 / dt / 1e12
print(json.dumps(res))

"""Per-launch HBM traffic from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section):
bytes = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 — FETCH_SIZE / WRITE_SIZE are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads (both the GEMM's
global_load_lds and the mat-vec's loads are such reads).

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv \\
           --N 65536 --shape 64 32 32 --k 50 --out profiles/traffic_r1.json
"""
import argparse
import csv
import json
from collections import defaultdict

CATEGORY = (("gemm_glds_kernel", "gemm_f64"), ("gemm_ref_kernel", "gemm_f64"),
            ("greedy_trmv_kernel<false>", "greedy_trmv"), ("greedy_trmv_kernel<true>", "greedy_colsq"),
            ("kernel_matrix_kernel", "kernel_matrix"), ("potrf_leaf_kernel", "potrf_diag"),
            ("greedy_update_kernel", "greedy_update"))


def category(name):
    for key, cat in CATEGORY:
        if key in name:
            return cat
    return None


def per_dispatch(path, counter):
    vals = defaultdict(float)
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[d] += float(row["Counter_Value"])
            names[d] = row["Kernel_Name"]
    return vals, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--N", type=int, required=True)
    ap.add_argument("--shape", type=int, nargs=3, required=True)
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    fv, fn = per_dispatch(a.fetch_csv, "FETCH_SIZE")
    wv, wn = per_dispatch(a.write_csv, "WRITE_SIZE")
    agg = defaultdict(lambda: [0.0, 0.0, 0])
    for d, name in fn.items():
        cat = category(name)
        if cat:
            agg[cat][0] += fv[d]
            agg[cat][2] += 1
    for d, name in wn.items():
        cat = category(name)
        if cat:
            agg[cat][1] += wv[d]
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vgposp_amd._lib import source_hash
    kernels = {}
    for cat, (fetch, write, n) in agg.items():
        kernels[cat] = {"launches": n, "fetch_kib_per_launch": fetch / n,
                        "write_kib_per_launch": write / n,
                        "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0 / n,
                        "source_sha256": source_hash(cat)}
    out = {"workload": {"N": a.N, "shape": a.shape, "k": a.k}, "command": a.command,
           "formula": "(FETCH_SIZE * 2 + WRITE_SIZE) * 1024 per dispatch, averaged per kernel",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

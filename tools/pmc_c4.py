"""Per-kernel PMC summary of config C4's kernels (rocprofv3 --pmc passes over tools/c4_time.py):
python tools/pmc_c4.py FETCH.csv WRITE.csv HITMISS.csv --runs R --out profiles/pmc_c4_r4.json

Per kernel family (exact_bounds*, exact_cg_a/b, exact_window, exact_rows, exact_step, ...):
launches per run, FETCH_SIZE / WRITE_SIZE bytes per run (KiB x 1024, as reported: these kernels'
8- and 16-byte scattered loads are outside the guide's calibrated 16-B streaming case, so no x2
correction is applied and FETCH is a lower bound), and the L2 hit rate TCC_HIT / (HIT + MISS)."""
import argparse
import csv
import json
import re
from collections import defaultdict


def family(name):
    m = re.match(r"(?:void )?(?:vgposp::)?([A-Za-z_0-9]+)", name.strip())
    return m.group(1) if m else name


def load(path, counters):
    out = defaultdict(lambda: defaultdict(float))
    seen = defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            c = row.get("Counter_Name")
            if c not in counters:
                continue
            fam = family(row["Kernel_Name"])
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            out[fam][c] += float(row["Counter_Value"])
            seen[fam].add(d)
    return out, {k: len(v) for k, v in seen.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("hitmiss")
    ap.add_argument("--runs", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--N", type=int, default=128 ** 3)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    f, nf = load(a.fetch, {"FETCH_SIZE"})
    w, _ = load(a.write, {"WRITE_SIZE"})
    h, _ = load(a.hitmiss, {"TCC_HIT_sum", "TCC_MISS_sum"})
    res = {}
    for fam in sorted(set(f) | set(w) | set(h)):
        if not fam.startswith("exact_") and not fam.startswith("vgposp_") and "exact" not in fam:
            continue
        hit, miss = h[fam]["TCC_HIT_sum"], h[fam]["TCC_MISS_sum"]
        res[fam] = {"launches_per_run": nf.get(fam, 0) / a.runs,
                    "fetch_bytes_per_run": f[fam]["FETCH_SIZE"] * 1024 / a.runs,
                    "write_bytes_per_run": w[fam]["WRITE_SIZE"] * 1024 / a.runs,
                    "l2_hit_rate": hit / (hit + miss) if hit + miss else None}
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from vgposp_amd._lib import source_hash
    json.dump({"runs": a.runs, "workload": {"N": a.N, "k": 50, "beta": 4.0, "cutoff": 3},
               "source_sha256": source_hash("exact"), "command": a.command,
               "note": "bytes = counter KiB x 1024 as reported (no x2: scattered 8 / 16-B loads)",
               "kernels": res}, open(a.out, "w"), indent=1)
    for k, v in res.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()

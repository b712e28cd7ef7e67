"""Dispatch-summed PMC counters per kernel family from rocprofv3 --pmc counter_collection.csv files
(one or more passes of the same command): python tools/pmc_sum.py OUT.json --command "..." CSV...

Per family: dispatches, the counters summed over its dispatches, and derived fractions where the
counters are present — SQ_* wave-cycle shares (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY of
WAVE_CYCLES), instructions per wave-cycle, and SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 4
SIMDs x CUs / 8) (GRBM_GUI_ACTIVE is summed over the 8 XCDs; the MFMA-busy fraction of the
dispatches' GPU-active cycles, as tools/pmc_gemm_step.py)."""
import argparse
import csv
import json
import re
from collections import defaultdict


def family(name):
    m = re.match(r"(?:void )?(?:vgposp::)?([A-Za-z_0-9]+(?:<[^()]*>)?)", name.strip())
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--command", default="")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in a.csv:
        with open(path) as f:
            for row in csv.DictReader(f):
                fam = family(row["Kernel_Name"])
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                tot[fam][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[fam].add((path, d))
    res = {}
    for fam, c in sorted(tot.items()):
        r = {"dispatches": len(disp[fam]) // max(1, len(a.csv)), "counters": dict(c)}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in c:
                    r[k.lower() + "_frac"] = c[k] / wc
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
                if k in c:
                    r[k.lower() + "_per_wave_cycle"] = c[k] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            r["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 4 * a.cus)
        res[fam] = r
    with open(a.out, "w") as f:
        json.dump({"command": a.command, "note": a.note, "kernels": res}, f, indent=1)
    for fam, r in res.items():
        print(fam, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()
                    if k != "counters"})


if __name__ == "__main__":
    main()

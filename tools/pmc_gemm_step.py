"""Summarise tools/pmc_gemm_step.sh: per GEMM instantiation over one 65k step, the MFMA busy
fraction SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1,024 SIMDs) and the wave
fractions SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES,
SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (all dispatch-summed)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void vgposp::", "")
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                n[k].add(r["Dispatch_Id"])
    return acc, n


a, na = load(sys.argv[1])
b, nb = load(sys.argv[2])
print(f"{'instantiation':48s} {'launches':>8s} {'mfma_busy':>9s} {'wait_any':>8s} "
      f"{'wait_inst':>9s} {'active_inst':>11s}")
for k in sorted(a, key=lambda k: -a[k].get("GRBM_GUI_ACTIVE", 0)):
    ca, cb = a[k], b.get(k, {})
    busy = ca.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(ca.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024, 1)
    wc = max(cb.get("SQ_WAVE_CYCLES", 0), 1)
    print(f"{k:48s} {len(na[k]):8d} {busy:9.3f} {cb.get('SQ_WAIT_ANY', 0) / wc:8.3f} "
          f"{cb.get('SQ_WAIT_INST_ANY', 0) / wc:9.3f} {cb.get('SQ_ACTIVE_INST_ANY', 0) / wc:11.3f}")

"""Phase timing inside the C4 per-round kernels (A/B builds with -DVGPOSP_EXACT_DBG=1,
tools/build_exact_variant.sh dbg -DVGPOSP_EXACT_DBG=1; run with
VGPOSP_LIB=$PWD/tools/variants/lib_dbg.so python tools/exact_dbg.py; the library from SRC=../../tools/variants/exact_greedy_dbg.hip tools/build_exact_variant.sh dbg -DVGPOSP_EXACT_DBG=1 [--one-level]).
Prints the mean phase durations (us) of the stall kernel and the step kernel over one 128^3 run:
stall: argmax | top-B | slot staging | slot ranking | batch write;
step: window keys | argmax | slot lookup | pick + key refresh | factor rows;
--dbg2 (a -DVGPOSP_EXACT_DBG=2 build): the step kernel's key refresh instead — window list |
level-2 loads | block keys | superblock keys | arg-max;
--dbg3 (a -DVGPOSP_EXACT_DBG=3 build): the stall kernel's top-B instead — superblock level |
block level | entry level first pass | entry level merge and output;
window (workgroup 0, wave 0, which computes the new LQ row; from the end of the staging): - | new
row | - | wait at the barrier for the candidates' waves | -."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd import _lib  # noqa: E402
from vgposp_amd.sparse_placement import ExactTaperPlacement  # noqa: E402
from vgposp_amd.workloads import c4_grid  # noqa: E402

X, shape, ls = c4_grid()
run = ExactTaperPlacement(X, shape, 50, 3, 4.0, ls=ls, diag_shift=0.01 + 1e-6, method="bounds")
run.greedy.two_level = "--one-level" not in sys.argv
run.run()
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (64 * 8))()
lib.vgposp_exact_dbg(buf)  # reset
out = {}
for kind, name, phases in ((1, "stall", ["sb_level", "blk_level", "entry_pass1", "entry_merge", "_"] if "--dbg3" in sys.argv
                            else ["argmax", "topb", "stage", "rank", "write"]),
                           (2, "step", ["list", "loads", "keys", "superkeys", "argmax"] if "--dbg2" in sys.argv
                            else ["window_keys", "argmax", "slot", "pick_keys", "rows"]),
                           (3, "window", ["_", "new_row", "_", "barrier", "_"])):
    out[name] = {"phases": phases}
run.run()
torch.cuda.synchronize()
lib.vgposp_exact_dbg(buf)
rec = np.frombuffer(buf, dtype=np.uint64).reshape(64, 8).astype(np.int64)
for kind, name in ((1, "stall"), (2, "step"), (3, "window")):
    r = rec[rec[:, 7] == kind]
    if len(r) == 0:
        continue
    d = np.diff(r[:, :6], axis=1) * 0.01  # 100 MHz ticks -> us
    out[name].update({"records": int(len(r)), "mean_us": [round(float(v), 2) for v in d.mean(0)],
                      "total_us": round(float(d.sum(1).mean()), 2)})
print(json.dumps(out), flush=True)

"""Write bench.py's 65k grid (placement_split((64, 32, 32), 0): the jittered grid, seed 0) for
tools/step65k.cpp: int64 n, int64 d, float64 ls, then X [n, d] float64 row-major.  numpy only."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vgposp_amd.workloads import placement_split  # noqa: E402

shape = tuple(int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (64, 32, 32)
X, ls = placement_split(shape, 0)
with open(sys.argv[1], "wb") as f:
    np.asarray(X.shape, dtype=np.int64).tofile(f)
    np.asarray([ls], dtype=np.float64).tofile(f)
    np.ascontiguousarray(X, dtype=np.float64).tofile(f)

"""Loader of the algorithm-3 golden fixtures (tests/golden/alg3_*.npz + alg3_golden.json), made by
tests/golden/make_golden_alg3.py from the REFERENCE's own numpy arithmetic
(placement_algorithm2.nominator / denominator / argmax_cache_linear driven through the window loop
of snippets_a3.py:43-364)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    with open(os.path.join(GOLDEN, "alg3_golden.json")) as f:
        return json.load(f)


def load(name):
    meta = cases()[name]
    z = np.load(os.path.join(GOLDEN, f"alg3_{name}.npz"))
    return meta, {k: z[k] for k in z.files}


NAMES = sorted(cases())

"""Helpers to load the committed golden fixtures (tests/golden/)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def placement_cases():
    with open(os.path.join(GOLDEN, "placement_golden.json")) as f:
        return json.load(f)


def placement_cov(name, entry=None):
    """Rebuild the covariance of a golden case (stored directly when small)."""
    z = np.load(os.path.join(GOLDEN, f"placement_{name}.npz"))
    if "cov" in z.files:
        return z["cov"]
    from oracle import gp as ogp
    p = entry["params"]
    X = z["X"]
    K = ogp.kernel_matrix(p["kind"], X, X, p["amp"], p["ls"])[0]
    return K + (p["noise"] + p["gp_jitter"]) * np.eye(X.shape[0])


def placement_points(name):
    z = np.load(os.path.join(GOLDEN, f"placement_{name}.npz"))
    return z["X"] if "X" in z.files else None

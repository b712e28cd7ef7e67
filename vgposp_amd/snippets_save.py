"""File formats of the reference's placement data, byte-compatible:

* ``cov_vv.csv``: ``pandas.DataFrame(cov_vv).to_csv(path)``, read back with the index column
  dropped (``snippets_save.py:18-31``);
* the selection and the per-round cache CSVs (``main_architecture_2_sampledistribution.py:915-932``),
  also ``DataFrame(...).to_csv``.

Host-side text I/O (pandas); the device arrays are copied to / from the host around it.
"""
from __future__ import annotations

import numpy as np
import pandas as pd


def _host(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def load_cov_vv(file_name="cov_vv.csv"):
    """snippets_save.py:18-24: read_csv, drop the index column -> float64 [N, N]."""
    df = pd.read_csv(file_name, encoding="utf-8", engine="c")
    return np.array(df.iloc[:, 1:])


def save_cov_vv(cov_vv, file_name="cov_vv.csv"):
    """snippets_save.py:27-31."""
    pd.DataFrame(_host(cov_vv)).to_csv(file_name)


def save_selection(selection_idxs, file_name):
    """main_architecture_2_sampledistribution.py:932 (SAVE_SELECTION)."""
    pd.DataFrame(_host(selection_idxs)).to_csv(file_name)


def save_delta_cached_iters(delta_cached_iters, file_name):
    """main_architecture_2_sampledistribution.py:931 (SAVE_CACHE)."""
    pd.DataFrame(_host(delta_cached_iters)).to_csv(file_name)


def save_cov_idxs(xyz_cov_idxs, file_name):
    """main_architecture_2_sampledistribution.py:918 (file_cov_idxs)."""
    pd.DataFrame(_host(xyz_cov_idxs)).to_csv(file_name)


def load_csv_matrix(file_name):
    """Any of the above read back (index column dropped)."""
    return load_cov_vv(file_name)


__all__ = ["load_cov_vv", "save_cov_vv", "save_selection", "save_delta_cached_iters",
           "save_cov_idxs", "load_csv_matrix"]

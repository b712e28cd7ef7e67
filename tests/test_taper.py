"""The beta-decay taper tables of config C4 (vgposp_amd.taper, used by the exact C4 kernels)
against the oracle's and against the dense index taper (main_architecture_2_sampledistribution.py
:375-420)."""
import numpy as np
import pytest

from oracle import taper as lp
from oracle.covariance import index_taper
from vgposp_amd.taper import taper_support


def test_taper_tables_match_reference_decay():
    """decay(beta, d2) is index_taper's g; the support sizes of the betas the C4 tests use."""
    sizes = {4.0: 7, 3.0: 27, 2.5: 33, 2.2: 57}
    for beta, m in sizes.items():
        offs, tau = taper_support(beta)
        assert len(offs) + 1 == m
        o2, t2 = lp.taper_support(beta)
        assert np.array_equal(offs, o2) and np.array_equal(tau, t2)
        C = index_taper(np.ones((125, 125)), (5, 5, 5), beta)
        centre = 62
        nz = np.flatnonzero(C[centre])
        exp = sorted(int(centre + (o[0] * 5 + o[1]) * 5 + o[2]) for o in offs) + [centre]
        assert sorted(nz.tolist()) == sorted(exp)
    with pytest.raises(ValueError):
        taper_support(1.0)


def test_window_is_the_reference_index_window():
    """snippets_a3.py:205-303: [i - c, i + c) per axis, clipped to the grid, C order."""
    shape = (5, 6, 7)
    y = (2 * 6 + 0) * 7 + 6
    w = lp.window(y, shape, 2)
    exp = [(a * 6 + b) * 7 + c for a in range(0, 4) for b in range(0, 2) for c in range(4, 7)]
    assert w.tolist() == exp
    assert lp.window(y, shape, 0).size == 0

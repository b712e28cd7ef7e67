"""Executes the reference-side ctypes stub printed in INTEGRATION.md (the block between the
stub:begin / stub:end markers), so the documented binding is the tested one."""
import os
import re

import pytest

from tests.golden_io import placement_cases, placement_cov

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_namespace():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    m = re.search(r"<!-- stub:begin -->\s*```python\n(.*?)```\s*<!-- stub:end -->", text, re.S)
    assert m, "stub block missing from INTEGRATION.md"
    os.environ.setdefault("VGPOSP_LIB", os.path.join(REPO, "vgposp_amd", "libvgposp.so"))
    ns = {"__name__": "placement_algorithm2_mi355x"}
    exec(compile(m.group(1), "INTEGRATION.md:stub", "exec"), ns)
    return ns


def test_stub_binds_libraries():
    ns = _stub_namespace()
    for name in ("placement_algorithm_1", "placement_algorithm_2"):
        assert callable(ns[name])
    assert ns["_vg"].vgposp_greedy_workspace_bytes(64, 4) > 0
    with pytest.raises(ValueError):
        ns["placement_algorithm_2"]([[1.0, 0.0]], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cov4x4", "grid5", "grid654", "grid5m12"])
def test_stub_matches_golden(name):
    ns = _stub_namespace()
    e = placement_cases()[name]
    cov = placement_cov(name, e)
    assert [int(a) for a in ns["placement_algorithm_2"](cov, e["k"])] == e["alg2"]
    if "alg1" in e:
        assert [int(a) for a in ns["placement_algorithm_1"](cov, e["k"])] == e["alg1"]


@pytest.mark.gpu
def test_stub_singular_cov_retries():
    import numpy as np
    from vgposp_amd.placement_algorithm2 import placement_algorithm_2
    ns = _stub_namespace()
    rng = np.random.default_rng(3)
    X = rng.uniform(-1, 1, (40, 3))
    X[7] = X[3]                                   # duplicated location: rank-deficient kernel
    K = np.exp(-0.5 * ((X[:, None] - X[None]) ** 2).sum(-1) / 0.3 ** 2)
    T = rng.normal(size=(60, 12))                 # 12 samples < 60 locations
    E = np.cov(T)
    for cov in (K, E):
        want = [int(a) for a in placement_algorithm_2(cov, 6)]
        assert [int(a) for a in ns["placement_algorithm_2"](cov, 6)] == want

"""GPU: config C4's algorithm 3 against fixtures produced by the REFERENCE's own arithmetic
(tests/golden/make_golden_alg3.py: placement_algorithm2.nominator / denominator / argmax_cache_linear
through the window loop of snippets_a3.py:43-364, on tapered 5^3..7^3 grids, beta 4 and 2.5,
cutoffs 1-3, EQ / Matern kernels).

* tapered_placement_algorithm_3, the C4 boundary, in both exact forms: the multifrontal selected
  inverse (picks, pick deltas, every delta_cached_iters column) and the bounded-lazy rounds (picks
  and pick deltas; beta = 4 only, where the Gershgorin bracket holds);
* the dense algorithm-3 engine (snippets_a3.sparse_placement_algorithm_3 over the fixture's
  cov_vv itself)."""
import numpy as np
import pytest

from golden_alg3 import NAMES, load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", NAMES)
def test_selected_inverse_matches_reference_arithmetic(name):
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    m, z = load(name)
    A, deltas, dci = tapered_placement_algorithm_3(
        z["X"], m["k"], m["shape"], m["cutoff"], m["beta"], kernel=m["kernel"], ls=m["ls"],
        diag_shift=m["diag_shift"], snapshots=True, leaf=32, method="selinv")
    assert [int(a) for a in A] == [int(a) for a in z["order"]]
    np.testing.assert_allclose(deltas, m["pick_deltas"], rtol=1e-10)
    np.testing.assert_allclose(dci, z["dci"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name", [n for n in NAMES if load(n)[0]["beta"] >= 4.0])
def test_bounded_lazy_matches_reference_arithmetic(name):
    from vgposp_amd.sparse_placement import tapered_placement_algorithm_3
    m, z = load(name)
    A, deltas, _ = tapered_placement_algorithm_3(
        z["X"], m["k"], m["shape"], m["cutoff"], m["beta"], kernel=m["kernel"], ls=m["ls"],
        diag_shift=m["diag_shift"], method="bounds")
    assert [int(a) for a in A] == [int(a) for a in z["order"]]
    np.testing.assert_allclose(deltas, m["pick_deltas"], rtol=1e-10)


@pytest.mark.parametrize("name", NAMES)
def test_dense_engine_matches_reference_arithmetic(name):
    from vgposp_amd.snippets_a3 import placement_algorithm_3, sparse_placement_algorithm_3
    m, z = load(name)
    Aset, cache, dci = sparse_placement_algorithm_3(z["cov"], m["k"], m["shape"], m["cutoff"])
    assert sorted(int(a) for a in Aset.values) == sorted(int(a) for a in z["order"])
    order = placement_algorithm_3(z["cov"], m["k"], m["shape"], m["cutoff"])
    assert [int(a) for a in order] == [int(a) for a in z["order"]]
    np.testing.assert_allclose(dci, z["dci"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(cache.reshape(-1), z["cache"], rtol=1e-9, atol=1e-12)

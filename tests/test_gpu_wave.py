"""GPU: the library's cross-lane wave reductions (csrc/common.h — DPP row rotates / quad perms and
v_permlane32/16_swap; the key arg-max on an order-preserving integer encoding) return bit for bit
what the __shfl_xor / key_gt butterflies they replaced returned,
on values chosen to make the summation order visible (mixed magnitudes and signs), ties in the key
arg-max, NaN keys and missing (-1) indices.  The checker kernel is tests/hip/wave_check.hip."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libwavecheck.so")


def test_wave_reductions_bit_identical_to_shuffle_butterfly():
    import torch
    torch.cuda.set_device(0)
    assert os.path.exists(LIB), "tests/_build/libwavecheck.so: run __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)
    rng = np.random.default_rng(7)
    nw = 512
    x = rng.standard_normal(nw * 64) * np.exp(rng.uniform(-30, 30, nw * 64))
    x[: 64 * 8] = np.round(x[: 64 * 8], 0) % 3          # many ties in the first waves
    x[64 * 8: 64 * 9: 7] = np.nan                        # NaN keys rank below every number
    idx = rng.permutation(nw * 64).astype(np.int64)
    idx[64 * 10: 64 * 11: 3] = -1                        # no candidate
    idx[64 * 11: 64 * 12] = -1                           # a wave with none at all
    out = np.zeros(nw * 64 * 8)
    rc = lib.wave_check(x.ctypes.data_as(ctypes.c_void_p), idx.ctypes.data_as(ctypes.c_void_p),
                        ctypes.c_int(nw), out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    o = out.reshape(nw, 64, 8)
    bits = o.view(np.uint64)
    for new, old in ((0, 1), (2, 3), (4, 5), (6, 7)):
        same = bits[..., new] == bits[..., old]
        # a NaN is NaN either way (its payload bits are not compared); the key arg-max returns
        # -0.0 as +0.0 (key_gt ranks them equal)
        same |= np.isnan(o[..., new]) & np.isnan(o[..., old])
        if new == 4:
            same |= o[..., 4] == o[..., 5]
            same |= o[..., 7].view(np.int64) < 0  # no candidate: the value carries nothing
        bad = np.argwhere(~same)
        assert bad.size == 0, (new, bad[:8].tolist(), o[tuple(bad[0])][[new, old]])
    # and the values are the reductions (every lane holds the same result)
    finite = ~np.isnan(x.reshape(nw, 64)).any(1)
    xs = x.reshape(nw, 64)[finite]
    assert (np.abs(o[finite, 0, 0] - xs.sum(1)) <= 1e-13 * np.abs(xs).sum(1)).all()
    assert (o[..., 6].view(np.int64) == o[:, :1, 6].view(np.int64)).all()

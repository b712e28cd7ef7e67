"""C-ABI boundary checks that run without a GPU: the library loads and exports every symbol the
header declares; host-only queries answer; argument validation reports the bad argument."""
import ctypes

import pytest

from vgposp_amd import _lib


def test_library_exports_header_symbols():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"


def test_abi_version():
    assert _lib.load().vgposp_abi_version() == _lib.ABI_VERSION


def test_workspace_queries():
    # leaf inverses (ceil(n/128) x 128^2) + the trtri scratch of the top split (n1 x n2)
    assert _lib.query("vgposp_potrf_workspace_bytes", 1000) >= (8 * 128 * 128 + 512 * 488) * 8
    assert _lib.query("vgposp_potrf_workspace_bytes", 0) == 0
    n, k = 65536, 50
    ws = _lib.query("vgposp_greedy_workspace_bytes", n, k)
    fact = _lib.query("vgposp_potrf_workspace_bytes", n)
    assert ws >= 2 * k * n * 8 + fact  # W and V rows + factorization scratch
    assert ws < 16 * n * 8 + 2 * k * n * 8 + (n // 512 + 1) * n * 8 + fact + 2 ** 22
    assert _lib.query("vgposp_greedy_workspace_bytes", 0, 5) == 0
    assert _lib.query("vgposp_lml_workspace_bytes", 100, 2) == 1600


def test_argument_validation_without_gpu():
    # invalid kernel kind is rejected before any device work
    with pytest.raises(_lib.VgpospError, match="bad argument 1"):
        _lib.call("vgposp_kernel_matrix", 9, None, 1, None, 1, 3, None, None, None, 1, 0, None, 1, 0, None)
    with pytest.raises(_lib.VgpospError, match="bad argument 6"):
        _lib.call("vgposp_kernel_matrix", 0, ctypes.c_void_p(8), 1, ctypes.c_void_p(8), 1, 9,
                  ctypes.c_void_p(8), ctypes.c_void_p(8), None, 1, 0, ctypes.c_void_p(8), 1, 0, None)
    with pytest.raises(_lib.VgpospError, match="bad argument 4"):
        _lib.call("vgposp_greedy_init", ctypes.c_void_p(8), 10, 10, 11, ctypes.c_void_p(8),
                  ctypes.c_void_p(8), 1 << 20, None)

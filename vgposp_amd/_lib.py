"""ctypes binding of libvgposp.so (the C-ABI declared in include/vgposp.h).

The library is built in-tree by ``__graft_entry__.build()`` (``make -C vgposp_amd/csrc``).  There
is no fallback: if the shared object is missing or cannot be loaded, every entry point raises
``VgpospUnavailable`` — the product path never silently degrades to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VGPOSP_LIB", os.path.join(_HERE, "libvgposp.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "vgposp.h")

ABI_VERSION = 2
E_HIP = -100
E_WS = -101

KERNEL_KINDS = {"eq": 0, "matern12": 1, "matern32": 2, "matern52": 3}
FULL, LOWER = 0, 1


class VgpospError(RuntimeError):
    """A libvgposp entry point returned a non-zero status."""


class VgpospUnavailable(VgpospError):
    """libvgposp.so is missing or failed to load (build it with __graft_entry__.build())."""


class CholeskyError(VgpospError):
    """Mirror of TF's InvalidArgumentError 'Cholesky decomposition was not successful.'"""

    def __init__(self, info, batch_index=0):
        super().__init__(
            "Cholesky decomposition was not successful. The input might not be valid. "
            f"(leading minor of order {info} is not positive definite, batch {batch_index})")
        self.info = int(info)
        self.batch_index = int(batch_index)


_c_void_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f64 = ctypes.c_double
_size = ctypes.c_size_t

# the common leading arguments of vgposp_exact_prepare / vgposp_exact_round
_EXACT = [_i32, _c_void_p, _i64, _i64, _i64, _f64, _f64, _f64, _f64, _f64, _c_void_p, _i32,
          _c_void_p, _i32, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
          _size]

# name -> (restype, argtypes)
SIGNATURES = {
    "vgposp_abi_version": (_i32, []),
    "vgposp_last_error": (ctypes.c_char_p, []),
    "vgposp_kernel_matrix": (_i32, [_i32, _c_void_p, _i64, _c_void_p, _i64, _i32, _c_void_p,
                                    _c_void_p, _c_void_p, _i32, _i32, _c_void_p, _i64, _i64,
                                    _c_void_p]),
    "vgposp_gemm": (_i32, [_i32, _i32, _i64, _i64, _i64, _f64, _c_void_p, _i64, _c_void_p, _i64,
                           _f64, _c_void_p, _i64, _i32, _i32, _i32, _c_void_p]),
    "vgposp_gemm_set_split_depth": (_i32, [_i32]),
    "vgposp_gemm_split_depth": (_i32, []),
    "vgposp_gemm_splitk_workspace_bytes": (_size, [_i64, _i64, _i64, _i32, _i32]),
    "vgposp_gemm_batched_workspace_bytes": (_size, [_i64, _i64, _i64, _i32, _i32]),
    "vgposp_gemm_batched": (_i32, [_i32, _i32, _i64, _i64, _i64, _f64, _c_void_p, _i64, _i64,
                                   _c_void_p, _i64, _i64, _f64, _c_void_p, _i64, _i64, _i32, _i32,
                                   _i32, _i32, _c_void_p, _size, _c_void_p]),
    "vgposp_gemm_splitk": (_i32, [_i32, _i32, _i64, _i64, _i64, _f64, _c_void_p, _i64, _c_void_p,
                                  _i64, _f64, _c_void_p, _i64, _i32, _i32, _i32, _i32, _c_void_p,
                                  _size, _c_void_p]),
    "vgposp_kernel_matrix_matvec_workspace_bytes": (_size, [_i64, _i64]),
    "vgposp_kernel_matrix_matvec": (_i32, [_i32, _c_void_p, _i64, _c_void_p, _i64, _i32,
                                           _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                                           _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_vgp_sinv": (_i32, [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _f64, _f64, _c_void_p,
                               _i32, _c_void_p]),
    "vgposp_sym_from_lower": (_i32, [_c_void_p, _i64, _i64, _c_void_p]),
    "vgposp_lincomb": (_i32, [_i64, _i64, _i64, _i32, _c_void_p, _c_void_p, _c_void_p, _f64, _f64,
                              _i32, _c_void_p, _f64, _c_void_p, _c_void_p]),
    "vgposp_vgp_kzz_bar": (_i32, [_i64, _c_void_p, _c_void_p, _c_void_p, _f64, _c_void_p,
                                  _c_void_p, _c_void_p]),
    "vgposp_dots_workspace_bytes": (_size, [_i32]),
    "vgposp_dots": (_i32, [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                           _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_vgp_scalars": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                  _c_void_p, _f64, _f64, _f64, _f64, _c_void_p, _c_void_p]),
    "vgposp_kernel_vjp_workspace_bytes": (_size, [_i64, _i64, _i32]),
    "vgposp_kernel_vjp": (_i32, [_i32, _c_void_p, _i64, _c_void_p, _i64, _i32, _c_void_p,
                                 _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _c_void_p,
                                 _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_kernel_matvec": (_i32, [_i32, _c_void_p, _i64, _c_void_p, _i64, _i32, _c_void_p,
                                    _c_void_p, _c_void_p, _f64, _c_void_p, _c_void_p]),
    "vgposp_center_rows": (_i32, [_c_void_p, _i64, _i64, _i64, _f64, _c_void_p]),
    "vgposp_index_taper": (_i32, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _f64, _f64, _i32,
                                  _c_void_p]),
    "vgposp_potrf_batched_workspace_bytes": (_size, [_i64, _i32]),
    "vgposp_potrf_workspace_bytes": (_size, [_i64]),
    "vgposp_potrf_lower": (_i32, [_c_void_p, _i64, _i64, _i64, _i32, _i32, _c_void_p, _c_void_p,
                                  _c_void_p, _size, _c_void_p]),
    "vgposp_trsm_workspace_bytes": (_size, [_i64, _i64]),
    "vgposp_trsm_lower": (_i32, [_c_void_p, _i64, _i64, _i32, _c_void_p, _i64, _i64, _c_void_p,
                                 _size, _c_void_p]),
    "vgposp_lml_workspace_bytes": (_size, [_i64, _i32]),
    "vgposp_lml": (_i32, [_c_void_p, _i64, _i64, _i64, _i32, _c_void_p, _c_void_p, _c_void_p,
                          _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_lml_grad_workspace_bytes": (_size, [_i64, _i32]),
    "vgposp_lml_grad": (_i32, [_i32, _c_void_p, _i64, _i32, _c_void_p, _c_void_p, _c_void_p, _i64,
                               _i64, _c_void_p, _i32, _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_workspace_bytes": (_size, [_i64, _i32]),
    "vgposp_greedy_init": (_i32, [_c_void_p, _i64, _i64, _i32, _c_void_p, _c_void_p, _size,
                                  _c_void_p]),
    "vgposp_greedy_init_ex": (_i32, [_c_void_p, _i64, _i64, _i32, _f64, _f64, _f64, _c_void_p,
                                     _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_cache": (_i32, [_c_void_p, _i64, _i32, ctypes.POINTER(_c_void_p)]),
    "vgposp_greedy_exclude": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p]),
    "vgposp_greedy_select_window": (_i32, [_i64, _i32, _i32, _i64, _i64, _i64, _i32, _i64, _i64,
                                           _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size,
                                           _c_void_p]),
    "vgposp_front_factor_workspace_bytes": (_size, [_i64, _i64, _i32]),
    "vgposp_front_assemble": (_i32, [_i32, _c_void_p, _i64, _i64, _i64, _f64, _f64, _f64, _f64,
                                     _c_void_p, _i32, _c_void_p, _i32, _c_void_p, _c_void_p,
                                     _c_void_p, _i64, _c_void_p, _i64, _c_void_p, _c_void_p, _i32,
                                     _c_void_p, _c_void_p, _c_void_p]),
    "vgposp_front_extend_add": (_i32, [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _c_void_p,
                                       _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p,
                                       _c_void_p]),
    "vgposp_front_factor": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i32, _c_void_p,
                                   _c_void_p, _size, _c_void_p]),
    "vgposp_front_gather": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                   _c_void_p, _i32, _i64, _c_void_p, _c_void_p]),
    "vgposp_front_selinv": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _i64, _i32, _c_void_p,
                                   _c_void_p, _c_void_p]),
    "vgposp_front_diag": (_i32, [_c_void_p, _i64, _i32, _c_void_p, _c_void_p, _c_void_p]),
    "vgposp_exact_workspace_bytes": (_size, [_i64, _i64, _i64, _i32, _i32, _i32, _i32]),
    "vgposp_exact_prepare": (_i32, _EXACT + [_i32, _c_void_p]),
    "vgposp_exact_round": (_i32, _EXACT + [_i32, _i32, _c_void_p, _c_void_p, _f64, _c_void_p]),
    "vgposp_exact_coef": (_i32, _EXACT + [_c_void_p]),
    "vgposp_exact_bounds": (_i32, _EXACT + [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _f64,
                                            _f64, _i64, _i64, _c_void_p]),
    "vgposp_exact_steps_reset": (_i32, _EXACT + [_c_void_p]),
    "vgposp_exact_steps": (_i32, _EXACT + [_i32, _i32, _i32, _i32, _c_void_p, _c_void_p,
                                           _c_void_p]),
    "vgposp_exact_refine_pending": (_i32, _EXACT + [_i32, _c_void_p, _f64, _c_void_p]),
    "vgposp_exact_tighten_pending": (_i32, _EXACT + [_c_void_p, _c_void_p, _c_void_p, _i32, _i32,
                                                     _f64, _f64, _c_void_p, _c_void_p]),
    "vgposp_exact_pretighten": (_i32, _EXACT + [_c_void_p, _c_void_p, _c_void_p, _i32, _i32,
                                                _f64, _f64, _i64, _c_void_p]),
    "vgposp_exact_ctl": (_i32, [_c_void_p, _i64, _i64, _i64, _i32, _i32, _i32, _i32,
                                ctypes.POINTER(_c_void_p)]),
    "vgposp_exact_update": (_i32, _EXACT + [_i32, _c_void_p, _c_void_p]),
    "vgposp_exact_buffers": (_i32, [_c_void_p, _i64, _i64, _i64, _i32, _i32, _i32, _i32]
                             + [ctypes.POINTER(_c_void_p)] * 6),
    "vgposp_adam_update": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f64, _f64,
                                  _f64, _f64, _c_void_p, _f64, _c_void_p]),
    "vgposp_softplus_values": (_i32, [_c_void_p, _i64, _i32, ctypes.POINTER(_i32),
                                      ctypes.POINTER(_f64), _c_void_p, _c_void_p]),
    "vgposp_adam_update_softplus": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f64,
                                           _f64, _f64, _f64, _c_void_p, _f64, _i32,
                                           ctypes.POINTER(_i32), ctypes.POINTER(_c_void_p),
                                           _c_void_p]),
    "vgposp_gemm_group_workspace_bytes": (_size, [_i32, ctypes.POINTER(_i32),
                                                 ctypes.POINTER(_i64)]),
    "vgposp_gemm_group": (_i32, [_i32, ctypes.POINTER(_i32), ctypes.POINTER(_i64),
                                 ctypes.POINTER(_f64), ctypes.POINTER(_f64),
                                 ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64),
                                 ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64),
                                 ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64), _c_void_p,
                                 _size, _c_void_p]),
    "vgposp_prof_enable": (_i32, [_i32]),
    "vgposp_prof_dump": (_i64, [ctypes.c_char_p, _size]),
    "vgposp_prof_query": (_i32, [ctypes.c_char_p, ctypes.POINTER(_f64), ctypes.POINTER(_i64),
                                 ctypes.POINTER(_f64), ctypes.POINTER(_f64)]),
    "vgposp_greedy_update": (_i32, [_c_void_p, _i64, _i64, _i32, _i32, _i64, _i64, _c_void_p,
                                    _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_select": (_i32, [_i64, _i32, _i32, _i32, _i64, _i64, _c_void_p, _c_void_p,
                                    _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_slab_tmp_bytes": (_size, [_i64, _i64, _i64]),
    "vgposp_greedy_init_slab": (_i32, [_c_void_p, _i64, _i64, _i32, _f64, _f64, _f64, _i64, _i64,
                                       _c_void_p, _size, _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_extract": (_i32, [_c_void_p, _i64, _i64, _i32, _i32, _i64, _i64, _c_void_p,
                                     _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_update_ex": (_i32, [_c_void_p, _i64, _i64, _i32, _i32, _i64, _i64, _c_void_p,
                                       _i32, _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_prepare": (_i32, [_c_void_p, _i64, _i64, _i32, _f64, _f64, _f64, _c_void_p,
                                     _c_void_p, _size, _c_void_p]),
    "vgposp_greedy_fact_ws": (_i32, [_c_void_p, _i64, _i32, ctypes.POINTER(_c_void_p),
                                     ctypes.POINTER(_size)]),
    "vgposp_greedy_finish_slab": (_i32, [_c_void_p, _i64, _i64, _i32, _i64, _i64, _c_void_p,
                                         _size, _c_void_p, _size, _c_void_p]),
    "vgposp_potrf_mixed_workspace_bytes": (_size, [_i64]),
    "vgposp_potrf_mixed": (_i32, [_c_void_p, _i64, _i64, _c_void_p, _i64, _c_void_p, _i32,
                                  _c_void_p, _c_void_p, _c_void_p, _size, _c_void_p]),
    "vgposp_potrf_split": (_i64, [_i64]),
    "vgposp_potrf_block": (_i32, [_c_void_p, _i64, _i64, _i64, _i64, _c_void_p, _c_void_p, _size,
                                  _c_void_p]),
    "vgposp_potrf_panel": (_i32, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _i64, _c_void_p, _size,
                                  _c_void_p]),
    "vgposp_potrf_trailing": (_i32, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _i64, _c_void_p,
                                     _size, _c_void_p]),
    "vgposp_pack_elems": (_i64, [_i64, _i64, _i64, _i64, _i32]),
    "vgposp_pack_rows": (_i32, [_c_void_p, _i64, _i64, _i64, _i64, _i64, _i32, _c_void_p, _i32,
                                _c_void_p]),
    "vgposp_greedy_xcol": (_i32, [_c_void_p, _i64, _i32, ctypes.POINTER(_c_void_p)]),
    "vgposp_greedy_buffers": (_i32, [_c_void_p, _i64, _i32, ctypes.POINTER(_c_void_p),
                                     ctypes.POINTER(_c_void_p), ctypes.POINTER(_i64)]),
    "vgposp_greedy_step": (_i32, [_c_void_p, _i64, _i64, _i32, _i32, _i32, _c_void_p, _c_void_p,
                                  _c_void_p, _c_void_p, _size, _c_void_p]),
}

_lock = threading.Lock()
_lib = None


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/vgposp.h."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(vgposp_[a-z0-9_]+)\s*\(", text)))


def load():
    """Load libvgposp.so once (raises VgpospUnavailable if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise VgpospUnavailable(
                f"{LIB_PATH} not found: build the HIP library first (python -c "
                "'import __graft_entry__ as g; g.build()')")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover
            raise VgpospUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.vgposp_abi_version()
        if v != ABI_VERSION:
            raise VgpospUnavailable(f"libvgposp ABI {v} != expected {ABI_VERSION}")
        _lib = lib
        return lib


def last_error():
    return load().vgposp_last_error().decode(errors="replace")


def call(name, *args):
    """Call an int-returning entry point; raise VgpospError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise VgpospError(f"{name} failed (rc={rc}): {last_error()}")
    return rc


def query(name, *args):
    """Call a size-returning query (workspace sizes)."""
    return int(getattr(load(), name)(*args))


# source files whose compiled code each profiled kernel family runs (for matching PMC traffic
# records to the build they were measured on)
KERNEL_SOURCES = {
    "gemm_f64": ["gemm.hip", "common.h", "Makefile"],
    "greedy_trmv": ["greedy.hip", "common.h", "Makefile"],
    "greedy_colsq": ["greedy.hip", "common.h", "Makefile"],
    "kernel_matrix": ["kernel_matrix.hip", "psd.h", "common.h", "Makefile"],
    "exact": ["exact_greedy.hip", "psd.h", "common.h", "Makefile"],
}


def source_hash(kernel):
    """sha256 (16 hex digits) of the sources a kernel family is compiled from."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES.get(kernel, []):
        with open(os.path.join(_HERE, "csrc", name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


_prof_state = [False]


def prof_enable(on=True):
    call("vgposp_prof_enable", int(on))
    _prof_state[0] = bool(on)


def prof_on():
    """Whether the library's per-launch event timing is on (set through prof_enable)."""
    return _prof_state[0]


def prof_query(name):
    """(total_ms, launches, algorithmic_flops, algorithmic_bytes) of a kernel since prof_enable."""
    ms, n, fl, by = _f64(), _i64(), _f64(), _f64()
    call("vgposp_prof_query", name.encode(), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl),
         ctypes.byref(by))
    return ms.value, n.value, fl.value, by.value


def prof_fold(dump):
    """Fold the per-class entries of a prof_dump ("gemm_f64[nt,triA]" ...) into their family
    ("gemm_f64"): {family: (ms, launches, flops, bytes)}."""
    out = {}
    for name, v in dump.items():
        fam = name.split("[", 1)[0]
        a = out.get(fam, (0.0, 0, 0.0, 0.0))
        out[fam] = tuple(x + y for x, y in zip(a, v))
    return out


def prof_dump():
    """{name: (ms, launches, flops, bytes)} of everything recorded since prof_enable."""
    fn = load().vgposp_prof_dump
    need = fn(None, 0)
    if need < 0:
        raise VgpospError(last_error())
    buf = ctypes.create_string_buffer(int(need))
    fn(buf, need)
    out = {}
    for line in buf.value.decode().splitlines():
        name, ms, n, fl, by = line.split("\t")
        out[name] = (float(ms), int(n), float(fl), float(by))
    return out

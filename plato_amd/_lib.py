"""ctypes binding of ``libplato_agg.so`` (the C ABI in ``include/plato_agg.h``).

The library is the only compute path of this package: there is no CPU or
PyTorch fallback.  If the shared object is missing or fails to load,
:func:`lib` raises ``RuntimeError`` with the build command to run.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libplato_agg.so")
TUNE_LIB_PATH = os.path.join(_HERE, "libplato_agg_tune.so")
ABI_VERSION = 4

PLATO_AGG_OK = 0
PLATO_AGG_EINVAL = -1
PLATO_AGG_EHIP = -2
PLATO_AGG_ERCCL = -3
PLATO_AGG_ADD_BASE = 1
PLATO_AGG_FLAT_DELTA = 0
PLATO_AGG_FLAT_CAST_DIFF = 1
PLATO_AGG_FLAT_RAW = 2
PLATO_AGG_PORT_CAST_FIRST = 1
PLATO_AGG_SEG_NEG_DIV = 1
PLATO_AGG_FEDADP_TABLES_READY = 1
PLATO_AGG_DECODE = {"native": 0, "bf16": 1, "qsgd": 2}

_c_void_p = ctypes.c_void_p
_c_size_t = ctypes.c_size_t
_c_int = ctypes.c_int
_c_float = ctypes.c_float
_c_u64 = ctypes.c_uint64

# name -> (restype, argtypes); must match include/plato_agg.h exactly (tests/test_abi.py
# checks the export list of libplato_agg.so against it).
SIGNATURES = {
    "plato_agg_abi_version": (_c_int, []),
    "plato_agg_last_error": (ctypes.c_char_p, []),
    "plato_agg_fedavg_weights": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
         _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_fedavg_weights_bf16": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
         _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_fedavg_deltas": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_compute_deltas": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_update_weights": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_cast_f32_i64": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "plato_agg_mix_weights": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_float, _c_float,
         _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_fill_synth_f32": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_u64, _c_u64, _c_int, _c_void_p]
    ),
    "plato_agg_fill_synth_i64": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_u64, _c_u64, _c_u64, _c_void_p]
    ),
    "plato_agg_fill_synth_f32_at": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_u64, _c_u64, _c_u64, _c_int, _c_void_p]
    ),
    "plato_agg_fill_synth_i64_at": (
        _c_int, [_c_void_p, _c_void_p, _c_size_t, _c_u64, _c_u64, _c_u64, _c_u64, _c_void_p]
    ),
    "plato_agg_client_dots_workspace": (_c_size_t, [_c_int, _c_size_t]),
    "plato_agg_client_dots": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_size_t,
         _c_void_p, _c_void_p, _c_void_p],
    ),
    "plato_agg_entry_stats_workspace": (_c_size_t, [_c_int, ctypes.c_uint32]),
    "plato_agg_entry_stats": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_void_p, ctypes.c_uint32, _c_void_p, ctypes.c_uint32, _c_int, _c_size_t, _c_size_t,
         _c_void_p, _c_void_p, _c_void_p],
    ),
    "plato_agg_fedavg_entrywise": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_int, _c_void_p, ctypes.c_uint32, _c_void_p,
         ctypes.c_uint32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_float, _c_float, _c_int,
         _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_entry_norms_f32": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_void_p,
         ctypes.c_uint32, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p],
    ),
    "plato_agg_fedavg_qsgd": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_int, _c_float, _c_void_p, _c_void_p, _c_void_p,
         ctypes.c_uint32, _c_void_p, ctypes.c_uint32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_weighted_sum_f64": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_void_p, _c_size_t, _c_void_p]),
    "plato_agg_fedavg_w64": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_flatten": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_float, _c_void_p, _c_void_p],
    ),
    "plato_agg_sdot_pairs": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_size_t, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_sdot_shared_workspace": (_c_size_t, [_c_int, _c_int]),
    "plato_agg_sdot_shared": (
        _c_int, [_c_void_p, _c_void_p, _c_int, _c_size_t, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_fedadp_dots_workspace": (_c_size_t, [_c_int, _c_int, _c_size_t, _c_size_t, ctypes.c_uint32]),
    "plato_agg_fedadp_dots": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_size_t, _c_size_t, _c_float, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_fedadp_dots_ex": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_size_t, _c_size_t, _c_float, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int]),
    "plato_agg_port_norms": (
        _c_int,
        [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_size_t, _c_int, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_torch_cosine_workspace": (_c_size_t, [_c_int, _c_int]),
    "plato_agg_torch_cosine_sum_scaled": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_size_t, _c_void_p, _c_float, _c_int, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_scale_by_norm": (_c_int, [_c_void_p, _c_size_t, _c_void_p, _c_float, _c_void_p, _c_void_p]),
    "plato_agg_torch_cosine_sum": (
        _c_int,
        [_c_void_p, _c_void_p, _c_int, _c_size_t, _c_void_p, _c_void_p, _c_float, _c_int, _c_void_p, _c_void_p,
         _c_void_p],
    ),
    "plato_agg_np_sumsq_workspace": (_c_size_t, [_c_int, ctypes.c_uint32]),
    "plato_agg_np_sumsq": (
        _c_int,
        [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, ctypes.c_uint32, _c_void_p,
         _c_void_p, _c_void_p],
    ),
    "plato_agg_decode_rows": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_float, _c_void_p, ctypes.c_uint32, _c_void_p,
         ctypes.c_uint32, _c_size_t, _c_void_p, _c_void_p]),
    "plato_agg_comm_create": (_c_int, [_c_int, _c_void_p, ctypes.POINTER(_c_void_p)]),
    "plato_agg_comm_destroy": (_c_int, [_c_void_p]),
    "plato_agg_comm_size": (_c_int, [_c_void_p]),
    "plato_agg_comm_allgather_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "plato_agg_comm_reduce_scatter_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_void_p]),
}

# include/plato_agg_tune.h: exported by libplato_agg_tune.so only (the same sources built with every
# kernel variant; bench.py --sweep, scripts/ and the variant tests load it beside the product library)
TUNE_SIGNATURES = {
    "plato_agg_tune_num_variants": (_c_int, []),
    "plato_agg_tune_set_launch_groups": (None, [_c_u64]),
    "plato_agg_tune_set_entrywise_block": (None, [_c_int]),
    "plato_agg_tune_describe": (
        _c_int,
        [_c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int), ctypes.POINTER(_c_int),
         ctypes.POINTER(_c_int)],
    ),
    "plato_agg_tune_num_bf16_variants": (_c_int, []),
    "plato_agg_tune_fedavg_bf16": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
         _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_tune_stream": (_c_int, [_c_int, _c_void_p, _c_void_p, _c_size_t, _c_int, _c_void_p]),
    "plato_agg_tune_num_qsgd_variants": (_c_int, []),
    "plato_agg_tune_qsgd_chunk": (_c_int, [_c_int]),
    "plato_agg_tune_fedavg_qsgd": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_int, _c_float, _c_void_p, _c_void_p, _c_void_p,
         ctypes.c_uint32, _c_void_p, ctypes.c_uint32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
         _c_size_t, _c_size_t, _c_void_p],
    ),
    "plato_agg_tune_num_sdot_shared_variants": (_c_int, []),
    "plato_agg_tune_sdot_shared": (
        _c_int, [_c_int, _c_void_p, _c_void_p, _c_int, _c_size_t, _c_int, _c_void_p, _c_void_p, _c_void_p,
                 _c_void_p]),
    "plato_agg_tune_num_fedadp_variants": (_c_int, []),
    "plato_agg_tune_fedadp_is_probe": (_c_int, [_c_int]),
    "plato_agg_tune_fedadp_is_delta": (_c_int, [_c_int]),
    "plato_agg_tune_num_port_norms_variants": (_c_int, []),
    "plato_agg_tune_num_np_sumsq_variants": (_c_int, []),
    "plato_agg_tune_num_cosine_variants": (_c_int, []),
    "plato_agg_tune_torch_cosine_sum_scaled": (
        _c_int, [_c_int, _c_void_p, _c_void_p, _c_int, _c_size_t, _c_void_p, _c_float, _c_int, _c_void_p, _c_void_p,
                 _c_void_p]),
    "plato_agg_tune_num_entry_norms_variants": (_c_int, []),
    "plato_agg_tune_np_sumsq": (
        _c_int,
        [_c_int, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, ctypes.c_uint32, _c_void_p,
         _c_void_p, _c_void_p]),
    "plato_agg_tune_port_norms": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_size_t, _c_int, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_tune_fedadp_dots": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_size_t,
         _c_size_t, _c_size_t, _c_float, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "plato_agg_tune_entry_norms": (
        _c_int,
        [_c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, ctypes.c_uint32, _c_void_p,
         ctypes.c_uint32, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p],
    ),
    "plato_agg_tune_fedavg": (
        _c_int,
        [_c_int, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p,
         _c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_size_t, _c_void_p],
    ),
}

_lock = threading.Lock()
_lib = None
_tune = None


def _bind(handle, signatures):
    for name, (restype, argtypes) in signatures.items():
        fn = getattr(handle, name)
        fn.restype = restype
        fn.argtypes = argtypes


def lib() -> ctypes.CDLL:
    """Load (once) and return the engine library; raise if it is unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"plato_amd: HIP extension {LIB_PATH} is not built; run "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C plato_amd`)"
            )
        try:
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as exc:  # pragma: no cover - depends on the host
            raise RuntimeError(f"plato_amd: cannot load {LIB_PATH}: {exc}") from exc
        _bind(handle, SIGNATURES)
        version = handle.plato_agg_abi_version()
        if version != ABI_VERSION:
            raise RuntimeError(
                f"plato_amd: {LIB_PATH} has ABI {version}, expected {ABI_VERSION}; rebuild it"
            )
        _lib = handle
        return _lib


def tune() -> ctypes.CDLL:
    """Load (once) the tuning library: every product entry point plus the plato_agg_tune_* variants."""
    global _tune
    if _tune is not None:
        return _tune
    lib()
    with _lock:
        if _tune is not None:
            return _tune
        if not os.path.exists(TUNE_LIB_PATH):
            raise RuntimeError(f"plato_amd: {TUNE_LIB_PATH} is not built; run __graft_entry__.build()")
        handle = ctypes.CDLL(TUNE_LIB_PATH)  # RTLD_LOCAL: its symbols never interpose the product's
        _bind(handle, SIGNATURES)
        _bind(handle, TUNE_SIGNATURES)
        if handle.plato_agg_abi_version() != ABI_VERSION:
            raise RuntimeError(f"plato_amd: {TUNE_LIB_PATH} has another ABI version; rebuild it")
        _tune = handle
        return _tune


def check(status: int, what: str) -> None:
    """Map a C-ABI status code to the Python exception the reference would raise."""
    if status == PLATO_AGG_OK:
        return
    msg = lib().plato_agg_last_error().decode(errors="replace")
    if status == PLATO_AGG_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what}: {msg} (status {status})")


def call(name: str, *args) -> None:
    """Call a C-ABI entry point and raise on a non-zero status."""
    check(getattr(lib(), name)(*args), name)


def tune_call(name: str, *args) -> None:
    """Call an entry point of the tuning library (kernel variants) and raise on a non-zero status."""
    h = tune()
    status = getattr(h, name)(*args)
    if status != PLATO_AGG_OK:
        msg = h.plato_agg_last_error().decode(errors="replace")
        raise (ValueError if status == PLATO_AGG_EINVAL else RuntimeError)(f"{name}: {msg} (status {status})")

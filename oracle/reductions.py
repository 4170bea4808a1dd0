"""TEST INFRASTRUCTURE ONLY — ctypes front end of oracle/reductions.c and the flattenings the
reference's variant servers apply before reducing.

Imported by tests/ only, as the checker of plato_amd's flattened-reduction
kernels (never by plato_amd/).  ``oracle/libplato_oracle.so`` is built by
``__graft_entry__.build()`` (plain gcc, -ffp-contract=off).
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libplato_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built (run __graft_entry__.build())")
        h = ctypes.CDLL(LIB_PATH)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        for name, res, args in (
            ("plato_oracle_sdot_skx", ctypes.c_float, [i64, vp, vp]),
            ("plato_oracle_torch_norm", ctypes.c_float, [vp, i64]),
            ("plato_oracle_torch_sum", ctypes.c_float, [vp, i64, ctypes.c_int]),
            ("plato_oracle_torch_cosine", ctypes.c_float, [vp, vp, i64, ctypes.c_int, ctypes.c_float, vp]),
            ("plato_oracle_np_sum", ctypes.c_float, [vp, i64]),
        ):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
        _lib = h
    return _lib


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def sdot(x, y) -> np.float32:
    """numpy's float32 ``np.inner(x, y)`` (OpenBLAS sdot_k_SKYLAKEX order)."""
    x, y = _f32(x), _f32(y)
    return np.float32(lib().plato_oracle_sdot_skx(x.size, x.ctypes.data, y.ctypes.data))


def np_norm(x) -> np.float32:
    """``np.linalg.norm`` of a float32 vector: sqrt of its sdot with itself, in float32."""
    return np.sqrt(sdot(x, x))


def torch_norm(x) -> np.float32:
    x = _f32(x)
    return np.float32(lib().plato_oracle_torch_norm(x.ctypes.data, x.size))


def torch_sum(x, threads: int) -> np.float32:
    x = _f32(x)
    return np.float32(lib().plato_oracle_torch_sum(x.ctypes.data, x.size, threads))


def torch_cosine(a, b, threads: int, eps: float = 1e-8) -> np.float32:
    a, b = _f32(a), _f32(b)
    tmp = np.empty(a.size, dtype=np.float32)
    return np.float32(lib().plato_oracle_torch_cosine(a.ctypes.data, b.ctypes.data, a.size, threads, eps,
                                                      tmp.ctypes.data))


def np_sum(x) -> np.float32:
    """numpy's float32 ``np.sum`` (8192-element inner loops of pairwise sums)."""
    x = _f32(x)
    return np.float32(lib().plato_oracle_np_sum(x.ctypes.data, x.size))


# --------------------------------------------------------------------------
# the reference's flattenings
# --------------------------------------------------------------------------
def port_current_minus_previous(entries, bf, bi, pf, pi) -> np.ndarray:
    """port_server.py:36-48: ``torch.cat`` of every entry (state_dict order) into an fp32
    vector for each model, then ``current - previous``: int64 entries are cast to fp32
    by the concatenation before the subtraction."""
    parts = []
    for e in entries:
        if e.region == "f32":
            parts.append(np.subtract(bf[e.offset:e.offset + e.numel], pf[e.offset:e.offset + e.numel],
                                     dtype=np.float32))
        else:
            parts.append(np.subtract(bi[e.offset:e.offset + e.numel].astype(np.float32),
                                     pi[e.offset:e.offset + e.numel].astype(np.float32), dtype=np.float32))
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)


def port_delta(entries, bf, bi, xf, xi) -> np.ndarray:
    """port_server.py:45-48: the client's delta dict (x - b per entry, int64 exact) concatenated as fp32."""
    parts = []
    for e in entries:
        if e.region == "f32":
            parts.append(np.subtract(xf[e.offset:e.offset + e.numel], bf[e.offset:e.offset + e.numel],
                                     dtype=np.float32))
        else:
            d = xi[e.offset:e.offset + e.numel].astype(np.int64) - bi[e.offset:e.offset + e.numel].astype(np.int64)
            parts.append(d.astype(np.float32))
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)

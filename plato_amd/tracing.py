"""roctx ranges around the engine's stages, so rocprofv3 traces line up with Plato rounds.

``rocprofv3 --marker-trace`` records them (the reference has no
tracing beyond ad-hoc ``time.perf_counter``).  The marker library is bound
lazily with ctypes (rocprofiler-sdk's roctx, else the legacy libroctx64);
without either, ranges are no-ops — they carry no computation.
"""

from __future__ import annotations

import contextlib
import ctypes
import threading

_lock = threading.Lock()
_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if _tried:
        return _lib
    with _lock:
        if not _tried:
            for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                         "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so.4"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.argtypes = []
                    lib.roctxRangePop.restype = ctypes.c_int
                    _lib = lib
                    break
                except (OSError, AttributeError):
                    continue
            _tried = True
    return _lib


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx's vocabulary
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()

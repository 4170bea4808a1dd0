"""Payload ingestion: pickled ``state_dict`` bytes -> tensors in one flat (pinned) arena.

Replaces ``pickle.loads`` of a client payload on the server
(plato/servers/base.py:822; ``pickle.load`` at :791-792 for comm_simulation)
with ``libplato_ingest.so`` (include/plato_ingest.h): a C++ parser that only
recognises a pickled dict of CPU tensors and executes nothing, and a
multi-threaded gather of the tensor bytes straight into the arena the engine
copies to HBM.  With a layout, the result is an :class:`ArenaStateDict` whose
tensors are views of that arena, so staging it needs no pack step.
"""

from __future__ import annotations

import ctypes
import os
import threading
from collections import OrderedDict

import numpy as np
import torch

from .arena import CODECS, F32, I64, ArenaLayout

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libplato_ingest.so")
MAX_DIMS = 8

DTYPES = {
    0: torch.float32, 1: torch.int64, 2: torch.float64, 3: torch.float16, 4: torch.bfloat16,
    5: torch.int32, 6: torch.int16, 7: torch.int8, 8: torch.uint8, 9: torch.bool,
}


class TensorInfo(ctypes.Structure):
    _fields_ = [
        ("name_offset", ctypes.c_uint64),
        ("name_len", ctypes.c_uint32),
        ("dtype", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("contiguous", ctypes.c_int32),
        ("shape", ctypes.c_int64 * MAX_DIMS),
        ("stride", ctypes.c_int64 * MAX_DIMS),
        ("numel", ctypes.c_uint64),
        ("storage_offset", ctypes.c_uint64),
        ("storage_numel", ctypes.c_uint64),
        ("data_offset", ctypes.c_uint64),
        ("storage_id", ctypes.c_int32),
        ("element_size", ctypes.c_int32),
    ]


class IngestError(ValueError):
    """The bytes are not a pickled dict of CPU tensors this parser accepts."""


_lock = threading.Lock()
_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"plato_amd: {LIB_PATH} is not built; run __graft_entry__.build()")
            h = ctypes.CDLL(LIB_PATH)
            h.plato_ingest_last_error.restype = ctypes.c_char_p
            h.plato_ingest_last_error.argtypes = []
            h.plato_ingest_parse.restype = ctypes.c_int
            h.plato_ingest_parse.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(TensorInfo),
                                             ctypes.c_int]
            h.plato_ingest_gather.restype = ctypes.c_int
            h.plato_ingest_gather.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(TensorInfo),
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_int]
            vp, sz = ctypes.c_void_p, ctypes.c_size_t
            h.plato_ingest_join.restype = ctypes.c_int
            h.plato_ingest_join.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            for name, res, args in (
                ("plato_ingest_pack", ctypes.c_int, [vp, vp, vp, ctypes.c_int, vp, sz, ctypes.c_int]),
                ("plato_ingest_read_fd", ctypes.c_int64, [ctypes.c_int, vp, sz, ctypes.c_int]),
                ("plato_ingest_zstd_available", ctypes.c_int, []),
                ("plato_ingest_zstd_content_size", ctypes.c_int64, [vp, sz]),
                ("plato_ingest_zstd_decompress", ctypes.c_int64, [vp, sz, vp, sz]),
                ("plato_ingest_zstd_bound", sz, [sz]),
                ("plato_ingest_zstd_compress", ctypes.c_int64, [vp, sz, vp, sz, ctypes.c_int]),
            ):
                fn = getattr(h, name)
                fn.restype, fn.argtypes = res, args
            _lib = h
    return _lib


class ArenaStateDict(OrderedDict):
    """A ``state_dict`` whose tensors are views of one flat arena (layout order).

    ``arena_f32`` / ``arena_i64`` are the backing buffers (pinned when built
    for staging) and ``layout_signature`` identifies the layout; the engine's
    stager copies them to HBM directly instead of packing tensor by tensor.
    """

    arena_f32: torch.Tensor | None = None
    arena_i64: torch.Tensor | None = None
    layout_signature: tuple | None = None

    def __reduce__(self):  # pickles (e.g. for payload-size accounting) as a plain OrderedDict
        return (OrderedDict, (list(self.items()),))

    # Any change to the mapping (a processor or weights_received hook replacing
    # an entry) detaches the arena: the stager then packs the dict's current
    # tensors instead of copying stale arena bytes.  In-place writes to the
    # tensors themselves land in the arena and need nothing.
    def _detach_arena(self) -> None:
        self.arena_f32 = self.arena_i64 = self.layout_signature = None

    def __setitem__(self, key, value):
        self._detach_arena()
        super().__setitem__(key, value)

    def __delitem__(self, key):
        self._detach_arena()
        super().__delitem__(key)

    def pop(self, *args):
        self._detach_arena()
        return super().pop(*args)

    def popitem(self, last=True):
        self._detach_arena()
        return super().popitem(last)

    def setdefault(self, key, default=None):
        if key not in self:
            self._detach_arena()
        return super().setdefault(key, default)

    def update(self, *args, **kwargs):
        self._detach_arena()
        super().update(*args, **kwargs)

    def clear(self):
        self._detach_arena()
        super().clear()

    def __ior__(self, other):
        self._detach_arena()
        return super().__ior__(other)


def _buffer(data):
    """(address, length, keepalive) of a bytes-like object without copying."""
    if isinstance(data, (bytes, bytearray)):
        arr = np.frombuffer(data, dtype=np.uint8)
    else:
        arr = np.frombuffer(memoryview(data), dtype=np.uint8)
    return arr.ctypes.data, arr.size, arr


# output capacity per payload length: the parser's capacity-exceeded exit is slow (~20 ms on a ResNet-18
# payload), and the payloads of one server repeat their length, so the tensor count a length parsed to is
# remembered (a bounded table: one large payload no longer makes every later parse allocate for it)
_PARSE_CAP_DEFAULT = 256
_parse_caps: "OrderedDict[int, int]" = OrderedDict()
_PARSE_CAPS_KEPT = 64
_parse_caps_lock = threading.Lock()


def parse(data) -> tuple[list[TensorInfo], list[str], object]:
    """Parse pickled payload bytes; returns (tensor infos, keys, keepalive)."""
    addr, n, keep = _buffer(data)
    h = lib()
    with _parse_caps_lock:
        cap = _parse_caps.get(n, _PARSE_CAP_DEFAULT)
    while True:
        out = (TensorInfo * cap)()
        rc = h.plato_ingest_parse(addr, n, out, cap)
        if rc == -5:  # capacity
            cap *= 8
            continue
        if rc < 0:
            raise IngestError(f"payload rejected ({rc}): {h.plato_ingest_last_error().decode()}")
        with _parse_caps_lock:
            _parse_caps[n] = max(rc, 1)
            _parse_caps.move_to_end(n)
            while len(_parse_caps) > _PARSE_CAPS_KEPT:
                _parse_caps.popitem(last=False)
        infos = list(out[:rc])
        keys = [bytes(keep[t.name_offset : t.name_offset + t.name_len]).decode("utf-8") for t in infos]
        return infos, keys, keep


def _gather(keep, addr, n, infos, offsets, dst: torch.Tensor, threads: int):
    arr = (TensorInfo * len(infos))(*infos)
    offs = (ctypes.c_uint64 * len(infos))(*offsets)
    rc = lib().plato_ingest_gather(addr, n, arr, len(infos), offs, dst.data_ptr(),
                                   dst.numel() * dst.element_size(), threads)
    if rc < 0:
        raise IngestError(f"gather failed ({rc}): {lib().plato_ingest_last_error().decode()}")


def _owned_view(storage, byte_offset: int, nbytes: int, dtype, shape) -> torch.Tensor:
    """A tensor over ``storage[byte_offset : byte_offset + nbytes]`` whose storage is that slice.

    The slice shares the arena's memory (and keeps it alive), but the tensor
    owns a storage of exactly its own bytes, as the tensors pickle.loads
    builds do: re-pickling it (the reference sizes every payload with
    pickle.dumps, servers/base.py:839-846) writes its own bytes, not the
    whole arena once per tensor.
    """
    sub = storage[byte_offset : byte_offset + nbytes]
    return torch.empty(0, dtype=dtype).set_(sub, 0, shape)


def loads(data, layout: ArenaLayout | None = None, pin: bool = False, threads: int = 0,
          codec: str | None = None) -> OrderedDict:
    """``pickle.loads`` for a pickled ``state_dict`` of CPU tensors, natively.

    Without ``layout``: an ``OrderedDict`` of fresh contiguous tensors (one
    backing buffer).  With ``layout`` (the engine's arena for the baseline):
    an :class:`ArenaStateDict` laid out exactly as the arena, fp32 entries in
    the fp32 region and int64 entries in the int64 region; raises
    ``KeyError``/``ValueError`` if the payload does not match the layout.
    """
    infos, keys, keep = parse(data)
    addr, n = keep.ctypes.data, keep.size
    if layout is None:
        offsets, total = [], 0
        for t in infos:
            total = (total + 63) // 64 * 64
            offsets.append(total)
            total += t.numel * t.element_size
        buf = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=pin)
        _gather(keep, addr, n, infos, offsets, buf, threads)
        storage = buf.untyped_storage()
        out = OrderedDict()
        for key, t, off in zip(keys, infos, offsets):
            out[key] = _owned_view(storage, off, t.numel * t.element_size, DTYPES[t.dtype],
                                   tuple(t.shape[: t.ndim]))
        return out

    if len(keys) != len(layout.entries):
        raise KeyError(f"payload has {len(keys)} entries, the layout has {len(layout.entries)}")
    if codec is None:  # bf16 payloads (model_quantize) keep their dtype in the arena
        codec = "bf16" if infos and DTYPES[infos[0].dtype] == torch.bfloat16 else "native"
    dt_f, dt_i = CODECS[codec]
    f32 = torch.empty(layout.row_f32, dtype=dt_f, pin_memory=pin)
    i64 = torch.empty(layout.row_i64, dtype=dt_i, pin_memory=pin)
    es_f, es_i = f32.element_size(), i64.element_size()
    f_infos, f_offs, i_infos, i_offs = [], [], [], []
    for key, t in zip(keys, infos):
        if key not in layout._by_name:
            raise KeyError(f"payload entry {key!r} is not in the layout")
        e = layout[key]
        want = dt_f if e.region == F32 else dt_i
        shape = tuple(t.shape[: t.ndim])
        if DTYPES[t.dtype] != want or shape != e.shape:
            raise ValueError(f"payload[{key!r}] is {DTYPES[t.dtype]}{shape}, expected {want}{e.shape}")
        if e.region == F32:
            f_infos.append(t)
            f_offs.append(e.offset * es_f)
        else:
            i_infos.append(t)
            i_offs.append(e.offset * es_i)
    if f_infos:
        _gather(keep, addr, n, f_infos, f_offs, f32, threads)
    if i_infos:
        _gather(keep, addr, n, i_infos, i_offs, i64, threads)
    storages = {F32: (f32.untyped_storage(), es_f, dt_f), I64: (i64.untyped_storage(), es_i, dt_i)}
    out = ArenaStateDict()
    for key in keys:
        e = layout[key]
        storage, es, dt = storages[e.region]
        OrderedDict.__setitem__(out, key, _owned_view(storage, e.offset * es, e.numel * es, dt, e.shape))
    out.arena_f32, out.arena_i64 = f32, i64
    out.layout_signature = layout.signature
    return out


_scratch = threading.local()


def join(chunks, threads: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """``b"".join(chunks)`` (servers/base.py:821) as one parallel native copy.

    Into ``out`` if it is large enough (its first bytes are returned), else
    into a fresh buffer.
    """
    keeps = [_buffer(c) for c in chunks]
    total = sum(k[1] for k in keeps)
    if out is None or out.size < total:
        out = np.empty(max(total, 1), dtype=np.uint8)
    n = len(keeps)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[k[0] for k in keeps])
    lens = (ctypes.c_size_t * max(n, 1))(*[k[1] for k in keeps])
    rc = lib().plato_ingest_join(ptrs, lens, n, out.ctypes.data, total, threads)
    if rc < 0:
        raise IngestError(f"join failed ({rc}): {lib().plato_ingest_last_error().decode()}")
    del keeps
    return out[:total]


def _scratch_buffer(nbytes: int) -> np.ndarray:
    """This thread's reusable byte buffer, grown to at least ``nbytes``.

    Received bytes only live until their tensors are gathered out of them, so
    one buffer per thread serves every payload and steady-state reads and
    joins take no page faults.
    """
    buf = getattr(_scratch, "buf", None)
    if buf is None or buf.size < nbytes:
        buf = _scratch.buf = np.empty(max(nbytes, 1), dtype=np.uint8)
    return buf


def loads_chunks(chunks, layout: ArenaLayout | None = None, pin: bool = False, threads: int = 0):
    """``pickle.loads(b"".join(chunks))`` for a chunked payload, natively (join + parse + gather)."""
    total = sum(memoryview(c).nbytes for c in chunks)
    data = join(chunks, threads, out=_scratch_buffer(total))
    return loads(data, layout=layout, pin=pin, threads=threads)


def read_file(path: str, out: np.ndarray | None = None, threads: int = 0) -> np.ndarray:
    """The bytes of the file at ``path`` (parallel pread), into ``out`` if it is large enough.

    Raises what ``open(path, "rb")`` raises for a missing or unreadable file.
    """
    fd = os.open(path, os.O_RDONLY)
    try:
        size = os.fstat(fd).st_size
        if out is None or out.size < size:
            out = np.empty(max(size, 1), dtype=np.uint8)
        rc = lib().plato_ingest_read_fd(fd, out.ctypes.data, size, threads)
        if rc < 0:
            raise OSError(f"{path}: {lib().plato_ingest_last_error().decode()}")
        return out[:size]
    finally:
        os.close(fd)


EFORMAT, ECAPACITY, ENOCODEC, EUNKNOWNSIZE, EIO = -3, -5, -6, -7, -8


def zstd_available() -> bool:
    """True if the system libzstd.so.1 could be bound (model_compress payloads)."""
    return bool(lib().plato_ingest_zstd_available())


def _zstd_error(rc: int, what: str):
    msg = lib().plato_ingest_last_error().decode(errors="replace")
    if rc == ENOCODEC:
        return RuntimeError(f"{what}: {msg}")
    return IngestError(f"{what} failed ({rc}): {msg}")


def zstd_decompress(data) -> np.ndarray:
    """``zstd.decompress(data)`` (model_decompress.py:24) into a fresh uint8 array."""
    addr, n, keep = _buffer(data)
    h = lib()
    size = h.plato_ingest_zstd_content_size(addr, n)
    if size == EUNKNOWNSIZE:
        cap = max(4 * n, 1 << 16)  # streamed frame: grow until it fits
    elif size < 0:
        raise _zstd_error(size, "zstd content size")
    else:
        cap = size
    while True:
        out = np.empty(max(cap, 1), dtype=np.uint8)
        got = h.plato_ingest_zstd_decompress(addr, n, out.ctypes.data, cap)
        if got == ECAPACITY and size == EUNKNOWNSIZE:
            cap *= 4
            continue
        if got < 0:
            raise _zstd_error(got, "zstd decompress")
        del keep
        return out[:got]


def zstd_compress(data, level: int = 1) -> bytes:
    """``zstd.compress(data, level)`` (model_compress.py:25): one frame with its content size."""
    addr, n, keep = _buffer(data)
    h = lib()
    cap = h.plato_ingest_zstd_bound(n)
    if cap == 0:
        raise _zstd_error(ENOCODEC, "zstd compress")
    out = np.empty(cap, dtype=np.uint8)
    got = h.plato_ingest_zstd_compress(addr, n, out.ctypes.data, cap, int(level))
    if got < 0:
        raise _zstd_error(got, "zstd compress")
    del keep
    return out[:got].tobytes()


def loads_compressed(data, layout: ArenaLayout | None = None, pin: bool = False, threads: int = 0):
    """``pickle.loads(zstd.decompress(data))`` for a compressed ``state_dict``, natively."""
    return loads(zstd_decompress(data), layout=layout, pin=pin, threads=threads)


def load_file(path: str, layout: ArenaLayout | None = None, pin: bool = False, threads: int = 0) -> OrderedDict:
    """``pickle.load(open(path, 'rb'))`` of a comm_simulation payload file, natively.

    The file is read (in parallel) into this thread's scratch buffer and the
    tensors are gathered out of it, as for :func:`loads_chunks`.
    """
    data = read_file(path, out=_scratch_buffer(os.path.getsize(path)), threads=threads)
    return loads(data, layout=layout, pin=pin, threads=threads)

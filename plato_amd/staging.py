"""Host side of the H2D path: native packing into pinned arenas, and pinned result buffers.

The reference aggregates the K payload ``state_dict``s tensor by tensor on
the CPU (plato/servers/fedavg.py:148-154).  The engine moves each payload to
HBM as one flat arena: its tensors are packed into a pinned staging slot by
``plato_ingest_pack`` (the native copy pool, up to 16 threads) and the slot is
DMA'd to the device on a copy stream, while the next payload is packed into
the next slot.  Payloads that arrived through the native ingestion path
(:class:`~plato_amd.ingest.ArenaStateDict`) already are a pinned arena and skip
the pack.

Results come back into pinned buffers that are reused across rounds once no
tensor of an earlier result still refers to them (the reference hands the
server fresh tensors every round, so a buffer is never recycled under a dict
the caller kept).
"""

from __future__ import annotations

import threading
from typing import Mapping

import numpy as np
import torch

from . import ingest
from .arena import CODECS, F32, I64, ArenaLayout


class HostPacker:
    """Packs a CPU ``state_dict`` into flat (pinned) region buffers with the native copy pool."""

    def __init__(self, layout: ArenaLayout, codec: str = "native"):
        self.layout = layout
        self.codec = codec
        dt_f, dt_i = CODECS[codec]
        self.es = {F32: torch.empty(0, dtype=dt_f).element_size(), I64: torch.empty(0, dtype=dt_i).element_size()}
        self.dtypes = {F32: dt_f, I64: dt_i}
        self.names = {r: [e.name for e in layout.entries if e.region == r and e.numel] for r in (F32, I64)}
        self.offsets = {r: np.asarray([e.offset * self.es[r] for e in layout.entries if e.region == r and e.numel],
                                      dtype=np.uint64) for r in (F32, I64)}
        self.bytes = {r: np.asarray([e.numel * self.es[r] for e in layout.entries if e.region == r and e.numel],
                                    dtype=np.uint64) for r in (F32, I64)}
        self.numels = {r: [e.numel for e in layout.entries if e.region == r and e.numel] for r in (F32, I64)}

    def pack(self, state_dict: Mapping[str, torch.Tensor], out_f: torch.Tensor, out_i: torch.Tensor) -> None:
        """Copy ``state_dict`` into ``out_f`` / ``out_i`` (host buffers, layout order)."""
        lib = ingest.lib()
        keep = []
        for region, out in ((F32, out_f), (I64, out_i)):
            names = self.names[region]
            if not names:
                continue
            want = self.dtypes[region]
            src = np.empty(len(names), dtype=np.uint64)
            for j, name in enumerate(names):
                t = state_dict[name]
                if t.dtype != want or t.device.type != "cpu" or t.numel() != self.numels[region][j]:
                    raise ValueError(f"payload[{name!r}] is {t.dtype}[{t.numel()}] on {t.device}, expected "
                                     f"{want}[{self.numels[region][j]}] on the CPU")
                if not t.is_contiguous():
                    t = t.contiguous()
                    keep.append(t)
                src[j] = t.data_ptr()
            rc = lib.plato_ingest_pack(src.ctypes.data, self.bytes[region].ctypes.data,
                                       self.offsets[region].ctypes.data, len(names), out.data_ptr(),
                                       out.numel() * out.element_size(), 0)
            if rc < 0:
                raise ingest.IngestError(f"pack failed ({rc}): {lib.plato_ingest_last_error().decode()}")


def payload_fingerprint(state_dict) -> tuple:
    """Identity + in-place version of every tensor of a payload (and its arena, if ingested).

    A payload prestaged on arrival is adopted only if this is unchanged: a
    processor or hook that replaced an entry (new tensor object) or wrote one
    in place (torch bumps the tensor's version counter) after the copy was
    taken makes the round stage the payload again from its current tensors.
    """
    return (getattr(state_dict, "layout_signature", None),
            tuple((name, id(t), getattr(t, "_version", 0)) for name, t in state_dict.items()))


def baseline_key(state_dict) -> tuple:
    """Storage + in-place version of every tensor of a model's ``state_dict`` (delta arenas).

    ``extract_weights`` returns fresh tensor objects over the model's storage on every call, so a
    model is keyed by where its tensors live and their version counters: ``load_state_dict`` writes
    them in place (the counters move), a replaced parameter moves its storage.  Rows staged as deltas
    at arrival are adopted only by a round whose baseline has the same key.
    """
    try:
        return tuple((name, t.data_ptr(), t._version, tuple(t.shape), str(t.dtype)) for name, t in state_dict.items())
    except (AttributeError, RuntimeError):  # not tensors, or inference tensors (no version counter): no key
        return None


def arena_source(state_dict, layout: ArenaLayout, codec: str):
    """The pinned arena regions of an ingested payload, or None if it must be packed."""
    arena_f = getattr(state_dict, "arena_f32", None)
    if (arena_f is None or getattr(state_dict, "layout_signature", None) != layout.signature
            or arena_f.dtype != CODECS[codec][0] or not arena_f.is_pinned()):
        return None
    return arena_f, state_dict.arena_i64


class PinnedRing:
    """``depth`` pinned full-arena slots; a slot is reused once its copies have completed.

    Staging runs on the aggregation executor while arrivals may be prestaged
    from the event loop: a caller holds :attr:`lock` from :meth:`acquire`
    through the pack, the copies and :meth:`fence`, so two threads never pack
    into one slot or reuse a slot whose DMA is still unfenced.
    """

    def __init__(self, layout: ArenaLayout, codec: str = "native", depth: int = 4):
        dt_f, dt_i = CODECS[codec]
        self.slots = [(torch.empty(layout.row_f32, dtype=dt_f, pin_memory=True),
                       torch.empty(layout.row_i64, dtype=dt_i, pin_memory=True)) for _ in range(depth)]
        self.events: list[list] = [[] for _ in range(depth)]
        self.next = 0
        self.lock = threading.RLock()

    def acquire(self) -> int:
        j = self.next
        self.next = (j + 1) % len(self.slots)
        for ev in self.events[j]:
            ev.synchronize()
        self.events[j] = []
        return j

    def fence(self, j: int, events) -> None:
        self.events[j] = list(events)


def _in_use(t: torch.Tensor) -> bool:
    # the pool's own tensor + the temporary storage object = 2 references
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata) > 2


class ResultPool:
    """Pinned result buffers (fp32 arena + fp32 values of the int64 entries), reused when free."""

    def __init__(self, layout: ArenaLayout, keep: int = 4):
        self.layout = layout
        self.keep = keep
        self.bufs: list[tuple[torch.Tensor, torch.Tensor]] = []

    def get(self) -> tuple[torch.Tensor, torch.Tensor]:
        """A free pair, as views: the caller's views mark it busy until every result tensor is gone."""
        for pair in self.bufs:
            if not _in_use(pair[0]) and not _in_use(pair[1]):
                return pair[0][:], pair[1][:]
        pair = (torch.empty(self.layout.n_f32, dtype=torch.float32, pin_memory=True),
                torch.empty(self.layout.n_i64, dtype=torch.float32, pin_memory=True))
        if len(self.bufs) < self.keep:
            self.bufs.append(pair)
        return pair[0][:], pair[1][:]

"""Flat-arena layout of a Plato ``state_dict``.

The reference aggregates tensor by tensor (122 tensors for ResNet-18, median
256 elements: ``plato/servers/fedavg.py:152-154``).  On the GPU one launch per
tensor would be launch-bound, so the engine packs a ``state_dict`` into two
flat device regions and runs one kernel over the whole model:

* an fp32 region holding every ``torch.float32`` entry back to back in
  ``state_dict`` order, and
* an int64 region holding every ``torch.int64`` entry (BatchNorm
  ``num_batches_tracked`` counters).

The key -> (region, offset, shape) map is built from the baseline's key order
(``algorithms/fedavg.py:34``).  Client payloads must carry the same keys,
dtypes and shapes (the reference would fail on a mismatch too:
``algorithms/fedavg.py:20`` indexes the baseline by the client's key).
"""

from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Mapping

import numpy as np
import torch

F32 = "f32"
I64 = "i64"

# Arena rows are padded to a multiple of 64 fp32 (256 B) so that every client
# row of a [K, row] slab starts 256-byte aligned (dwordx4-friendly).
ROW_ALIGN = 64

# Payload codecs: element dtypes of (fp32 region, int64 region) as the client
# sends them.  "native": the model's own dtypes.  "bf16": Plato's
# model_quantize outbound processor (plato/processors/model_quantize.py:15)
# casts every entry to bfloat16.
CODECS = {"native": (torch.float32, torch.int64), "bf16": (torch.bfloat16, torch.bfloat16),
          # all-fp32 arrays over the model's keys (FedAtt's noise draws)
          "f32": (torch.float32, torch.float32),
          # QSGD code bytes (plato_amd.processors.qsgd.QsgdPayload)
          "qsgd": (torch.uint8, torch.uint8)}


def payload_codec(state_dict) -> str:
    """The codec a payload arrives in (all-bf16 entries -> "bf16"; QSGD payloads say so)."""
    codec = getattr(state_dict, "plato_codec", None)
    if codec is not None:
        return codec
    for tensor in state_dict.values():
        return "bf16" if isinstance(tensor, torch.Tensor) and tensor.dtype == torch.bfloat16 else "native"
    return "native"


@dataclass(frozen=True)
class Entry:
    name: str
    region: str  # F32 or I64
    offset: int  # element offset inside its region
    numel: int
    shape: tuple


# Arena alignments (``ArenaLayout.align``).  None: fp32 entries back to back.  "fedadp": every fp32
# entry starts at an arena offset congruent, mod FEDADP_ALIGN elements, to its position in FedAdp's
# flattened vector (process_grad: entries sorted by name.lower(), int64 counters one position per
# element; examples/server_aggregation/fedadp/fedadp_server.py:122-133), so the dot kernel's
# 16-byte gathers of a client arena start on whole 128-byte lines (csrc/fedadp.hip; an entry whose
# arena offset and flat position differ mod 4 costs ~15 % of the kernel's time).
# The padding (< FEDADP_ALIGN floats per entry) is never read as model data.
ALIGNMENTS = (None, "fedadp")
FEDADP_ALIGN = 32


def fedadp_order(names) -> list[int]:
    """Entry indices in FedAdp's flattening order (sorted by ``name.lower()``, stable)."""
    return sorted(range(len(names)), key=lambda i: names[i].lower())


class ArenaLayout:
    """Key -> region offsets for one model's ``state_dict``."""

    def __init__(self, entries: list[Entry], n_f32: int, n_i64: int, align: str | None = None):
        if align not in ALIGNMENTS:
            raise ValueError(f"unknown arena alignment {align!r}")
        self.entries = entries
        self.n_f32 = n_f32  # fp32 region length, padding included
        self.n_i64 = n_i64
        self.align = align
        # model elements of the fp32 region (algorithmic bytes count these, not the padding); a raw
        # arena without an entry map (bench pieces, distributed buckets) is all data
        self.n_f32_data = sum(e.numel for e in entries if e.region == F32) if entries else n_f32
        self.row_f32 = _round_up(max(n_f32, 1), ROW_ALIGN)
        self.row_i64 = max(n_i64, 1)
        self._by_name = {e.name: e for e in entries}
        self.signature = tuple((e.name, e.region, e.shape) for e in entries) + ((("align", align),) if align else ())
        self._cache: dict = {}

    @property
    def packed(self) -> bool:
        """fp32 entries back to back (no alignment padding)."""
        return self.n_f32 == self.n_f32_data

    def f32_padding(self, device) -> torch.Tensor | None:
        """Bool mask over the fp32 region, True at alignment padding (None for a packed region).

        The padding of a staged arena holds whatever its host staging buffer held there (the
        packer writes entries only), so two stagings of one model agree on the entries alone.
        """
        if self.packed:
            return None
        key = ("f32_padding", str(device))
        mask = self._cache.get(key)
        if mask is None:
            mask = torch.ones(self.n_f32, dtype=torch.bool)
            for e in self.entries:
                if e.region == F32:
                    mask[e.offset:e.offset + e.numel] = False
            mask = self._cache[key] = mask.to(device)
        return mask


    # ------------------------------------------------------------------ build
    @classmethod
    def _build(cls, items, align: str | None) -> "ArenaLayout":
        """``items``: [(name, region, numel, shape)] in state_dict order."""
        if align not in ALIGNMENTS:
            raise ValueError(f"unknown arena alignment {align!r}")
        flat_at = None
        if align == "fedadp":
            flat_at, flat = {}, 0
            for i in fedadp_order([it[0] for it in items]):
                flat_at[i] = flat
                flat += items[i][2]
        entries = []
        n = {F32: 0, I64: 0}
        for i, (name, region, numel, shape) in enumerate(items):
            off = n[region]
            if region == F32 and flat_at is not None:
                off += (flat_at[i] - off) % FEDADP_ALIGN
            entries.append(Entry(name, region, off, numel, shape))
            n[region] = off + numel
        return cls(entries, n[F32], n[I64], align)

    @classmethod
    def from_state_dict(cls, state_dict: Mapping[str, torch.Tensor], align: str | None = None) -> "ArenaLayout":
        items = []
        for name, tensor in state_dict.items():
            if not isinstance(tensor, torch.Tensor):
                raise TypeError(f"state_dict entry {name!r} is not a tensor")
            if tensor.dtype == torch.float32:
                region = F32
            elif tensor.dtype == torch.int64:
                region = I64
            else:
                raise TypeError(
                    f"state_dict entry {name!r} has dtype {tensor.dtype}; the aggregation "
                    "engine handles torch.float32 and torch.int64 entries"
                )
            items.append((name, region, tensor.numel(), tuple(tensor.shape)))
        return cls._build(items, align)

    @classmethod
    def from_shapes(cls, spec, align: str | None = None) -> "ArenaLayout":
        """Build from ``[(name, shape, 'f32'|'i64'), ...]`` (synthetic workloads)."""
        items = []
        for name, shape, region in spec:
            numel = 1
            for dim in shape:
                numel *= int(dim)
            items.append((name, region, numel, tuple(shape)))
        return cls._build(items, align)

    def aligned(self, align: str | None) -> "ArenaLayout":
        """The same entries under another alignment (self if it already has it)."""
        if align == self.align:
            return self
        key = ("aligned", align)
        hit = self._cache.get(key)
        if hit is None:
            hit = self._cache[key] = ArenaLayout._build([(e.name, e.region, e.numel, e.shape) for e in self.entries],
                                                        align)
        return hit

    # ---------------------------------------------------------------- queries
    def __len__(self) -> int:
        return len(self.entries)

    def __getitem__(self, name: str) -> Entry:
        return self._by_name[name]

    def keys(self):
        return [e.name for e in self.entries]

    def algorithmic_bytes(self, k: int) -> int:
        """HBM bytes of one fused FedAvg launch: read K clients + baseline, write result.

        SURVEY.md §8(d): (K+2)·P_f32·4 + (K+2)·P_i64·8 over the model's elements (alignment
        padding, which the kernels also stream, is not counted).
        """
        return (k + 2) * (self.n_f32_data * 4 + self.n_i64 * 8)

    def check_compatible(self, state_dict: Mapping[str, torch.Tensor], what: str,
                         codec: str = "native") -> None:
        if len(state_dict) != len(self.entries):
            raise KeyError(
                f"{what} has {len(state_dict)} entries, the baseline has {len(self.entries)}"
            )
        for entry in self.entries:
            if entry.name not in state_dict:
                raise KeyError(f"{what} is missing {entry.name!r}")
            tensor = state_dict[entry.name]
            want = CODECS[codec][0] if entry.region == F32 else CODECS[codec][1]
            # coded payloads keep flat code bytes and carry the tensor shapes separately
            shape = tuple(getattr(state_dict, "shapes", {}).get(entry.name, tensor.shape))
            if tensor.dtype != want or shape != entry.shape or tensor.numel() != entry.numel:
                raise ValueError(
                    f"{what}[{entry.name!r}] is {tensor.dtype}{tuple(tensor.shape)}, "
                    f"expected {want}{entry.shape}"
                )

    def chunk_tables(self, cap: int):
        """Per-entry work pieces for the chunked kernels (``plato_agg_chunk`` rows).

        Returns two ``uint32 [n, 4]`` arrays, (entry index, begin, end, 0), for
        the fp32 and the int64 region, sorted by entry.  fp32 entries are cut
        at multiples of ``cap`` elements of the arena (``cap`` % 4 == 0), so
        only the first and last piece of an entry start or end inside a
        float4 group; each int64 entry is one piece.  Empty entries get none.
        """
        if cap <= 0 or cap % 4:
            raise ValueError("chunk capacity must be a positive multiple of 4")
        key = ("chunks", cap)
        cached = self._cache.get(key)
        if cached is not None:
            return cached
        f32, i64 = [], []
        for idx, e in enumerate(self.entries):
            if e.numel == 0:
                continue
            if e.region == I64:
                i64.append((idx, e.offset, e.offset + e.numel, 0))
                continue
            lo, end = e.offset, e.offset + e.numel
            while lo < end:
                hi = min(end, (lo // cap + 1) * cap)
                f32.append((idx, lo, hi, 0))
                lo = hi
        out = (np.asarray(f32, dtype=np.uint32).reshape(-1, 4), np.asarray(i64, dtype=np.uint32).reshape(-1, 4))
        self._cache[key] = out
        return out

    def promoted(self) -> "ArenaLayout":
        """The same entries, all fp32: the int64 counters as fp32 entries after the fp32 region.

        What a dequantized payload is in the reference (every entry float32 after
        model_dequantize / model_dequantize_qsgd), so the per-entry reductions
        of the variant servers run on it with float32(x) - float32(b) for a
        counter (plato_agg_decode_rows builds the rows).  Entry order, names and
        shapes are unchanged; a counter's offset is ``row_f32 + its int64 offset``.
        """
        hit = self._cache.get("promoted")
        if hit is None:
            entries = [e if e.region == F32 else Entry(e.name, F32, self.row_f32 + e.offset, e.numel, e.shape)
                       for e in self.entries]
            hit = ArenaLayout(entries, self.row_f32 + self.n_i64 if self.n_i64 else self.n_f32, 0, self.align)
            self._cache["promoted"] = hit
        return hit

    # ---------------------------------------------------------- pack / unpack
    def pack(self, state_dict: Mapping[str, torch.Tensor], out_f32: torch.Tensor,
             out_i64: torch.Tensor | None) -> None:
        """Copy ``state_dict`` into flat (host or device) buffers ``out_f32``/``out_i64``."""
        f32 = [state_dict[e.name].reshape(-1) for e in self.entries if e.region == F32]
        i64 = [state_dict[e.name].reshape(-1) for e in self.entries if e.region == I64]
        if f32 and self.packed:
            torch.cat(f32, out=out_f32[: self.n_f32])
        elif f32:
            for e in self.entries:
                if e.region == F32:
                    out_f32[e.offset:e.offset + e.numel].copy_(state_dict[e.name].reshape(-1))
        if i64:
            torch.cat(i64, out=out_i64[: self.n_i64])

    def unpack(self, flat_f32: torch.Tensor, flat_i64: torch.Tensor | None
               ) -> "OrderedDict[str, torch.Tensor]":
        """Views of flat buffers as an ``OrderedDict`` in baseline key order.

        ``flat_i64`` holds the int64 entries' values in whatever dtype the
        caller produced (fp32 results of update_weights, or int64 weights).
        """
        out = OrderedDict()
        for e in self.entries:
            src = flat_f32 if e.region == F32 else flat_i64
            out[e.name] = src[e.offset : e.offset + e.numel].view(e.shape)
        return out


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def same_f32_bits(a: torch.Tensor, b: torch.Tensor, padding: torch.Tensor | None) -> bool:
    """Whether two fp32 arena regions (device tensors of one length) hold the same bits outside ``padding``."""
    a, b = a.view(torch.int32), b.view(torch.int32)
    if padding is None:
        return torch.equal(a, b)
    return not bool(torch.any((a != b) & ~padding))

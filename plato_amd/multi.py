"""Multi-GPU aggregation inside one Plato server process (parameter-bucket sharding).

Plato's server is a single process on one asyncio event loop
(plato/servers/base.py:323-327) that calls ``aggregate_weights`` once per round
(plato/servers/fedavg.py:171-182).  :class:`MultiDeviceEngine` keeps that
contract and drives every GPU of the node from the server process:

* the flat fp32 arena is cut into one contiguous, 256-byte-aligned bucket per
  GPU (:class:`~plato_amd.distributed.BucketPlan`; the int64 counters ride
  with bucket 0);
* each payload is packed once into a pinned host slot (or used in place when
  it arrived through native ingestion) and GPU g receives only bucket g of it,
  on its own copy stream: the N PCIe links each carry 1/N of every payload;
* GPU g runs the same sequential-K FedAvg kernel on its bucket.  Every element
  still sums its K clients in ``self.updates`` order, so the result is
  bit-identical to the one-GPU and CPU-reference results — there is no
  cross-GPU arithmetic;
* the new model is assembled by a per-bucket D2H into one pinned host result
  (what ``load_weights`` consumes), and, when it should stay device-resident,
  by an RCCL all-gather over xGMI (``plato_agg_comm_allgather_f32``, one
  communicator per GPU from ``ncclCommInitAll``).

Rounds that reduce per entry — FedAtt's norms and attentive sum, Polaris'
per-layer squared sums, QSGD payloads with their per-entry scales — are
sharded by whole entries instead (:attr:`MultiDeviceEngine.entries`,
:class:`~plato_amd.distributed.EntryPlan`): GPU g runs the single-GPU engine
on its contiguous group of entries, every value stays on one GPU and the
per-entry results are concatenated in layout order.  Rounds whose weights need
serial reductions over the whole flattened model (Port's cosine similarity,
FedAdp's dots: one fma chain per vector in the reference's order) cannot cut the
model, but each client's chain is independent of the others': they are staged and
finished bucket-sharded like a plain round, and the reductions are split by
client (:attr:`MultiDeviceEngine.clients`, :class:`ClientRound`) — client j's
whole arena is assembled on GPU j mod N from the buckets, FedAdp's global
gradient is formed bucket-sharded and all-gathered, and every GPU runs the
single-GPU kernels on its own clients, so every value is still computed by one
chain on one GPU, bit-identical to the one-GPU result.
"""

from __future__ import annotations

import ctypes
import time
from collections import OrderedDict
from typing import Mapping, Sequence

import numpy as np
import torch

from . import _lib
from .arena import CODECS, ArenaLayout, payload_codec, same_f32_bits
from .distributed import BucketPlan, EntryPlan
from .engine import FedAvgEngine, fp32_weights, require_device
from .staging import HostPacker, PinnedRing, ResultPool, arena_source, baseline_key, payload_fingerprint

MULTI_CODECS = ("native", "bf16")


def _ptr(t):
    return None if t is None else t.data_ptr()


class _Shard:
    """Bucket ``index`` of the arena on one GPU: baseline, client rows, result, streams."""

    def __init__(self, index: int, device: torch.device, plan: BucketPlan):
        self.index = index
        self.device = device
        self.lo, self.hi = plan.f32_range(index)
        self.ilo, self.ihi = plan.i64_range(index)
        self.n = self.hi - self.lo
        self.ni = self.ihi - self.ilo
        self.per = plan.per
        self.layout = ArenaLayout([], self.n, self.ni)  # kernel sizes of this bucket
        with torch.cuda.device(device):
            self.copy_stream = torch.cuda.Stream(device)
            self.stream = torch.cuda.Stream(device)
        self.base_f = torch.empty(self.per, dtype=torch.float32, device=device)
        self.base_i = torch.empty(max(self.ni, 1), dtype=torch.int64, device=device)
        self.slabs: dict[str, tuple[torch.Tensor, torch.Tensor]] = {}
        self.arrival_slabs: dict[str, list] = {}

    def slab(self, codec: str, capacity: int):
        hit = self.slabs.get(codec)
        if hit is None or hit[0].shape[0] < capacity:
            self.slabs.pop(codec, None)
            dt_f, dt_i = CODECS[codec]
            hit = (torch.empty((capacity, self.per), dtype=dt_f, device=self.device),
                   torch.empty((capacity, max(self.ni, 1)), dtype=dt_i, device=self.device))
            self.slabs[codec] = hit
        return hit

    def new_arrival_slab(self, codec: str, rows: int):
        dt_f, dt_i = CODECS[codec]
        slab = (torch.empty((rows, self.per), dtype=dt_f, device=self.device),
                torch.empty((rows, max(self.ni, 1)), dtype=dt_i, device=self.device))
        self.arrival_slabs.setdefault(codec, []).append(slab)
        return slab

    def arrival_base(self):
        """This bucket of the model the arrivals are turned into deltas against (allocated on first use)."""
        if getattr(self, "_arr", None) is None:
            self._arr = (torch.empty(self.per, dtype=torch.float32, device=self.device),
                         torch.empty(max(self.ni, 1), dtype=torch.int64, device=self.device))
        return self._arr

    def to_delta(self, row_f: torch.Tensor, row_i: torch.Tensor, base_f: torch.Tensor, base_i: torch.Tensor) -> None:
        """row -= base for this bucket, in place, on the copy stream (behind the row's and the base's H2D)."""
        if not (self.n or self.ni):
            return
        _lib.call("plato_agg_compute_deltas", _ptr(row_f) if self.n else None, _ptr(row_i) if self.ni else None,
                  _ptr(base_f) if self.n else None, _ptr(base_i) if self.ni else None,
                  _ptr(row_f) if self.n else None, _ptr(row_i) if self.ni else None, self.n, self.ni,
                  self.copy_stream.cuda_stream)

    def same_bits(self, a_f: torch.Tensor, a_i: torch.Tensor, b_f: torch.Tensor, b_i: torch.Tensor,
                  layout: ArenaLayout | None = None) -> bool:
        """Whether two copies of this bucket hold the same bits (after this shard's copy stream); with the
        full model's ``layout``, outside its alignment padding (ArenaLayout.f32_padding)."""
        with torch.cuda.device(self.device):
            torch.cuda.current_stream(self.device).wait_stream(self.copy_stream)
            pad = None if layout is None else layout.f32_padding(self.device)
            return (same_f32_bits(a_f[: self.n], b_f[: self.n], None if pad is None else pad[self.lo:self.hi])
                    and torch.equal(a_i[: self.ni], b_i[: self.ni]))

    def copy_in(self, host_f: torch.Tensor, host_i: torch.Tensor, dst_f: torch.Tensor, dst_i: torch.Tensor):
        """Bucket slice of a full host arena -> this GPU (on the copy stream)."""
        with torch.cuda.stream(self.copy_stream):
            if self.n:
                dst_f[: self.n].copy_(host_f[self.lo:self.hi], non_blocking=True)
            if self.ni:
                dst_i[: self.ni].copy_(host_i[self.ilo:self.ihi], non_blocking=True)


def _row_ptr(t: torch.Tensor, row: int) -> int:
    return t.data_ptr() + row * t.stride(0) * t.element_size()


def _copy_rows(dst: torch.Tensor, rows: Sequence[torch.Tensor]) -> None:
    """``dst[i] = rows[i]`` (stream-ordered): one strided copy when the rows are equally spaced in one storage
    (a slab's rows, the common case), else one copy per row (rows adopted from several arrival slabs)."""
    r0 = rows[0]
    step = rows[1].data_ptr() - r0.data_ptr() if len(rows) > 1 else r0.numel() * r0.element_size()
    one = step > 0 and step % r0.element_size() == 0 and r0.is_contiguous() and all(
        b.untyped_storage().data_ptr() == r0.untyped_storage().data_ptr() and b.shape == r0.shape
        and b.data_ptr() - a.data_ptr() == step for a, b in zip(rows, rows[1:]))
    if one:
        src = r0.as_strided((len(rows), r0.numel()), (step // r0.element_size(), 1), r0.storage_offset())
        dst.copy_(src, non_blocking=True)
        return
    for i, row in enumerate(rows):
        dst[i].copy_(row, non_blocking=True)


class MultiDeviceEngine:
    """Bucket-sharded FedAvg over several GPUs of one node, driven from one process."""

    ARRIVAL_CHUNK = 16

    def __init__(self, devices: Sequence, variant: int | None = None, ring_depth: int = 4):
        if not devices:
            raise ValueError("MultiDeviceEngine needs at least one device")
        self.devices = [require_device(d) for d in devices]
        self.lib = _lib.lib()
        self.variant = variant
        self.ring_depth = ring_depth
        self.primary = FedAvgEngine(self.devices[0], variant=variant)
        self._layout: ArenaLayout | None = None
        self._plan: BucketPlan | None = None
        self._shards: list[_Shard] = []
        self._rings: dict[str, PinnedRing] = {}
        self._packers: dict[str, HostPacker] = {}
        self._results: ResultPool | None = None
        self._arrivals: dict = {}
        self._arrival_free: dict = {}
        self._comm = None
        self._entries: "EntryShardedEngine | None" = None
        self._clients: "ClientShardedEngine | None" = None
        self._client_engines: list[FedAvgEngine] = [self.primary]
        self._pool = None
        self._delta_arenas = False
        self._arrival_base_key = None

    @property
    def delta_arenas(self) -> bool:
        """Stage clients as their deltas x - b (FedAvgEngine.delta_arenas) on every device of this engine.

        Bucket rounds (and ClientRound's client-split reductions) then hold deltas, formed per bucket right
        behind each H2D (at arrival with ``prestage(..., baseline)``); the entry shards' and the primary's
        engines follow the same setting.
        """
        return self._delta_arenas

    @delta_arenas.setter
    def delta_arenas(self, on: bool) -> None:
        self._delta_arenas = bool(on)
        for eng in self._client_engines:
            eng.delta_arenas = self._delta_arenas
        if self._entries is not None:
            for eng in self._entries._engines:
                eng.delta_arenas = self._delta_arenas

    @property
    def world(self) -> int:
        return len(self.devices)

    @property
    def device(self) -> torch.device:
        return self.devices[0]

    @property
    def clients(self) -> "ClientShardedEngine":
        """The same devices for FedAdp / Port rounds: bucket-sharded staging, reductions split by client."""
        if self._clients is None:
            self._clients = ClientShardedEngine(self)
        return self._clients

    def client_engine(self, g: int) -> FedAvgEngine:
        """The single-GPU engine on device g that holds the whole arenas of the clients ClientRound gives it."""
        while len(self._client_engines) <= g:
            eng = FedAvgEngine(self.devices[len(self._client_engines)], variant=self.variant)
            eng.layout_align = self.layout_align
            eng.delta_arenas = self._delta_arenas
            self._client_engines.append(eng)
        return self._client_engines[g]

    def each(self, fn, items):
        """``[fn(item) ...]`` with one worker thread per device (torch / HIP calls release the GIL)."""
        items = list(items)
        if len(items) <= 1:
            return [fn(x) for x in items]
        if self._pool is None:
            import concurrent.futures

            self._pool = concurrent.futures.ThreadPoolExecutor(self.world, thread_name_prefix="plato-amd-device")
        return list(self._pool.map(fn, items))

    @property
    def entries(self) -> "EntryShardedEngine":
        """The same devices sharded by whole entries (per-entry variant rounds, QSGD payloads)."""
        if self._entries is None:
            self._entries = EntryShardedEngine(self)
        return self._entries

    # ------------------------------------------------------------ layout
    @property
    def layout_align(self) -> str | None:
        """Arena alignment of the layouts this engine builds (passed on to every per-device engine)."""
        return self.primary.layout_align

    @layout_align.setter
    def layout_align(self, align: str | None) -> None:
        self.primary.layout_align = align
        for eng in self._client_engines:
            eng.layout_align = align
        if self._entries is not None:
            for eng in self._entries._engines:
                eng.layout_align = align

    def _prepare(self, template: Mapping[str, torch.Tensor] | ArenaLayout) -> ArenaLayout:
        layout = (template if isinstance(template, ArenaLayout)
                  else ArenaLayout.from_state_dict(template, align=self.layout_align))
        if self._layout is None or self._layout.signature != layout.signature:
            self._layout = layout
            self._plan = BucketPlan.for_layout(layout, self.world)
            self._shards = [_Shard(g, d, self._plan) for g, d in enumerate(self.devices)]
            self._rings, self._packers = {}, {}
            self._results = ResultPool(layout)
            self._arrivals, self._arrival_free = {}, {}
            self._arrival_base_key = None
        return self._layout

    def _ring(self, codec: str) -> tuple[PinnedRing, HostPacker]:
        if codec not in self._rings:
            self._rings[codec] = PinnedRing(self._layout, codec, self.ring_depth)
            self._packers[codec] = HostPacker(self._layout, codec)
        return self._rings[codec], self._packers[codec]

    def _stage(self, payload, codec: str, rows) -> None:
        """Send bucket g of ``payload`` to ``rows[g] = (dst_f row, dst_i row)`` on every GPU."""
        src = arena_source(payload, self._layout, codec)
        if src is not None:
            for shard, (df, di) in zip(self._shards, rows):
                shard.copy_in(src[0], src[1], df, di)
            return
        ring, packer = self._ring(codec)
        with ring.lock:  # acquire -> pack -> copies -> fence as one step (executor vs event loop)
            j = ring.acquire()
            hf, hi = ring.slots[j]
            packer.pack(payload, hf, hi)
            events = []
            for shard, (df, di) in zip(self._shards, rows):
                shard.copy_in(hf, hi, df, di)
                ev = torch.cuda.Event()
                ev.record(shard.copy_stream)
                events.append(ev)
            ring.fence(j, events)

    # ------------------------------------------------------------ rounds
    def begin(self, template, capacity: int, codec: str = "native", client_split: bool = False) -> "MultiRound":
        """A bucket-sharded round (``client_split``: a :class:`ClientRound`, native payloads)."""
        if capacity <= 0:
            raise ValueError("no client payloads to aggregate")
        if codec not in MULTI_CODECS:
            raise ValueError(f"codec {codec!r} is aggregated on one device (use .primary)")
        if client_split and codec != "native":
            raise ValueError("client-split rounds take native payloads (coded ones run on .primary)")
        layout = self._prepare(template)
        for shard in self._shards:
            shard.slab(codec, capacity)
            # the previous round's kernel (and a client-split assembly, on the current stream) may still
            # read this round's rows
            shard.copy_stream.wait_stream(shard.stream)
            shard.copy_stream.wait_stream(torch.cuda.current_stream(shard.device))
        return (ClientRound if client_split else MultiRound)(self, layout, capacity, codec)

    def prestage(self, payload: Mapping[str, torch.Tensor], baseline_layout: ArenaLayout,
                 baseline: Mapping[str, torch.Tensor] | None = None) -> bool:
        """Copy an arriving payload's buckets to their GPUs now (adopted by the next round).

        With :attr:`delta_arenas` and the server's current model as ``baseline``, each bucket of the
        row is turned into its delta right behind its H2D, against that model's bucket on the same GPU
        (FedAvgEngine.prestage, per bucket); a round adopts it only if its own baseline is that model
        unchanged (its :func:`baseline_key`, and the staged bits compared on the device)."""
        codec = payload_codec(payload)
        if codec not in MULTI_CODECS:
            return self.primary.prestage(payload, baseline_layout, baseline)
        try:
            baseline_layout.check_compatible(payload, "arriving payload", codec)
        except (KeyError, ValueError):
            return False
        self._prepare(baseline_layout)
        free = self._arrival_free.setdefault(codec, [])
        if not free:
            slabs = [s.new_arrival_slab(codec, self.ARRIVAL_CHUNK) for s in self._shards]
            free.extend((slabs, r) for r in range(self.ARRIVAL_CHUNK))
        slabs, row = free.pop()
        self._stage(payload, codec, [(f[row], i[row]) for f, i in slabs])
        delta_key = None
        if self._delta_arenas and codec == "native" and baseline is not None:
            delta_key = self._arrival_baseline(baseline)
            if delta_key is not None:  # x - b per bucket, in place, behind this payload's H2D
                for s, (f, i) in zip(self._shards, slabs):
                    af, ai = s.arrival_base()
                    s.to_delta(f[row], i[row], af, ai)
        ptrs = [(_row_ptr(f, row), _row_ptr(i, row)) for f, i in slabs]
        self._arrivals[id(payload)] = (payload, codec, self._layout.signature, ptrs, slabs, row,
                                       payload_fingerprint(payload), delta_key)
        return True

    def _arrival_baseline(self, baseline: Mapping[str, torch.Tensor]):
        """The arrival baseline's buckets on their GPUs (staged once per model version); its key, or None."""
        key = baseline_key(baseline)
        if key is None:
            return None
        if key == self._arrival_base_key:
            return key
        try:
            self._layout.check_compatible(baseline, "baseline")
        except (KeyError, ValueError):
            return None
        # copy-stream order: rows converted against the previous model ran before this copy
        self._stage(baseline, "native", [s.arrival_base() for s in self._shards])
        self._arrival_base_key = key
        return key

    def _arrival_base_matches(self, shards_base) -> bool:
        """The round's staged baseline (``[(base_f, base_i)]`` per shard) has the arrival baseline's bits."""
        return all(s.same_bits(bf, bi, *s.arrival_base(), layout=self._layout)
                   for s, (bf, bi) in zip(self._shards, shards_base))

    def _arrival_rows(self, payload, layout: ArenaLayout, codec: str):
        hit = self._arrivals.get(id(payload))
        if hit is None or hit[0] is not payload or hit[1] != codec or hit[2] != layout.signature:
            return None
        if hit[6] != payload_fingerprint(payload):
            return None  # edited after arrival: the round stages its current tensors
        return hit[3], [(f[hit[5]], i[hit[5]]) for f, i in hit[4]], hit[7]

    def release_arrivals(self) -> None:
        for _, codec, _, _, slabs, row, _, _ in self._arrivals.values():
            self._arrival_free.setdefault(codec, []).append((slabs, row))
        self._arrivals = {}
        self.primary.release_arrivals()
        if self._entries is not None:
            self._entries._release()

    def comm(self):
        """The RCCL communicator over the engine's devices (distinct GPUs only)."""
        if self._comm is None:
            ids = [d.index for d in self.devices]
            if len(set(ids)) != len(ids):
                return None
            handle = ctypes.c_void_p()
            arr = (ctypes.c_int * len(ids))(*ids)
            _lib.call("plato_agg_comm_create", len(ids), ctypes.cast(arr, ctypes.c_void_p), ctypes.byref(handle))
            self._comm = handle
        return self._comm

    def close(self) -> None:
        if self._comm is not None:
            _lib.call("plato_agg_comm_destroy", self._comm)
            self._comm = None

    def __del__(self):  # pragma: no cover - interpreter teardown order varies
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------- convenience API
    def aggregate_weights(self, baseline, weights_received, weights, scales=None):
        """``update_weights(aggregate_deltas(compute_weight_deltas(b, X)))`` over the GPUs."""
        k = len(weights_received)
        if k == 0:
            raise ValueError("no client payloads to aggregate")
        if len(weights) != k:
            raise ValueError("weights must have one entry per client")
        codec = payload_codec(weights_received[0])
        if codec not in MULTI_CODECS:
            return self.primary.aggregate_weights(baseline, weights_received, weights, scales)
        rnd = self.begin(baseline, k, codec)
        rnd.put_baseline(baseline)
        for i, sd in enumerate(weights_received):
            if not rnd.adopt(i, sd):
                rnd.put_client(i, sd)
        rnd.launch(weights, scales)
        return rnd.result()

    def aggregate_deltas(self, deltas_received, weights, scales=None):
        k = len(deltas_received)
        if k == 0:
            raise ValueError("no client deltas to aggregate")
        if len(weights) != k:
            raise ValueError("weights must have one entry per client")
        rnd = self.begin(deltas_received[0], k)
        for i, sd in enumerate(deltas_received):
            rnd.put_client(i, sd, what="deltas_received")
        rnd.launch(weights, scales, deltas=True)
        return rnd.result()


class MultiRound:
    """One bucket-sharded aggregation: stage (any order), launch on every GPU, assemble."""

    def __init__(self, engine: MultiDeviceEngine, layout: ArenaLayout, capacity: int, codec: str):
        self.engine = engine
        self.layout = layout
        self.capacity = capacity
        self.codec = codec
        self.staged = [False] * capacity
        self._ptrs: list = [None] * capacity  # per slot: per shard (fp32 row ptr, int64 row ptr)
        self._rows: list = [None] * capacity  # per slot: per shard (fp32 row, int64 row) tensors
        self.has_baseline = False
        self.events: list = []
        self._out = None
        self._keep = None
        self._device_results = None
        self._t0 = time.perf_counter()
        self.timings: dict = {}
        self._k = 0
        # delta arenas (MultiDeviceEngine.delta_arenas): every staged row holds x - b per bucket, formed on
        # its shard's copy stream behind its H2D; the launch is the deltas-form kernel plus b + acc
        self.deltas = bool(getattr(engine, "delta_arenas", False)) and codec == "native"
        self._base_key = None
        self._arrival_base_ok = None  # the device check of the arrival baseline, once per round
        self._converted: set = set()

    def put_baseline(self, baseline: Mapping[str, torch.Tensor]) -> None:
        self.layout.check_compatible(baseline, "baseline_weights")
        if self.deltas and any(self.staged):
            raise ValueError("delta arenas: the clients were staged as deltas of the previous baseline")
        eng = self.engine
        eng._stage(baseline, "native", [(s.base_f, s.base_i) for s in eng._shards])
        self.has_baseline = True
        self._base_key = baseline_key(baseline)
        self._arrival_base_ok = None

    def _to_delta(self, rows) -> None:
        key = tuple(r[0].data_ptr() for r in rows)
        if key in self._converted:
            return
        for s, (f, i) in zip(self.engine._shards, rows):
            s.to_delta(f, i, s.base_f, s.base_i)
        self._converted.add(key)

    def put_client(self, slot: int, payload, what: str = "weights_received") -> None:
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        self.layout.check_compatible(payload, f"{what}[{slot}]", self.codec)
        if self.deltas and not self.has_baseline:
            raise ValueError("delta arenas: stage the baseline before the clients")
        eng = self.engine
        rows = []
        ptrs = []
        for s in eng._shards:
            f, i = s.slabs[self.codec]
            rows.append((f[slot], i[slot]))
            ptrs.append((_row_ptr(f, slot), _row_ptr(i, slot)))
        eng._stage(payload, self.codec, rows)
        self._converted.discard(tuple(r[0].data_ptr() for r in rows))  # fresh weights in the rows
        if self.deltas:
            self._to_delta(rows)
        self._ptrs[slot] = ptrs
        self._rows[slot] = rows
        self.staged[slot] = True

    def adopt(self, slot: int, payload) -> bool:
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        hit = self.engine._arrival_rows(payload, self.layout, self.codec)
        if hit is None:
            return False
        ptrs, rows, delta_key = hit
        if delta_key is not None:
            if not (self.deltas and self.has_baseline and delta_key == self._base_key):
                return False  # a delta against another model (or a weight round): stage the payload again
            if self._arrival_base_ok is None:  # the key matched; the bits must too (an in-place write that
                # left the version counters alone, a reused address): compared once per round, on the devices
                self._arrival_base_ok = self.engine._arrival_base_matches([(s.base_f, s.base_i)
                                                                            for s in self.engine._shards])
            if not self._arrival_base_ok:
                return False
            self._converted.add(tuple(r[0].data_ptr() for r in rows))
        elif self.deltas:
            if not self.has_baseline:
                raise ValueError("delta arenas: stage the baseline before the clients")
            self._to_delta(rows)  # the arrival rows hold weights: their deltas now (the rows are this round's)
        self._ptrs[slot], self._rows[slot] = ptrs, rows
        self.staged[slot] = True
        return True

    def launch(self, weights: Sequence[float], scales: Sequence[float] | None = None,
               order: Sequence[int] | None = None, deltas: bool = False, gather: bool = False) -> None:
        """Enqueue every GPU's bucket kernel, then the per-bucket D2H (and the all-gather if ``gather``)."""
        order = list(range(len(weights))) if order is None else list(order)
        if len(order) != len(weights):
            raise ValueError("order and weights must have the same length")
        for slot in order:
            if not (0 <= slot < self.capacity and self.staged[slot]):
                raise ValueError(f"client slot {slot} was not staged")
        if not deltas and not self.has_baseline:
            raise ValueError("baseline not staged")
        if deltas and self.codec != "native":
            raise ValueError("deltas are fp32 (x - b promotes coded payloads); use the native codec")
        if scales is not None and len(scales) != len(weights):
            raise ValueError("scales must have one entry per client")
        # delta arenas: acc = sum_i d_i * w_i per bucket (the deltas-form kernel), then b + acc
        # (plato_agg_update_weights: the fused epilogue's sum)
        update = self.deltas and not deltas
        eng = self.engine
        k = len(order)
        self._k = k
        w_host = torch.from_numpy(fp32_weights(weights)).pin_memory()
        s_host = None if scales is None else torch.from_numpy(fp32_weights(scales)).pin_memory()
        host_f, host_i = eng._results.get()
        keep = [w_host, s_host]
        self.timings["stage_ms"] = (time.perf_counter() - self._t0) * 1e3
        self.events, kernel_events = [], []
        outs = []
        for s in eng._shards:
            pf = np.asarray([self._ptrs[i][s.index][0] for i in order], dtype=np.int64)
            pi = np.asarray([self._ptrs[i][s.index][1] for i in order], dtype=np.int64)
            with torch.cuda.device(s.device), torch.cuda.stream(s.stream):
                s.stream.wait_stream(s.copy_stream)
                w = w_host.to(s.device, non_blocking=True)
                sc = None if s_host is None else s_host.to(s.device, non_blocking=True)
                tf = torch.from_numpy(pf).pin_memory().to(s.device, non_blocking=True)
                ti = torch.from_numpy(pi).pin_memory().to(s.device, non_blocking=True)
                out_f = torch.empty(s.per, dtype=torch.float32, device=s.device)
                out_i = torch.empty(max(s.ni, 1), dtype=torch.float32, device=s.device)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s.stream)
                h = s.stream.cuda_stream
                n_i = s.ni
                if self.codec == "bf16":
                    _lib.call("plato_agg_fedavg_weights_bf16", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w),
                              _ptr(sc), k, _ptr(s.base_f), _ptr(s.base_i) if n_i else None, _ptr(out_f),
                              _ptr(out_i) if n_i else None, s.n, n_i, h)
                elif update:
                    acc_f = torch.empty(s.per, dtype=torch.float32, device=s.device)
                    acc_i = torch.empty(max(s.ni, 1), dtype=torch.float32, device=s.device)
                    _lib.call("plato_agg_fedavg_deltas", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w), _ptr(sc),
                              k, _ptr(acc_f), _ptr(acc_i) if n_i else None, s.n, n_i, h)
                    _lib.call("plato_agg_update_weights", _ptr(s.base_f), _ptr(s.base_i) if n_i else None,
                              _ptr(acc_f), _ptr(acc_i) if n_i else None, _ptr(out_f), _ptr(out_i) if n_i else None,
                              s.n, n_i, h)
                    keep.extend((acc_f, acc_i))
                elif eng.variant is not None:
                    _lib.tune_call("plato_agg_tune_fedavg", eng.variant, int(not deltas), _ptr(tf),
                              _ptr(ti) if n_i else None, _ptr(w), _ptr(sc), k,
                              None if deltas else _ptr(s.base_f), None if (deltas or not n_i) else _ptr(s.base_i),
                              _ptr(out_f), _ptr(out_i) if n_i else None, s.n, n_i, h)
                elif deltas:
                    _lib.call("plato_agg_fedavg_deltas", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w), _ptr(sc),
                              k, _ptr(out_f), _ptr(out_i) if n_i else None, s.n, n_i, h)
                else:
                    _lib.call("plato_agg_fedavg_weights", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w), _ptr(sc),
                              k, _ptr(s.base_f), _ptr(s.base_i) if n_i else None, _ptr(out_f),
                              _ptr(out_i) if n_i else None, s.n, n_i, h)
                e1.record(s.stream)
                kernel_events.append((e0, e1))
                keep.extend((w, sc, tf, ti))
                outs.append((out_f, out_i))
        if gather:
            self._device_results = self._gather(outs)
        for s, (out_f, out_i) in zip(eng._shards, outs):
            with torch.cuda.device(s.device), torch.cuda.stream(s.stream):
                if s.n:
                    host_f[s.lo:s.hi].copy_(out_f[: s.n], non_blocking=True)
                if s.ni:
                    host_i[s.ilo:s.ihi].copy_(out_i[: s.ni], non_blocking=True)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(s.stream)
                self.events.append(ev)
        self._kernel_events = kernel_events
        self._out = (host_f, host_i)
        self._keep = (keep, outs)

    def _gather(self, outs):
        """Every GPU gets the whole new model: RCCL all-gather of the buckets (device copies if GPUs repeat)."""
        eng = self.engine
        per, world = eng._plan.per, eng.world
        fulls = [torch.empty(per * world, dtype=torch.float32, device=s.device) for s in eng._shards]
        comm = eng.comm() if world > 1 else None
        if comm is not None:
            send = (ctypes.c_void_p * world)(*[o[0].data_ptr() for o in outs])
            recv = (ctypes.c_void_p * world)(*[f.data_ptr() for f in fulls])
            streams = (ctypes.c_void_p * world)(*[s.stream.cuda_stream for s in eng._shards])
            _lib.call("plato_agg_comm_allgather_f32", comm, ctypes.cast(send, ctypes.c_void_p),
                      ctypes.cast(recv, ctypes.c_void_p), per, ctypes.cast(streams, ctypes.c_void_p))
        else:
            for g, s in enumerate(eng._shards):
                with torch.cuda.device(s.device), torch.cuda.stream(s.stream):
                    for r, src in enumerate(eng._shards):
                        if r != g:
                            s.stream.wait_stream(src.stream)
                        fulls[g][r * per:(r + 1) * per].copy_(outs[r][0], non_blocking=True)
        ints = []
        s0 = eng._shards[0]
        for s in eng._shards:
            with torch.cuda.device(s.device), torch.cuda.stream(s.stream):
                s.stream.wait_stream(s0.stream)
                ints.append(outs[0][1][: s0.ni].to(s.device, non_blocking=True))
        return [(f[: self.layout.n_f32], i) for f, i in zip(fulls, ints)]

    def device_result(self, g: int = 0):
        """(fp32 arena, fp32 values of the int64 entries) of the new model on GPU ``g`` (``gather=True``)."""
        if self._device_results is None:
            raise RuntimeError("launch(..., gather=True) first")
        return self._device_results[g]

    def algorithmic_bytes(self) -> int:
        return self.layout.algorithmic_bytes(self._k)

    def ready(self) -> bool:
        return bool(self.events) and all(ev.query() for ev in self.events)

    def wait(self) -> None:
        for ev in self.events:
            ev.synchronize()

    def result(self) -> "OrderedDict[str, torch.Tensor]":
        if not self.events:
            raise RuntimeError("launch() first")
        self.wait()
        self.timings["kernel_ms"] = max(a.elapsed_time(b) for a, b in self._kernel_events)
        self.timings["d2h_ms"] = max(b.elapsed_time(ev) for (_, b), ev in zip(self._kernel_events, self.events))
        self.timings["total_ms"] = (time.perf_counter() - self._t0) * 1e3
        host_f, host_i = self._out
        self._out = None
        self._keep = None
        return self.layout.unpack(host_f, host_i)


# --------------------------------------------------------------- client-split reductions
class ClientShardedEngine:
    """The devices of a :class:`MultiDeviceEngine` for rounds whose weights reduce the whole model per client.

    FedAdp's dots (fedadp_server.py:91-99) and Port's similarity (port_server.py:36-52) are one serial
    fma chain per (client, chain) over the flattened model: a bucket cut would reorder the chain, a
    client cut does not.  Same surface as an engine (``begin`` / ``prestage`` / ``release_arrivals``);
    the rounds are :class:`ClientRound`.
    """

    def __init__(self, multi: MultiDeviceEngine):
        self.multi = multi

    @property
    def world(self) -> int:
        return self.multi.world

    @property
    def devices(self):
        return self.multi.devices

    @property
    def device(self) -> torch.device:
        return self.multi.device

    def begin(self, template, capacity: int, codec: str = "native") -> "ClientRound":
        return self.multi.begin(template, capacity, codec, client_split=True)

    def prestage(self, payload, baseline_layout: ArenaLayout, baseline=None) -> bool:
        return self.multi.prestage(payload, baseline_layout, baseline)

    def release_arrivals(self) -> None:
        self.multi.release_arrivals()


class ClientRound(MultiRound):
    """A bucket-sharded round whose whole-model reductions are split by client over the devices.

    Staging (N PCIe links, each carrying 1/N of every payload) and the final FedAvg launch are the
    :class:`MultiRound`'s.  For the reductions, client slot j's whole arena is assembled on device
    j mod N from the bucket shards (device-to-device copies over xGMI) into a single-GPU
    :class:`~plato_amd.engine.AggregationRound` per device, with the baseline; FedAdp's global
    gradient is formed bucket-sharded (``plato_agg_fedavg_entrywise`` per bucket, the same
    per-element arithmetic as one GPU) and all-gathered to every device; then each device runs the
    single-GPU kernels (``plato_agg_fedadp_dots``, ``plato_agg_port_norms`` + cosine sums) on its
    own clients.  Every value is computed by one chain on one GPU: bit-identical to one GPU.
    """

    def __init__(self, engine: MultiDeviceEngine, layout: ArenaLayout, capacity: int, codec: str):
        super().__init__(engine, layout, capacity, codec)
        self._baseline_sd = None
        self._split = None  # [(AggregationRound on device g, {slot: local slot})]
        self.last_norms = None

    def put_baseline(self, baseline) -> None:
        super().put_baseline(baseline)
        self._baseline_sd = baseline
        self._split = None

    def put_client(self, slot: int, payload, what: str = "weights_received") -> None:
        super().put_client(slot, payload, what)
        self._split = None

    def adopt(self, slot: int, payload) -> bool:
        ok = super().adopt(slot, payload)
        if ok:
            self._split = None
        return ok

    def decoded(self) -> "ClientRound":
        return self  # native payloads only (coded rounds run on the primary device)

    # ------------------------------------------------------------ client split
    def _client_rounds(self):
        """Per device g: a single-GPU round holding the whole arenas of the staged slots j = g mod N.

        Enqueued, never waited for on the host.  Each bucket's current stream first waits for its copy
        stream (the H2D of the buckets); then, per (destination, bucket), ONE strided device-to-device
        copy moves that bucket of every client the destination owns (their rows are equally spaced in
        the bucket's slab; rows adopted from arrival slabs fall back to a copy per row).  torch orders a
        cross-device copy after the current streams of both devices and makes the destination's current
        stream wait for it, so the reductions that follow on each device's current stream see the
        assembled arenas without a host synchronisation.  Destination device g then holds its clients'
        whole arenas next to its bucket shard (memory: one extra copy of the clients, split over the GPUs).
        ``timings["client_assembly_ms"]``: the longest destination's span (HIP events), filled once the
        reductions have synchronised.
        """
        if self._split is not None:
            return self._split
        if self._baseline_sd is None:
            raise ValueError("baseline not staged")
        eng = self.engine
        world = eng.world
        staged = [j for j in range(self.capacity) if self.staged[j]]
        for sh in eng._shards:  # this round's bucket copies (copy streams) before any read of them
            torch.cuda.current_stream(sh.device).wait_stream(sh.copy_stream)

        def build(g):
            mine = [j for j in staged if j % world == g]
            dev = eng.devices[g]
            e = eng.client_engine(g)
            with torch.cuda.device(dev):
                r = e.begin(self._baseline_sd, max(1, len(mine)), "native")
                if r.layout.signature != self.layout.signature:
                    raise RuntimeError("client engine built another arena layout")
                r.deltas = self.deltas  # the assembled rows are what the bucket rows hold: deltas or weights
                here = torch.cuda.current_stream(dev)
                here.wait_stream(e._copy_stream)  # the previous round's copies into this engine's slab
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(here)
                for sh in eng._shards:  # the baseline, bucket by bucket
                    if sh.n:
                        e._base.f32[sh.lo:sh.hi].copy_(sh.base_f[: sh.n], non_blocking=True)
                    if sh.ni:
                        e._base.i64[sh.ilo:sh.ihi].copy_(sh.base_i[: sh.ni], non_blocking=True)
                r.has_baseline = True
                if mine:
                    for sh in eng._shards:
                        if sh.n:
                            _copy_rows(r.slab.f32[: len(mine), sh.lo:sh.hi],
                                       [self._rows[j][sh.index][0][: sh.n] for j in mine])
                        if sh.ni:
                            _copy_rows(r.slab.i64[: len(mine), sh.ilo:sh.ihi],
                                       [self._rows[j][sh.index][1][: sh.ni] for j in mine])
                e1.record(here)
                pf, pi = r.slab.row_pointers(range(len(mine)))
                for local in range(len(mine)):
                    r._pf[local], r._pi[local] = int(pf[local]), int(pi[local])
                    r.staged[local] = True
            return r, {j: local for local, j in enumerate(mine)}, (e0, e1)

        built = eng.each(build, range(world))
        self._assembly_events = [b[2] for b in built]
        self._split = [(b[0], b[1]) for b in built]
        return self._split

    def _resolve_assembly(self) -> None:
        """``timings["client_assembly_ms"]`` once the devices have passed the assembly (after a reduction's sync)."""
        evs = getattr(self, "_assembly_events", None)
        if evs and all(e1.query() for _, e1 in evs):
            self.timings["client_assembly_ms"] = max(e0.elapsed_time(e1) for e0, e1 in evs)
            self._assembly_events = None

    def _by_device(self, slots):
        """[(device g, [local slots], [positions in ``slots``])] for the devices holding some of ``slots``."""
        split = self._client_rounds()
        groups = []
        for g, (_, where) in enumerate(split):
            pos = [i for i, j in enumerate(slots) if j in where]
            if pos:
                groups.append((g, [where[slots[i]] for i in pos], pos))
        missing = [j for j in slots if not any(j in where for _, where in split)]
        if missing:
            raise ValueError(f"client slots {missing} were not staged")
        return groups

    def launch_entrywise(self, weights: np.ndarray, order: Sequence[int] | None = None, scale: float = 1.0,
                         noise=None, noise_scale: float = 0.0, add_base: bool = True, deltas: bool = False,
                         device: bool = False):
        """``plato_agg_fedavg_entrywise`` per bucket, all-gathered: [(fp32 arena, int64 values)] per device.

        The device-resident form FedAdp's global gradient takes (``device=True``; no noise, not in deltas mode).
        """
        if not device or noise is not None or deltas:
            raise ValueError("client-split rounds offer the device-resident entrywise sum only (FedAdp)")
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        if self.deltas and add_base:
            raise ValueError("launch_entrywise(add_base=True) reads the clients' weights; this round holds deltas")
        rows_are_deltas = self.deltas  # the kernel's deltas form: no baseline read
        eng, lay = self.engine, self.layout
        n_e = len(lay.entries)
        order = list(range(np.asarray(weights).shape[1])) if order is None else list(order)
        for j in order:
            if not (0 <= j < self.capacity and self.staged[j]):
                raise ValueError(f"client slot {j} was not staged")
        k = len(order)
        w = np.ascontiguousarray(np.asarray(weights, dtype=np.float64).astype(np.float32))
        if w.shape != (n_e, k):
            raise ValueError(f"weights must be [entries={n_e}, clients={k}], got {w.shape}")
        tables = self._bucket_chunks()
        outs, keep = [], []
        for s, (cf, ci) in zip(eng._shards, tables):
            with torch.cuda.device(s.device), torch.cuda.stream(s.stream):
                s.stream.wait_stream(s.copy_stream)
                tf = torch.from_numpy(np.asarray([self._ptrs[j][s.index][0] for j in order], dtype=np.int64)).to(s.device)
                ti = torch.from_numpy(np.asarray([self._ptrs[j][s.index][1] for j in order], dtype=np.int64)).to(s.device)
                dw = torch.from_numpy(w).to(s.device)
                dcf = torch.from_numpy(cf.view(np.int32)).to(s.device)
                dci = torch.from_numpy(ci.view(np.int32)).to(s.device)
                out_f = torch.empty(s.per, dtype=torch.float32, device=s.device)
                out_i = torch.empty(max(s.ni, 1), dtype=torch.float32, device=s.device)
                ncf, nci = int(cf.shape[0]), int(ci.shape[0])
                if ncf or nci:
                    _lib.call("plato_agg_fedavg_entrywise", _ptr(tf), _ptr(ti) if s.ni else None, k, _ptr(dw), n_e,
                              _ptr(dcf) if ncf else None, ncf, _ptr(dci) if nci else None, nci,
                              None if rows_are_deltas else _ptr(s.base_f),
                              None if (rows_are_deltas or not s.ni) else _ptr(s.base_i), None, None, float(scale),
                              float(noise_scale), _lib.PLATO_AGG_ADD_BASE if add_base else 0, _ptr(out_f),
                              _ptr(out_i) if s.ni else None, s.n, s.ni, s.stream.cuda_stream)
                outs.append((out_f, out_i))
                keep.append((tf, ti, dw, dcf, dci))
        fulls = self._gather(outs)
        for s in eng._shards:  # the reductions run on each device's current stream: order them after the gather
            torch.cuda.current_stream(s.device).wait_stream(s.stream)
        self._keep_entrywise = keep  # stream-ordered inputs: alive until the next launch
        return fulls

    def _bucket_chunks(self):
        """Per bucket: (fp32, int64) ``plato_agg_chunk`` tables of the layout's entries cut to the bucket."""
        eng, lay = self.engine, self.layout
        key = ("bucket_chunks", eng.world, FedAvgEngine.ENTRYWISE_CHUNK)
        hit = lay._cache.get(key)
        if hit is None:
            cap = FedAvgEngine.ENTRYWISE_CHUNK
            hit = []
            for s in eng._shards:
                f32, i64 = [], []
                for idx, e in enumerate(lay.entries):
                    if e.numel == 0:
                        continue
                    if e.region != "f32":
                        if s.ni:
                            i64.append((idx, e.offset, e.offset + e.numel, 0))
                        continue
                    lo, end = max(e.offset, s.lo), min(e.offset + e.numel, s.hi)
                    while lo < end:  # cuts at multiples of cap of the arena (s.lo is a multiple of 64)
                        hi = min(end, (lo // cap + 1) * cap)
                        f32.append((idx, lo - s.lo, hi - s.lo, 0))
                        lo = hi
                hit.append((np.asarray(f32, dtype=np.uint32).reshape(-1, 4),
                            np.asarray(i64, dtype=np.uint32).reshape(-1, 4)))
            lay._cache[key] = hit
        return hit

    def fedadp_dots(self, grads, slots: Sequence[int], lr: float):
        """``AggregationRound.fedadp_dots`` on every device for its clients (``grads``: launch_entrywise's)."""
        slots = list(slots)
        groups = self._by_device(slots)
        split = self._split

        def run(item):
            g, local, _ = item
            with torch.cuda.device(self.engine.devices[g]):
                return split[g][0].fedadp_dots(grads[g], local, lr)

        parts = self.engine.each(run, groups)
        self._resolve_assembly()
        inner = np.zeros(len(slots), dtype=np.float32)
        l_sq = np.zeros(len(slots), dtype=np.float32)
        for (g, _, pos), (xy, gg, yy) in zip(groups, parts):
            inner[pos] = xy
            l_sq[pos] = yy
        g_sq = parts[0][1]  # the same g . g on every device (one chain, the same g)
        self.timings["fedadp_dots_ms"] = max(split[g][0].timings.get("fedadp_dots_ms", 0.0) for g, _, _ in groups)
        return inner, g_sq, l_sq

    def model_similarities(self, reference, slots: Sequence[int], eps: float = 1e-8, threads: int | None = None,
                           flat_norms: bool = False) -> list:
        """``AggregationRound.model_similarities`` on every device for its clients (Port)."""
        slots = list(slots)
        if not slots:
            return []
        threads = torch.get_num_threads() if threads is None else int(threads)
        groups = self._by_device(slots)
        split = self._split

        def run(item):
            g, local, _ = item
            with torch.cuda.device(self.engine.devices[g]):
                rnd = split[g][0]
                sims = rnd.model_similarities(reference, local, eps, threads, flat_norms)
                return sims, rnd.last_norms

        parts = self.engine.each(run, groups)
        self._resolve_assembly()
        sims = [None] * len(slots)
        norms = np.zeros(len(slots) + 1, dtype=np.float32)
        for (g, _, pos), (vals, dev_norms) in zip(groups, parts):
            for i, v in zip(pos, vals):
                sims[i] = v
            norms[0] = dev_norms[0]  # current - previous: the same on every device
            norms[[1 + i for i in pos]] = dev_norms[1:]
        self.last_norms = norms
        for key in ("port_norms_ms", "port_cosine_ms"):
            vals = [split[g][0].timings[key] for g, _, _ in groups if key in split[g][0].timings]
            if vals:
                self.timings[key] = max(vals)
        return sims


# --------------------------------------------------------------- entry-aligned shards
def _sub_payload(payload, names: Sequence[str]):
    """The entries ``names`` of a payload (same tensors, no copy); QSGD payloads keep their scales."""
    from .processors.qsgd import QsgdPayload

    if getattr(payload, "plato_codec", None) == "qsgd":
        return QsgdPayload(((n, payload[n]) for n in names), max_v={n: payload.max_v[n] for n in names},
                           shapes={n: payload.shapes[n] for n in names}, level=payload.level)
    return OrderedDict((n, payload[n]) for n in names)


class EntryShardedEngine:
    """The devices of a :class:`MultiDeviceEngine`, sharded by whole entries (:class:`EntryPlan`).

    Shard g is a single-GPU :class:`~plato_amd.engine.FedAvgEngine` on device g
    that sees only its contiguous group of the model's entries: payloads are
    split by key (the tensors are not copied), each shard packs and copies its
    entries on its own copy stream (N PCIe links), and every single-GPU round
    operation — the FedAvg launches of every codec, the decode of coded slots,
    ``entry_norms`` / ``entry_stats`` / ``np_sumsq`` / ``launch_entrywise`` —
    runs per shard, concurrently, on one worker thread per shard.  Same
    surface as an engine: ``begin`` / ``prestage`` / ``release_arrivals``.
    """

    def __init__(self, multi: MultiDeviceEngine):
        self.multi = multi
        self.devices = multi.devices
        self.variant = multi.variant
        # shard 0 gets its own engine rather than the multi engine's primary: an engine keeps one
        # staging layout, and the primary's (the whole model, for codecs staged on one GPU) and
        # shard 0's (its entries) would evict each other's arenas and arrivals every round
        self._engines = [FedAvgEngine(d, variant=multi.variant) for d in self.devices]
        for eng in self._engines:
            eng.delta_arenas = multi.delta_arenas
        self._plans: dict = {}
        self._arrivals: dict = {}
        self._pool = None

    @property
    def world(self) -> int:
        return len(self.devices)

    @property
    def device(self) -> torch.device:
        return self.devices[0]

    def plan(self, layout: ArenaLayout) -> tuple[EntryPlan, list]:
        """(plan, [(shard, entry names)] of the non-empty shards) for ``layout`` (cached by signature)."""
        hit = self._plans.get(layout.signature)
        if hit is None:
            plan = EntryPlan.for_layout(layout, self.world)
            parts = [(g, plan.names(layout, g)) for g in range(self.world) if plan.groups[g][1] > plan.groups[g][0]]
            hit = self._plans[layout.signature] = (plan, parts)
        return hit

    def each(self, fn, items):
        """``[fn(item) ...]`` with one worker thread per shard (torch / HIP calls release the GIL)."""
        items = list(items)
        if len(items) <= 1:
            return [fn(x) for x in items]
        if self._pool is None:
            import concurrent.futures

            self._pool = concurrent.futures.ThreadPoolExecutor(self.world, thread_name_prefix="plato-amd-shard")
        return list(self._pool.map(fn, items))

    def begin(self, template, capacity: int, codec: str = "native") -> "EntryRound":
        if capacity <= 0:
            raise ValueError("no client payloads to aggregate")
        if isinstance(template, ArenaLayout):
            raise TypeError("begin() needs the baseline state_dict (its tensors define every shard's arena)")
        layout = ArenaLayout.from_state_dict(template)
        _, parts = self.plan(layout)

        def start(part):
            g, names = part
            with torch.cuda.device(self.devices[g]):
                return self._engines[g].begin(OrderedDict((n, template[n]) for n in names), capacity, codec)

        return EntryRound(self, layout, [(g, names) for g, names in parts], self.each(start, parts), codec)

    def prestage(self, payload, baseline_layout: ArenaLayout, baseline=None) -> bool:
        """Copy each shard's entries of an arriving payload to its GPU now (adopted by the next round).

        ``baseline`` (the server's current model): with delta arenas each shard turns its entries into
        deltas against that model's entries at arrival (FedAvgEngine.prestage per shard)."""
        codec = payload_codec(payload)
        try:
            baseline_layout.check_compatible(payload, "arriving payload", codec)
        except (KeyError, ValueError):
            return False
        _, parts = self.plan(baseline_layout)
        subs = [_sub_payload(payload, names) for _, names in parts]
        try:
            bases = [None if baseline is None else OrderedDict((n, baseline[n]) for n in names) for _, names in parts]
        except KeyError:  # not the model these payloads update: arrivals stay weights
            bases = [None] * len(parts)
        done = []
        for (g, names), sub, base in zip(parts, subs, bases):
            lay = self._sub_layout(baseline_layout, names)
            with torch.cuda.device(self.devices[g]):
                if not self._engines[g].prestage(sub, lay, base):
                    for g0, sub0 in done:  # no half-staged payload keeps slots on the other shards
                        self._engines[g0].drop_arrival(sub0)
                    return False
            done.append((g, sub))
        self._arrivals[id(payload)] = (payload, payload_fingerprint(payload), subs)
        return True

    def _sub_layout(self, layout: ArenaLayout, names) -> ArenaLayout:
        key = ("entry_sub_layout", tuple(names))
        hit = layout._cache.get(key)
        if hit is None:
            hit = layout._cache[key] = ArenaLayout.from_shapes([(layout[n].name, layout[n].shape, layout[n].region)
                                                                for n in names])
        return hit

    def _arrival_subs(self, payload):
        hit = self._arrivals.get(id(payload))
        if hit is None or hit[0] is not payload or hit[1] != payload_fingerprint(payload):
            return None  # not prestaged here, or edited after arrival: the round stages its current tensors
        return hit[2]

    def _release(self) -> None:
        self._arrivals = {}
        for eng in self._engines:
            eng.release_arrivals()

    def release_arrivals(self) -> None:
        self.multi.release_arrivals()


class EntryRound:
    """One entry-sharded round: a single-GPU round per shard over its entries, results in layout order.

    Per-entry outputs are concatenated along the entry axis (``entry_norms``
    [E, K], ``np_sumsq`` [K, E], ``entry_stats``); model results are merged
    key by key in baseline order.  Whole-model flattened reductions (FedAdp's
    dots, Port's similarity) are not entry-local and are not offered here.
    """

    def __init__(self, engine: EntryShardedEngine, layout: ArenaLayout, parts, rounds, codec: str):
        self.engine = engine
        self.layout = layout
        self.codec = codec
        self._parts = parts          # [(shard, entry names)]
        self._rounds = rounds        # the shards' AggregationRounds (or their decoded views)
        self.capacity = rounds[0].capacity
        self.timings: dict = {}
        self._t0 = time.perf_counter()
        self._k = 0
        self._decoded = None

    def _each(self, fn):
        eng = self.engine

        def run(i):
            g = self._parts[i][0]
            with torch.cuda.device(eng.devices[g]):
                return fn(i, self._rounds[i])

        return eng.each(run, range(len(self._rounds)))

    def _split(self, state_dict):
        return [_sub_payload(state_dict, names) for _, names in self._parts]

    @property
    def has_baseline(self) -> bool:
        return all(r.has_baseline for r in self._rounds)

    @property
    def staged(self) -> list:
        return [all(r.staged[s] for r in self._rounds) for s in range(self.capacity)]

    # ------------------------------------------------------------ staging
    def put_baseline(self, baseline) -> None:
        self.layout.check_compatible(baseline, "baseline_weights")
        subs = self._split(baseline)
        self._each(lambda i, r: r.put_baseline(subs[i]))
        self._decoded = None

    def put_client(self, slot: int, payload, what: str = "weights_received") -> None:
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        self.layout.check_compatible(payload, f"{what}[{slot}]", self.codec)
        subs = self._split(payload)
        self._each(lambda i, r: r.put_client(slot, subs[i], what))
        self._decoded = None

    def adopt(self, slot: int, payload) -> bool:
        subs = self.engine._arrival_subs(payload)
        if subs is None or len(subs) != len(self._rounds):
            return False
        if not all(self._each(lambda i, r: r.adopt(slot, subs[i]))):
            return False  # some shard's copy is stale: the caller stages the payload whole
        self._decoded = None
        return True

    def decoded(self) -> "EntryRound":
        """Coded slots decoded per shard into fp32 rows (AggregationRound.decoded); native: this round."""
        if self.codec == "native":
            return self
        if self._decoded is None:
            rounds = self._each(lambda i, r: r.decoded())
            self._decoded = EntryRound(self.engine, self.layout.promoted(), self._parts, rounds, "native")
        return self._decoded

    # ------------------------------------------------------ per-entry reductions
    def entry_norms(self, slots: Sequence[int]) -> np.ndarray:
        slots = list(slots)
        return np.concatenate(self._each(lambda i, r: r.entry_norms(slots)), axis=0)

    def np_sumsq(self, slots: Sequence[int]) -> np.ndarray:
        slots = list(slots)
        return np.concatenate(self._each(lambda i, r: r.np_sumsq(slots)), axis=1)

    def entry_stats(self, slots: Sequence[int], v: tuple | None = None, deltas: bool = False):
        if v is not None:
            raise ValueError("entry_stats with a device vector runs on one GPU")
        slots = list(slots)
        outs = self._each(lambda i, r: r.entry_stats(slots, None, deltas))
        return None, np.concatenate([o[1] for o in outs], axis=1), None

    def _rows(self):
        """Entry rows of each shard in the layout (a shard's entries are contiguous)."""
        rows, lo = [], 0
        for _, names in self._parts:
            rows.append((lo, lo + len(names)))
            lo += len(names)
        return rows

    def launch_entrywise(self, weights: np.ndarray, order: Sequence[int] | None = None, scale: float = 1.0,
                         noise: Mapping[str, torch.Tensor] | None = None, noise_scale: float = 0.0,
                         add_base: bool = True, deltas: bool = False, device: bool = False):
        if device:
            raise ValueError("device-resident entrywise results stay on one GPU (FedAdp runs on the primary)")
        w = np.asarray(weights)
        if w.shape[0] != len(self.layout.entries):
            raise ValueError(f"weights must be [entries={len(self.layout.entries)}, clients], got {w.shape}")
        rows = self._rows()
        noises = None if noise is None else self._split(noise)
        self._t0 = time.perf_counter()
        self._each(lambda i, r: r.launch_entrywise(w[rows[i][0]:rows[i][1]], order, scale,
                                                   None if noises is None else noises[i], noise_scale,
                                                   add_base, deltas))
        self._k = w.shape[1]

    # --------------------------------------------------------- FedAvg launches
    def launch(self, weights: Sequence[float], scales: Sequence[float] | None = None,
               order: Sequence[int] | None = None, deltas: bool = False) -> None:
        self._each(lambda i, r: r.launch(weights, scales, order, deltas))
        self._k = len(weights)

    def launch_w64(self, weights64: Sequence[float], weights_i64: Sequence[float] | None = None,
                   order: Sequence[int] | None = None, deltas: bool = False) -> None:
        self._each(lambda i, r: r.launch_w64(weights64, weights_i64, order, deltas))
        self._k = len(weights64)

    def ready(self) -> bool:
        return all(r.ready() for r in self._rounds)

    def wait(self) -> None:
        for r in self._rounds:
            r.wait()

    def algorithmic_bytes(self) -> int:
        return sum(r.layout.algorithmic_bytes(self._k) for r in self._rounds)

    def result(self) -> "OrderedDict[str, torch.Tensor]":
        parts = self._each(lambda i, r: r.result())
        merged = {}
        for p in parts:
            merged.update(p)
        self.timings = {
            "stage_ms": max(r.timings.get("stage_ms", 0.0) for r in self._rounds),
            "kernel_ms": max(r.timings.get("kernel_ms", 0.0) for r in self._rounds),
            "d2h_ms": max(r.timings.get("d2h_ms", 0.0) for r in self._rounds),
            "total_ms": (time.perf_counter() - self._t0) * 1e3,
        }
        return OrderedDict((n, merged[n]) for n in self.layout.keys())

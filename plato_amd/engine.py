"""Device engine: HBM arenas, host staging and launches of the HIP kernels.

This is the host half of the drop-in boundary.  It takes what Plato's server
hands to its aggregation hooks (CPU ``state_dict`` payloads in
``self.updates`` order, the baseline from ``algorithm.extract_weights()``,
per-client weights) and returns what the reference would return, computed by
``libplato_agg.so`` on the GPU:

* :meth:`FedAvgEngine.aggregate_weights` — the fused deltas -> weighted sum ->
  update chain (``plato/servers/fedavg.py:184-194``), i.e. the value an
  ``aggregate_weights`` hook must produce (``servers/fedavg.py:171-182``).
* :meth:`FedAvgEngine.aggregate_deltas` — ``Server.aggregate_deltas``
  (``servers/fedavg.py:137-159``) for variants that compute their own deltas.
* :meth:`FedAvgEngine.compute_weight_deltas` / :meth:`update_weights` /
  :meth:`mix_weights` — ``algorithms/fedavg.py:13-37`` and FedAsync's
  ``fedasync_algorithm.py:9-20``.

Everything device-side goes through the C ABI; nothing here computes model
arithmetic on the CPU.
"""

from __future__ import annotations

import time
from collections import OrderedDict
from typing import Mapping, Sequence

import numpy as np
import torch

from . import _lib
from .arena import CODECS, F32, I64, ArenaLayout, fedadp_order, payload_codec, same_f32_bits
from .staging import HostPacker, PinnedRing, ResultPool, arena_source, baseline_key, payload_fingerprint


def fp32_weights(values: Sequence[float]) -> np.ndarray:
    """Round Python (double) weights to fp32 the way torch's scalar path does.

    ``delta * (n_i / N)`` multiplies an fp32 tensor by a Python float; torch
    converts the double scalar to the fp32 compute type (round to nearest even)
    before the multiply (measured).
    """
    out = np.empty(len(values), dtype=np.float32)
    for i, v in enumerate(values):
        if isinstance(v, torch.Tensor):
            raise TypeError("aggregation weights must be Python numbers, not tensors")
        out[i] = np.float32(float(v))
    return out


def fedavg_weights(num_samples: Sequence[int]) -> list[float]:
    """``n_i / N`` as the reference computes it (``servers/fedavg.py:140,154``)."""
    total = sum(num_samples)
    return [n / total for n in num_samples]


def require_device(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError(
            "plato_amd: no ROCm GPU visible; the aggregation engine runs only on the "
            "HIP path (there is no CPU fallback)"
        )
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"plato_amd: device must be a GPU, got {dev}")
    return dev


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream_handle(stream: torch.cuda.Stream) -> int:
    return stream.cuda_stream


class DeviceArena:
    """One model arena in HBM: fp32 region + int64 region (+ fp32 view of int64 results)."""

    def __init__(self, layout: ArenaLayout, device: torch.device, i64_dtype: torch.dtype = torch.int64):
        self.layout = layout
        self.f32 = torch.empty(layout.row_f32, dtype=torch.float32, device=device)
        self.i64 = torch.empty(layout.row_i64, dtype=i64_dtype, device=device)


class ClientSlab:
    """K client arenas in HBM as two row-major slabs ``[cap, row]``.

    ``codec`` selects the element types the payloads arrive in (arena.CODECS):
    bf16 payloads stay bf16 in HBM (half the bytes) and are widened by the kernel.
    """

    def __init__(self, layout: ArenaLayout, capacity: int, device: torch.device, codec: str = "native"):
        self.layout = layout
        self.capacity = capacity
        self.codec = codec
        dt_f, dt_i = CODECS[codec]
        self.f32 = torch.empty((capacity, layout.row_f32), dtype=dt_f, device=device)
        self.i64 = torch.empty((capacity, layout.row_i64), dtype=dt_i, device=device)

    def row_pointers(self, rows: Sequence[int]) -> tuple[np.ndarray, np.ndarray]:
        base_f = self.f32.data_ptr()
        base_i = self.i64.data_ptr()
        sf = self.f32.stride(0) * self.f32.element_size()
        si = self.i64.stride(0) * self.i64.element_size()
        rows = np.asarray(rows, dtype=np.int64)
        return (base_f + rows * sf).astype(np.int64), (base_i + rows * si).astype(np.int64)


class _Stager:
    """Pinned host ring: packs CPU ``state_dict``s natively and copies them H2D.

    Packing client j+1 (``plato_ingest_pack`` on the native copy pool) overlaps
    the H2D copy of client j on a dedicated copy stream; arena-backed payloads
    (native ingestion) are copied from their pinned arena without a pack.
    """

    def __init__(self, layout: ArenaLayout, device: torch.device, depth: int = 4, codec: str = "native",
                 stream: torch.cuda.Stream | None = None):
        self.layout = layout
        self.codec = codec
        self.stream = stream or torch.cuda.Stream(device)
        self.ring = PinnedRing(layout, codec, depth)
        self.packer = HostPacker(layout, codec)

    def put(self, state_dict: Mapping[str, torch.Tensor], dst_f32: torch.Tensor,
            dst_i64: torch.Tensor) -> None:
        n_f, n_i = self.layout.n_f32, self.layout.n_i64
        src = arena_source(state_dict, self.layout, self.codec)
        if src is not None:
            # already laid out as the arena, in pinned memory (plato_amd.ingest.loads): DMA it as is
            arena_f, arena_i = src
            with torch.cuda.stream(self.stream):
                if n_f:
                    dst_f32[:n_f].copy_(arena_f[:n_f], non_blocking=True)
                if n_i:
                    dst_i64[:n_i].copy_(arena_i[:n_i], non_blocking=True)
            return
        with self.ring.lock:  # acquire -> pack -> copy -> fence as one step (executor vs event loop)
            j = self.ring.acquire()
            hf, hi = self.ring.slots[j]
            self.packer.pack(state_dict, hf, hi)
            with torch.cuda.stream(self.stream):
                if n_f:
                    dst_f32[:n_f].copy_(hf[:n_f], non_blocking=True)
                if n_i:
                    dst_i64[:n_i].copy_(hi[:n_i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.ring.fence(j, [ev])

    def fence(self, stream: torch.cuda.Stream) -> None:
        """Make ``stream`` wait for every copy issued so far."""
        stream.wait_stream(self.stream)


class FedAvgEngine:
    """HIP FedAvg aggregation on one GPU (one process per GPU)."""

    #: QSGD kernel variant (tuning / tests; None = the library default)
    qsgd_variant: int | None = None
    port_variant: int | None = None  # plato_agg_tune_port_norms shape (tests / tuning), None = the default
    #: arena alignment of the layouts this engine builds (arena.ALIGNMENTS; FedAdp servers: "fedadp")
    layout_align: str | None = None
    #: native rounds hold each client as its delta x - b (``AggregationRound.deltas``): FedAdp's servers,
    #: whose dot kernel then streams no baseline
    delta_arenas: bool = False

    def __init__(self, device=None, variant: int | None = None):
        self.device = require_device(device)
        self.lib = _lib.lib()
        self.variant = variant
        self._layout: ArenaLayout | None = None
        self._slabs: dict[str, ClientSlab] = {}
        self._stagers: dict[str, _Stager] = {}
        self._base: DeviceArena | None = None
        self._copy_stream: torch.cuda.Stream | None = None
        self._slab: ClientSlab | None = None      # slab of the current round's codec
        self._stager: _Stager | None = None       # native-dtype stager (baselines)
        self._arrivals: dict = {}                 # id(payload) -> staged arrival row
        self._arrival_free: dict = {}
        self._arrival_slabs: dict = {}

    # ----------------------------------------------------------- allocation
    def _prepare(self, template: Mapping[str, torch.Tensor], k: int, codec: str = "native") -> ArenaLayout:
        if codec not in CODECS:
            raise ValueError(f"unknown payload codec {codec!r}")
        layout = ArenaLayout.from_state_dict(template, align=self.layout_align)
        if self._layout is None or self._layout.signature != layout.signature:
            self._layout = layout
            self._slabs = {}
            self._stagers = {}
            self._base = None
            self._arrivals, self._arrival_free, self._arrival_slabs = {}, {}, {}
        layout = self._layout
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device)
        slab = self._slabs.get(codec)
        if slab is None or slab.capacity < k:
            self._slabs.pop(codec, None)
            slab = ClientSlab(layout, k, self.device, codec)
            self._slabs[codec] = slab
        for c in {"native", codec}:
            if c not in self._stagers:
                self._stagers[c] = _Stager(layout, self.device, codec=c, stream=self._copy_stream)
        if self._base is None:
            self._base = DeviceArena(layout, self.device)
        self._slab = slab
        self._stager = self._stagers["native"]
        return layout

    def _upload_weights(self, weights: Sequence[float], scales: Sequence[float] | None):
        w = torch.from_numpy(fp32_weights(weights)).to(self.device, non_blocking=False)
        s = None
        if scales is not None:
            if len(scales) != len(weights):
                raise ValueError("scales must have one entry per client")
            s = torch.from_numpy(fp32_weights(scales)).to(self.device, non_blocking=False)
        return w, s

    def _pointer_tables(self, pf: np.ndarray, pi: np.ndarray):
        tf = torch.from_numpy(pf).to(self.device)
        ti = torch.from_numpy(pi).to(self.device)
        return tf, ti

    # per-entry kernels: chunk capacity (elements) per workgroup
    STATS_CHUNK = 4096      # entry_stats: 256 lanes x 4 float4 groups
    QSGD_CHUNK = 4096       # fedavg_qsgd: 256 lanes x 2 x 8 one-byte codes (plato_agg_tune_qsgd_chunk(29))
    ENTRYWISE_CHUNK = 256  # fedavg_entrywise: 64 lanes x 1 float4 group (round 5: 0.891 vs 0.917 ms for 256 x 2, r05i_entrywise.log)

    def _chunks(self, layout: ArenaLayout, cap: int):
        """Device copies of ``layout.chunk_tables(cap)`` (cached per layout)."""
        key = ("dev_chunks", cap, str(self.device))
        hit = layout._cache.get(key)
        if hit is None:
            cf, ci = layout.chunk_tables(cap)
            hit = (torch.from_numpy(cf.view(np.int32).copy()).to(self.device),
                   torch.from_numpy(ci.view(np.int32).copy()).to(self.device))
            layout._cache[key] = hit
        return hit

    def _norm_tables(self, layout: ArenaLayout):
        """One piece per entry, longest first (``plato_agg_entry_norms_f32``).

        Each (client, entry) norm is one serial fma chain (torch's CPU order),
        so the launch lasts at least as long as the longest chain; starting the
        longest entries first lets the short ones fill in behind them instead
        of delaying them (ResNet's largest convolutions come last in
        ``state_dict`` order).  The output is indexed by each piece's entry, so
        the table order changes only the schedule.
        """
        key = ("dev_norm_tables", str(self.device))
        hit = layout._cache.get(key)
        if hit is None:
            ef, ei = layout.chunk_tables(1 << 32)
            ef = ef[np.argsort(-(ef[:, 2].astype(np.int64) - ef[:, 1]), kind="stable")] if len(ef) else ef
            hit = (torch.from_numpy(np.ascontiguousarray(ef).view(np.int32).copy()).to(self.device),
                   torch.from_numpy(np.ascontiguousarray(ei).view(np.int32).copy()).to(self.device))
            layout._cache[key] = hit
        return hit

    #: fp32 entries at least this long get their per-(entry, client) norms from plato_agg_port_norms
    #: on a side stream (FedAtt); None (the default) = every entry through plato_agg_entry_norms_f32.
    #: Measured on 128 ResNet-18 clients: 1.45 ms with None, 1.71-2.15 ms with thresholds of 2^15-2^20
    #: (profiles/r03t_fedatt.log)
    norms_long_threshold: int | None = None

    def side_stream(self) -> torch.cuda.Stream:
        st = getattr(self, "_side", None)
        if st is None:
            st = self._side = torch.cuda.Stream(self.device)
        return st

    def _norm_tables_without(self, layout: ArenaLayout, drop: tuple) -> torch.Tensor:
        """The fp32 norm table (longest first) without the entries in ``drop``."""
        key = ("dev_norm_tables_without", drop, str(self.device))
        hit = layout._cache.get(key)
        if hit is None:
            ef, _ = layout.chunk_tables(1 << 32)
            ef = ef[np.argsort(-(ef[:, 2].astype(np.int64) - ef[:, 1]), kind="stable")] if len(ef) else ef
            ef = ef[~np.isin(ef[:, 0].astype(np.int64), np.asarray(drop, dtype=np.int64))] if len(ef) else ef
            hit = torch.from_numpy(np.ascontiguousarray(ef).view(np.int32).copy()).to(self.device)
            layout._cache[key] = hit
        return hit

    def _result_pool(self, layout: ArenaLayout) -> ResultPool:
        pool = layout._cache.get("result_pool")
        if pool is None:
            pool = layout._cache["result_pool"] = ResultPool(layout)
        return pool

    def _f32_stager(self, layout: ArenaLayout | None = None) -> "_Stager":
        """All-fp32 arrays over the model's keys (FedAtt's noise), packed in ``layout`` (default: the engine's)."""
        if layout is None or layout is self._layout:
            st = self._stagers.get("f32")
            if st is None:
                st = _Stager(self._layout, self.device, codec="f32", stream=self._copy_stream)
                self._stagers["f32"] = st
            return st
        st = layout._cache.get(("f32_stager", str(self.device)))
        if st is None:
            st = layout._cache[("f32_stager", str(self.device))] = _Stager(layout, self.device, codec="f32",
                                                                           stream=self._copy_stream)
        return st

    # ---------------------------------------------------- arrival staging
    ARRIVAL_CHUNK = 16  # rows per arrival slab; rows never move once staged

    def prestage(self, payload: Mapping[str, torch.Tensor], baseline_layout: ArenaLayout,
                 baseline: Mapping[str, torch.Tensor] | None = None) -> bool:
        """Copy one arriving payload to HBM now (H2D overlaps the other clients' arrival).

        The next aggregation round adopts it by identity (``AggregationRound.adopt``);
        the payload must not be modified after arrival.  Returns False if the
        payload does not fit the layout (it is then staged at aggregation time).
        With :attr:`delta_arenas` and the server's current model as ``baseline`` (the
        baseline of the round this payload will join), the row is turned into its delta
        right behind its H2D; a round adopts it only if its own baseline is that model
        unchanged (:func:`baseline_key`), else it stages the payload again.
        """
        codec = payload_codec(payload)
        try:
            baseline_layout.check_compatible(payload, "arriving payload", codec)
        except (KeyError, ValueError):
            return False
        if self._layout is None or self._layout.signature != baseline_layout.signature:
            self._layout = baseline_layout
            self._slabs, self._stagers, self._base = {}, {}, None
            self._arrivals, self._arrival_free, self._arrival_slabs = {}, {}, {}
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.device)
        for c in {codec, "native"}:
            if c not in self._stagers:
                self._stagers[c] = _Stager(self._layout, self.device, codec=c, stream=self._copy_stream)
        free = self._arrival_free.setdefault(codec, [])
        if not free:
            slabs = self._arrival_slabs.setdefault(codec, [])
            slab = ClientSlab(self._layout, self.ARRIVAL_CHUNK, self.device, codec)
            slabs.append(slab)
            free.extend((slab, r) for r in range(self.ARRIVAL_CHUNK))
        slab, row = free.pop()
        self._stagers[codec].put(payload, slab.f32[row], slab.i64[row])
        pf, pi = slab.row_pointers([row])
        delta_key = None
        if self.delta_arenas and codec == "native" and baseline is not None:
            delta_key = self._arrival_baseline(baseline)
            if delta_key is not None:  # x - b in place, behind this payload's H2D on the copy stream
                n_i = self._layout.n_i64
                _lib.call("plato_agg_compute_deltas", int(pf[0]), int(pi[0]) if n_i else None,
                          _ptr(self._arrival_base.f32), _ptr(self._arrival_base.i64) if n_i else None, int(pf[0]),
                          int(pi[0]) if n_i else None, self._layout.n_f32, n_i, _stream_handle(self._copy_stream))
        # keep the dict alive: its id() is the key; the fingerprint detects later edits
        self._arrivals[id(payload)] = (payload, codec, self._layout.signature, int(pf[0]), int(pi[0]), slab, row,
                                       payload_fingerprint(payload), delta_key)
        return True

    def _arrival_baseline(self, baseline: Mapping[str, torch.Tensor]):
        """The arrival baseline on the device (staged once per model version); its key, or None."""
        key = baseline_key(baseline)
        if key is None:  # a model without version counters: arrivals stay weights
            return None
        if key == getattr(self, "_arrival_base_key", None):
            return key
        try:
            self._layout.check_compatible(baseline, "baseline")
        except (KeyError, ValueError):
            return None
        if getattr(self, "_arrival_base", None) is None or self._arrival_base_layout is not self._layout:
            self._arrival_base = DeviceArena(self._layout, self.device)
            self._arrival_base_layout = self._layout
        # stream order on the copy stream: rows converted against the previous model ran before this copy
        self._stagers["native"].put(baseline, self._arrival_base.f32, self._arrival_base.i64)
        self._arrival_base_key = key
        return key

    def _arrival_rows(self, payload, layout: ArenaLayout, codec: str):
        hit = self._arrivals.get(id(payload))
        if hit is None or hit[0] is not payload or hit[1] != codec or hit[2] != layout.signature:
            return None
        if hit[7] != payload_fingerprint(payload):
            return None  # an entry was replaced or written after arrival: stage the current tensors
        return hit[3], hit[4], hit[8]

    def drop_arrival(self, payload) -> None:
        """Return one payload's arrival slot (a multi-GPU prestage that failed on another device).

        A copy still in flight into the row is ordered before any later copy into it (one copy stream)."""
        hit = self._arrivals.pop(id(payload), None)
        if hit is not None and hit[0] is payload:
            self._arrival_free.setdefault(hit[1], []).append((hit[5], hit[6]))
        elif hit is not None:
            self._arrivals[id(payload)] = hit

    def release_arrivals(self) -> None:
        """Return every arrival slot (after the round that used them has completed, or failed)."""
        for payload, codec, _, _, _, slab, row, _, _ in self._arrivals.values():
            self._arrival_free.setdefault(codec, []).append((slab, row))
        self._arrivals = {}

    # ------------------------------------------------------ raw device call
    def launch_fedavg(self, layout: ArenaLayout, ptr_f32: torch.Tensor, ptr_i64: torch.Tensor | None,
                      w: torch.Tensor, s: torch.Tensor | None, k: int,
                      base_f32: torch.Tensor | None, base_i64: torch.Tensor | None,
                      out_f32: torch.Tensor, out_i64f: torch.Tensor | None,
                      stream: torch.cuda.Stream | None = None) -> None:
        """Launch the fused kernel on device-resident arenas (no host traffic).

        ``base_f32 is None`` selects deltas mode (``aggregate_deltas``).
        """
        stream = stream or torch.cuda.current_stream(self.device)
        n_f, n_i = layout.n_f32, layout.n_i64
        if ptr_f32.numel() < k or w.numel() < k:
            raise ValueError("pointer table / weights shorter than K")
        args_tail = (n_f, n_i, _stream_handle(stream))
        ptr_i = _ptr(ptr_i64) if n_i else None
        if self.variant is None:
            if base_f32 is not None:
                _lib.call("plato_agg_fedavg_weights", _ptr(ptr_f32), ptr_i, _ptr(w), _ptr(s), k,
                          _ptr(base_f32), _ptr(base_i64) if n_i else None, _ptr(out_f32),
                          _ptr(out_i64f) if n_i else None, *args_tail)
            else:
                _lib.call("plato_agg_fedavg_deltas", _ptr(ptr_f32), ptr_i, _ptr(w), _ptr(s), k,
                          _ptr(out_f32), _ptr(out_i64f) if n_i else None, *args_tail)
        else:
            _lib.tune_call("plato_agg_tune_fedavg", self.variant, int(base_f32 is not None), _ptr(ptr_f32),
                      ptr_i, _ptr(w), _ptr(s), k, _ptr(base_f32),
                      _ptr(base_i64) if n_i else None, _ptr(out_f32),
                      _ptr(out_i64f) if n_i else None, *args_tail)

    # ------------------------------------------------------ host-facing API
    def begin(self, template: Mapping[str, torch.Tensor], capacity: int,
              codec: str = "native") -> "AggregationRound":
        """Start a round: device arenas for up to ``capacity`` client payloads.

        ``template`` is the baseline (its keys, shapes, dtypes define the arena);
        ``codec`` is how the client payloads arrive ("native" or "bf16").
        """
        if capacity <= 0:
            raise ValueError("no client payloads to aggregate")
        layout = self._prepare(template, capacity, codec)
        # The previous round's kernel may still read the slab / baseline arena:
        # order this round's H2D copies (copy stream) after it.
        self._copy_stream.wait_stream(torch.cuda.current_stream(self.device))
        return AggregationRound(self, layout, capacity, codec)

    def stage_clients(self, payloads: Sequence[Mapping[str, torch.Tensor]], template=None,
                      what: str = "weights_received") -> ArenaLayout:
        """Pack and copy K CPU payloads into the client slab (rows 0..K-1)."""
        template = template if template is not None else payloads[0]
        layout = self._prepare(template, len(payloads))
        for i, sd in enumerate(payloads):
            layout.check_compatible(sd, f"{what}[{i}]")
            self._stager.put(sd, self._slab.f32[i], self._slab.i64[i])
        return layout

    def aggregate_weights(self, baseline: Mapping[str, torch.Tensor],
                          weights_received: Sequence[Mapping[str, torch.Tensor]],
                          weights: Sequence[float], scales: Sequence[float] | None = None
                          ) -> "OrderedDict[str, torch.Tensor]":
        """``update_weights(aggregate_deltas(compute_weight_deltas(b, X)))`` on the GPU.

        Returns CPU tensors in baseline key order: fp32 for every entry (int64
        entries come back as fp32 ``float(b) + avg`` exactly like the
        reference's ``update_weights``; ``load_weights`` truncates them).
        """
        k = len(weights_received)
        if k == 0:
            raise ValueError("no client payloads to aggregate")
        if len(weights) != k:
            raise ValueError("weights must have one entry per client")
        rnd = self.begin(baseline, k, payload_codec(weights_received[0]))
        rnd.put_baseline(baseline)
        for i, sd in enumerate(weights_received):
            rnd.put_client(i, sd)
        rnd.launch(weights, scales)
        return rnd.result()

    def aggregate_deltas(self, deltas_received: Sequence[Mapping[str, torch.Tensor]],
                         weights: Sequence[float], scales: Sequence[float] | None = None
                         ) -> "OrderedDict[str, torch.Tensor]":
        """``Server.aggregate_deltas`` on the GPU: ``avg = sum_i delta_i * w_i`` (fp32)."""
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

    def weighted_sum(self, tensors: Sequence, weights: Sequence[float]) -> torch.Tensor:
        """``avg = trainer.zeros(n); avg += t_i * w_i`` over same-size vectors, in order.

        fp32 tensors follow torch's fp32 chain (one deltas-mode launch, fp32
        result).  float64 numpy vectors follow the reference's numpy promotion
        — the plaintext half of HE hybrid FedAvg (plato/servers/fedavg_he.py:
        88-98), whose vectors come from ``np.append`` into float64 arrays
        (plato/utils/homo_enc.py:50-63): ``avg += unenc_w * w`` falls back to
        numpy and the accumulator becomes float64, so the sum runs in float64
        (``plato_agg_weighted_sum_f64``) and the result is a float64 tensor.
        """
        if len(tensors) == 0:
            raise ValueError("no tensors to sum")
        if len(weights) != len(tensors):
            raise ValueError("weights must have one entry per vector")
        first = tensors[0]
        if (isinstance(first, np.ndarray) and first.dtype == np.float64) or \
                (isinstance(first, torch.Tensor) and first.dtype == torch.float64):
            return self._weighted_sum_f64(tensors, weights)
        sds = [OrderedDict(v=torch.as_tensor(t)) for t in tensors]
        return self.aggregate_deltas(sds, weights)["v"]

    def _weighted_sum_f64(self, vectors, weights) -> torch.Tensor:
        """float64 vectors: ``((0 + x_0*w_0) + x_1*w_1) + ...`` in float64 (``plato_agg_weighted_sum_f64``)."""
        n = int(np.asarray(vectors[0]).size)
        host = torch.empty((len(vectors), max(2, -(-n // 2) * 2)), dtype=torch.float64, pin_memory=True)
        for r, v in enumerate(vectors):
            v = torch.as_tensor(np.asarray(v, dtype=np.float64)).reshape(-1)
            if v.numel() != n:
                raise ValueError("vectors must have the same length")
            host[r, :n].copy_(v)
        dev = host.to(self.device, non_blocking=True)
        w = torch.tensor([float(x) for x in weights], dtype=torch.float64).to(self.device)
        ptrs = torch.tensor([dev.data_ptr() + r * dev.stride(0) * 8 for r in range(len(vectors))],
                            dtype=torch.int64).to(self.device)
        out = torch.empty(max(2, n), dtype=torch.float64, device=self.device)
        stream = torch.cuda.current_stream(self.device)
        _lib.call("plato_agg_weighted_sum_f64", _ptr(ptrs), _ptr(w), len(vectors), _ptr(out), n,
                  _stream_handle(stream))
        return out[:n].cpu()

    def compute_weight_deltas(self, baseline: Mapping[str, torch.Tensor],
                              weights_received: Sequence[Mapping[str, torch.Tensor]]
                              ) -> list["OrderedDict[str, torch.Tensor]"]:
        """``Algorithm.compute_weight_deltas`` (``algorithms/fedavg.py:13-27``) on the GPU.

        int64 entries keep int64 deltas, as ``current - baseline`` does.
        """
        k = len(weights_received)
        if k == 0:
            return []
        layout = self.stage_clients(weights_received, template=baseline)
        self._stager.put(baseline, self._base.f32, self._base.i64)
        stream = torch.cuda.current_stream(self.device)
        self._stager.fence(stream)
        h = _stream_handle(stream)
        out = []
        for i in range(k):
            df = torch.empty(layout.row_f32, dtype=torch.float32, device=self.device)
            di = torch.empty(layout.row_i64, dtype=torch.int64, device=self.device)
            _lib.call("plato_agg_compute_deltas", _ptr(self._slab.f32[i]), _ptr(self._slab.i64[i]),
                      _ptr(self._base.f32), _ptr(self._base.i64), _ptr(df), _ptr(di),
                      layout.n_f32, layout.n_i64, h)
            out.append(layout.unpack(df[: layout.n_f32].to("cpu"), di[: layout.n_i64].to("cpu")))
        return out

    def update_weights(self, baseline: Mapping[str, torch.Tensor],
                       deltas: Mapping[str, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
        """``Algorithm.update_weights`` (``algorithms/fedavg.py:29-37``): ``b + avg`` in fp32."""
        layout = self._prepare(baseline, 1)
        # avg is fp32 for every key (trainers/basic.py:63); stage it as a
        # float32 row for both regions.
        avg_f = torch.empty(layout.row_f32, dtype=torch.float32, device=self.device)
        avg_i = torch.empty(layout.row_i64, dtype=torch.float32, device=self.device)
        f32 = [deltas[e.name].reshape(-1).to(torch.float32) for e in layout.entries if e.region == F32]
        i64 = [deltas[e.name].reshape(-1).to(torch.float32) for e in layout.entries if e.region == I64]
        if f32:
            avg_f[: layout.n_f32].copy_(torch.cat(f32))
        if i64:
            avg_i[: layout.n_i64].copy_(torch.cat(i64))
        self._stager.put(baseline, self._base.f32, self._base.i64)
        stream = torch.cuda.current_stream(self.device)
        self._stager.fence(stream)
        out_f = torch.empty_like(avg_f)
        out_i = torch.empty_like(avg_i)
        _lib.call("plato_agg_update_weights", _ptr(self._base.f32), _ptr(self._base.i64), _ptr(avg_f),
                  _ptr(avg_i), _ptr(out_f), _ptr(out_i), layout.n_f32, layout.n_i64,
                  _stream_handle(stream))
        return layout.unpack(out_f[: layout.n_f32].to("cpu"), out_i[: layout.n_i64].to("cpu"))

    def mix_weights(self, baseline: Mapping[str, torch.Tensor],
                    received: Mapping[str, torch.Tensor], mixing: float
                    ) -> "OrderedDict[str, torch.Tensor]":
        """FedAsync: ``b * (1 - m) + x * m`` (``fedasync_algorithm.py:15-18``)."""
        layout = self.stage_clients([received], template=baseline)
        self._stager.put(baseline, self._base.f32, self._base.i64)
        stream = torch.cuda.current_stream(self.device)
        self._stager.fence(stream)
        one_minus = float(np.float32(1 - mixing))
        m = float(np.float32(mixing))
        out_f = torch.empty(layout.row_f32, dtype=torch.float32, device=self.device)
        out_i = torch.empty(layout.row_i64, dtype=torch.float32, device=self.device)
        _lib.call("plato_agg_mix_weights", _ptr(self._slab.f32[0]), _ptr(self._slab.i64[0]),
                  _ptr(self._base.f32), _ptr(self._base.i64), one_minus, m, _ptr(out_f),
                  _ptr(out_i), layout.n_f32, layout.n_i64, _stream_handle(stream))
        return layout.unpack(out_f[: layout.n_f32].to("cpu"), out_i[: layout.n_i64].to("cpu"))


class _KernelTimer:
    """HIP events on ``stream`` around the launches of a ``with`` block; the round's ``timings[name + "_ms"]``
    is filled once the stream has passed them (``AggregationRound._resolve_timers``, after the method's sync)."""

    def __init__(self, rnd: "AggregationRound", name: str, stream):
        self.rnd, self.name, self.stream = rnd, name, stream

    def __enter__(self):
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record(self.stream)
        return self

    def __exit__(self, *exc):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(self.stream)
        self.rnd._timers.append((self.name, self.e0, e1))
        return False


class AggregationRound:
    """One aggregation: client rows staged H2D (in any order), then one launch.

    Rows are slots; the summation order is given at :meth:`launch` time by
    ``order`` (default: slot order), matching ``self.updates`` order in the
    reference regardless of the order payloads arrived in.
    """

    deltas = False  # (set per round in __init__; decoded rounds hold decoded weights)

    def __init__(self, engine: FedAvgEngine, layout: ArenaLayout, capacity: int, codec: str = "native"):
        self.engine = engine
        self.layout = layout
        self.capacity = capacity
        self.codec = codec
        self.slab = engine._slabs[codec]
        self.stager = engine._stagers[codec]
        self.staged = [False] * capacity
        # per slot: device pointers of its fp32 / int64 rows (round slab or an arrival slot)
        self._pf = [0] * capacity
        self._pi = [0] * capacity
        # QSGD codec: per slot max_v per entry (layout order) and the clients' quantization level
        self._mv: list = [None] * capacity
        self._level: int | None = None
        self.has_baseline = False
        self.event: torch.cuda.Event | None = None
        self._out = None
        self._t0 = time.perf_counter()
        self._kernel_events = None
        self.timings: dict = {}
        self._k = 0
        self._decoded = None
        self._timers: list = []
        # Delta arenas: every staged slot is turned into x - b in place on the copy stream as it is staged
        # (compute_weight_deltas, plato/algorithms/fedavg.py:13-27, the same fp32 differences and int64
        # wrapping differences the kernels would form), so the reductions that re-read the baseline per
        # client (FedAdp's dots) stream no baseline.  The kernels then run in their deltas forms and the
        # final update adds the baseline once (plato_agg_update_weights: b + acc, the fused epilogue's sum).
        self.deltas = bool(getattr(engine, "delta_arenas", False)) and codec == "native"
        self._converted: set = set()

    def _to_delta(self, slot: int) -> None:
        """Turn staged slot ``slot`` into its delta x - b, in place, on the copy stream (after its H2D)."""
        if not self.has_baseline:
            raise ValueError("delta arenas: stage the baseline before the clients")
        key = (self._pf[slot], self._pi[slot])
        if key in self._converted:
            return
        eng, lay = self.engine, self.layout
        n_i = lay.n_i64
        cs = self.stager.stream
        _lib.call("plato_agg_compute_deltas", self._pf[slot], self._pi[slot] if n_i else None, _ptr(self._base.f32),
                  _ptr(self._base.i64) if n_i else None, self._pf[slot], self._pi[slot] if n_i else None,
                  lay.n_f32, n_i, _stream_handle(cs))
        self._converted.add(key)

    def _raw_only(self, what: str) -> None:
        if self.deltas:
            raise ValueError(f"{what} reads the clients' weights; this round holds deltas (engine.delta_arenas)")

    def _timed(self, name: str, stream) -> _KernelTimer:
        return _KernelTimer(self, name, stream)

    def _resolve_timers(self) -> None:
        """Device times of the timed launches (call after the stream has been synchronised)."""
        for name, e0, e1 in self._timers:
            self.timings[name + "_ms"] = e0.elapsed_time(e1)
        self._timers = []

    @property
    def _base(self) -> DeviceArena:
        """The baseline arena this round's kernels read (the engine's; a decoded round has its own)."""
        return self.engine._base

    def put_baseline(self, baseline: Mapping[str, torch.Tensor]) -> None:
        self.layout.check_compatible(baseline, "baseline_weights")
        eng = self.engine
        if self.deltas and any(self.staged):
            raise ValueError("delta arenas: the clients were staged as deltas of the previous baseline")
        eng._stager.put(baseline, eng._base.f32, eng._base.i64)
        self.has_baseline = True
        self._base_key = baseline_key(baseline)
        self._arrival_base_ok = None
        self._decoded = None

    def put_client(self, slot: int, payload: Mapping[str, torch.Tensor],
                   what: str = "weights_received") -> None:
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        self.layout.check_compatible(payload, f"{what}[{slot}]", self.codec)
        self._coded_scales(slot, payload)
        if self.deltas and not self.has_baseline:
            raise ValueError("delta arenas: stage the baseline before the clients")
        self.stager.put(payload, self.slab.f32[slot], self.slab.i64[slot])
        pf, pi = self.slab.row_pointers([slot])
        self._pf[slot], self._pi[slot] = int(pf[0]), int(pi[0])
        self._converted.discard((self._pf[slot], self._pi[slot]))  # fresh weights in the row
        if self.deltas:
            self._to_delta(slot)  # behind this client's H2D on the copy stream
        self.staged[slot] = True
        self._decoded = None  # decoded rows are per staged set

    def _coded_scales(self, slot: int, payload) -> None:
        if self.codec != "qsgd":
            return
        level = int(payload.level)
        if self._level is not None and level != self._level:
            raise ValueError(f"QSGD payloads of one round must share quantization_level ({level} != {self._level})")
        self._level = level
        self._mv[slot] = payload.max_v_array(self.layout.keys())

    def adopt(self, slot: int, payload: Mapping[str, torch.Tensor]) -> bool:
        """Use ``payload``'s copy already staged at arrival (``FedAvgEngine.prestage``), if any.

        Returns False (nothing done) when the payload was not prestaged for
        this round's layout and codec; the caller then stages it with put_client.
        """
        if not 0 <= slot < self.capacity:
            raise IndexError(f"slot {slot} outside [0, {self.capacity})")
        hit = self.engine._arrival_rows(payload, self.layout, self.codec)
        if hit is None:
            return False
        pf, pi, delta_key = hit
        if delta_key is not None and not (self.deltas and delta_key == getattr(self, "_base_key", None)
                                          and self._arrival_base_matches()):
            return False  # a delta against another model (or a weight round): stage the payload again
        self._coded_scales(slot, payload)
        self._pf[slot], self._pi[slot] = pf, pi
        if delta_key is not None:
            self._converted.add((pf, pi))  # turned into its delta at arrival, against this round's baseline
        elif self.deltas:  # the arrival row holds the weights: its delta now, in place (the row is this round's)
            self._to_delta(slot)
        self.staged[slot] = True
        self._decoded = None  # decoded rows are per staged set
        return True

    def _arrival_base_matches(self) -> bool:
        """The model the arrivals were turned into deltas against has this round's baseline bits.

        The keys (storage + version counters) already match; an in-place write that leaves the
        counters alone (``.data`` writes in a hook) or a freed storage reused at the same address
        would still let a stale delta in, so the two staged arenas are compared once per round on
        the device, after both copies (copy stream).  A mismatch makes every arrival row of the
        round staged again from its host tensors.
        """
        ok = getattr(self, "_arrival_base_ok", None)
        if ok is None:
            eng, lay = self.engine, self.layout
            arr = getattr(eng, "_arrival_base", None)
            if arr is None or eng._arrival_base_layout.signature != lay.signature:
                ok = False
            else:
                stream = torch.cuda.current_stream(eng.device)
                stream.wait_stream(eng._copy_stream)
                ok = (same_f32_bits(self._base.f32[: lay.n_f32], arr.f32[: lay.n_f32], lay.f32_padding(eng.device))
                      and torch.equal(self._base.i64[: lay.n_i64], arr.i64[: lay.n_i64]))
            self._arrival_base_ok = ok
        return ok

    def launch(self, weights: Sequence[float], scales: Sequence[float] | None = None,
               order: Sequence[int] | None = None, deltas: bool = False) -> None:
        """Enqueue the fused kernel (stream-ordered after every staged copy)."""
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
        eng = self.engine
        lay = self.layout
        self.timings["stage_ms"] = (time.perf_counter() - self._t0) * 1e3
        self._k = len(order)
        w, s = eng._upload_weights(weights, scales)
        pf = np.asarray([self._pf[i] for i in order], dtype=np.int64)
        pi = np.asarray([self._pi[i] for i in order], dtype=np.int64)
        tf, ti = eng._pointer_tables(pf, pi)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        out_f = torch.empty(lay.row_f32, dtype=torch.float32, device=eng.device)
        out_i = torch.empty(lay.row_i64, dtype=torch.float32, device=eng.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        if self.codec == "qsgd":
            n_i = lay.n_i64
            mv = torch.from_numpy(np.ascontiguousarray(np.stack([self._mv[i] for i in order], axis=1))).to(eng.device)
            cf, ci = eng._chunks(lay, eng.QSGD_CHUNK)
            ncf, nci = int(cf.shape[0]), int(ci.shape[0])
            args = (_ptr(tf), _ptr(ti) if n_i else None, len(order), _ptr(mv), len(lay.entries),
                    float(self._level - 1), _ptr(w), _ptr(s), _ptr(cf), ncf, _ptr(ci) if nci else None, nci,
                    _ptr(self._base.f32), _ptr(self._base.i64) if n_i else None, _ptr(out_f),
                    _ptr(out_i) if n_i else None, lay.n_f32, n_i, _stream_handle(stream))
            if eng.qsgd_variant is None:
                _lib.call("plato_agg_fedavg_qsgd", *args)
            else:  # tuning / tests
                _lib.tune_call("plato_agg_tune_fedavg_qsgd", eng.qsgd_variant, *args)
            w = (w, mv)
        elif self.codec == "bf16":
            n_i = lay.n_i64
            _lib.call("plato_agg_fedavg_weights_bf16", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w), _ptr(s),
                      len(order), _ptr(self._base.f32), _ptr(self._base.i64) if n_i else None, _ptr(out_f),
                      _ptr(out_i) if n_i else None, lay.n_f32, n_i, _stream_handle(stream))
        elif self.deltas and not deltas:  # delta arenas: acc = sum_i d_i * w_i, then b + acc
            acc_f = torch.empty_like(out_f)
            acc_i = torch.empty_like(out_i)
            eng.launch_fedavg(lay, tf, ti, w, s, len(order), None, None, acc_f, acc_i, stream)
            n_i = lay.n_i64
            _lib.call("plato_agg_update_weights", _ptr(self._base.f32), _ptr(self._base.i64) if n_i else None,
                      _ptr(acc_f), _ptr(acc_i) if n_i else None, _ptr(out_f), _ptr(out_i) if n_i else None,
                      lay.n_f32, n_i, _stream_handle(stream))
            w = (w, acc_f, acc_i)
        else:
            eng.launch_fedavg(lay, tf, ti, w, s, len(order), None if deltas else self._base.f32,
                              None if deltas else self._base.i64, out_f, out_i, stream)
        e1.record(stream)
        self._kernel_events = (e0, e1)
        self._fetch(stream, out_f, out_i, (tf, ti, w, s))

    def launch_w64(self, weights64: Sequence[float], weights_i64: Sequence[float] | None = None,
                   order: Sequence[int] | None = None, deltas: bool = False) -> None:
        """FedAvg with float64 weights on the fp32 entries (``plato_agg_fedavg_w64``).

        ``acc = fp32(double(acc) + double(d) * w64[i])`` for fp32 entries,
        ``acc += fp32(fp32(d) * fp32(w_i64[i]))`` for int64 entries (default:
        ``w_i64 = weights64``): the RL server's float64 smart weighting
        (rl_server.py:66-71) and HE's float64 plaintext vectors (fedavg_he.py:88-98).
        """
        order = list(range(len(weights64))) if order is None else list(order)
        if len(order) != len(weights64):
            raise ValueError("order and weights must have the same length")
        slots = self._check_slots(order)
        if not deltas and not self.has_baseline:
            raise ValueError("baseline not staged")
        if not deltas:
            self._raw_only("launch_w64")
        eng, lay = self.engine, self.layout
        self.timings["stage_ms"] = (time.perf_counter() - self._t0) * 1e3
        self._k = len(order)
        w64 = torch.from_numpy(np.asarray([float(w) for w in weights64], dtype=np.float64)).to(eng.device)
        wi = fp32_weights(weights64 if weights_i64 is None else weights_i64)
        if len(wi) != len(order):
            raise ValueError("weights_i64 must have one entry per client")
        wi = torch.from_numpy(wi).to(eng.device)
        pf = np.asarray([self._pf[i] for i in slots], dtype=np.int64)
        pi = np.asarray([self._pi[i] for i in slots], dtype=np.int64)
        tf, ti = eng._pointer_tables(pf, pi)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        out_f = torch.empty(lay.row_f32, dtype=torch.float32, device=eng.device)
        out_i = torch.empty(lay.row_i64, dtype=torch.float32, device=eng.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        n_i = lay.n_i64
        _lib.call("plato_agg_fedavg_w64", _ptr(tf), _ptr(ti) if n_i else None, _ptr(w64), _ptr(wi), len(order),
                  None if deltas else _ptr(self._base.f32), None if (deltas or not n_i) else _ptr(self._base.i64),
                  _ptr(out_f), _ptr(out_i) if n_i else None, lay.n_f32, n_i, _stream_handle(stream))
        e1.record(stream)
        self._kernel_events = (e0, e1)
        self._fetch(stream, out_f, out_i, (tf, ti, w64, wi))

    def _fetch(self, stream, out_f: torch.Tensor, out_i: torch.Tensor, keep=()) -> None:
        """D2H into pooled pinned buffers, stream-ordered; result() only waits."""
        lay = self.layout
        host_f, host_i = self.engine._result_pool(lay).get()
        host_f.copy_(out_f[: lay.n_f32], non_blocking=True)
        host_i.copy_(out_i[: lay.n_i64], non_blocking=True)
        self.event = torch.cuda.Event(enable_timing=True)
        self.event.record(stream)
        # keep device buffers alive until the copies finish
        self._out = (host_f, host_i, out_f, out_i, keep)

    def _check_slots(self, slots: Sequence[int]) -> list[int]:
        slots = list(slots)
        for slot in slots:
            if not (0 <= slot < self.capacity and self.staged[slot]):
                raise ValueError(f"client slot {slot} was not staged")
        if not slots:
            raise ValueError("no client slots")
        if self.codec != "native":
            raise ValueError("per-entry kernels take fp32 rows: run them on rnd.decoded() for coded payloads")
        return slots

    def stage_reference(self, state_dict: Mapping[str, torch.Tensor]) -> DeviceArena:
        """Port's stored global model as a device arena, staged ahead of :meth:`model_similarities`
        (which otherwise stages it itself: a PCIe copy of the whole model on the similarity's path)."""
        return self._stage_model(state_dict, "reference model", torch.cuda.current_stream(self.engine.device))

    def _stage_model(self, state_dict, what: str, stream) -> DeviceArena:
        """A native model (e.g. Port's stored global model) as a device arena of this round's layout."""
        self.layout.check_compatible(state_dict, what)
        eng = self.engine
        arena = DeviceArena(self.layout, eng.device)
        eng._stager.put(state_dict, arena.f32, arena.i64)
        eng._stager.fence(stream)
        return arena

    def decoded(self) -> "AggregationRound":
        """This round as the reference's server sees coded payloads: every entry float32.

        The reference dequantizes in its inbound processor (plato/processors/
        model_dequantize.py:15-18, model_dequantize_qsgd.py:34-60) before any
        server code runs, so FedAtt / FedAdp / Polaris / Port reduce float32
        state_dicts whose num_batches_tracked counters are float32 too.  The
        staged slots (bf16 or QSGD codes in HBM) and the baseline are decoded
        once by ``plato_agg_decode_rows`` into fp32 rows of ``layout.promoted()``
        (the counters become fp32 entries, the baseline's cast with RNE), and
        the returned round runs the per-entry kernels on them.  Slots are the
        same; the plain FedAvg launch stays on this round (decode in registers).
        A native round returns itself.
        """
        if self.codec == "native":
            return self
        if self._decoded is not None:
            return self._decoded
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        slots = [i for i in range(self.capacity) if self.staged[i]]
        if not slots:
            raise ValueError("no client slots staged")
        play = lay.promoted()
        rnd = _DecodedRound(self, play, slots)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        eng._stager.fence(stream)
        cf, ci = eng._chunks(lay, 4096)
        ncf, nci = int(cf.shape[0]), int(ci.shape[0])
        dst_off = lay.row_f32
        h = _stream_handle(stream)

        def decode(codec, src_f, src_i, dsts, mv=None, divisor=0.0):
            k = len(dsts)
            tab = torch.from_numpy(np.asarray(list(src_f) + list(src_i) + list(dsts), dtype=np.int64)).to(eng.device)
            _lib.call("plato_agg_decode_rows", _lib.PLATO_AGG_DECODE[codec], tab.data_ptr(), tab.data_ptr() + 8 * k, k,
                      _ptr(mv), float(divisor), _ptr(cf), ncf, _ptr(ci) if nci else None, nci, dst_off,
                      tab.data_ptr() + 16 * k, h)
            return tab

        keep = [decode("native", [_ptr(eng._base.f32)], [_ptr(eng._base.i64)], [_ptr(rnd._own_base.f32)])]
        rows = rnd.slab.row_pointers(range(len(slots)))[0]
        mv = None
        if self.codec == "qsgd":
            mv = torch.from_numpy(np.ascontiguousarray(np.stack([self._mv[i] for i in slots], axis=1))).to(eng.device)
        keep.append(decode(self.codec, [self._pf[i] for i in slots], [self._pi[i] for i in slots], list(rows), mv,
                           0.0 if self._level is None else float(self._level - 1)))
        rnd._keep_decode = (keep, mv)
        self._decoded = rnd
        return rnd

    def entry_stats(self, slots: Sequence[int], v: tuple | None = None, deltas: bool = False):
        """Per (client, entry) fp64 sums over the staged slots (``plato_agg_entry_stats``).

        ``d_i = x_i - baseline`` (``deltas=False``) or ``x_i``.  ``v`` is an
        optional device vector ``(fp32 arena, fp32 values of the int64
        entries)``, e.g. :meth:`launch_entrywise`'s ``device=True`` output.
        Returns ``(dv [K, E] | None, dd [K, E], vv [E] | None)`` as float64
        numpy arrays, entries in layout order.
        """
        slots = self._check_slots(slots)
        deltas = deltas or self.deltas  # delta arenas: the rows are the deltas
        if not deltas and not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        k, n_e = len(slots), len(lay.entries)
        cf, ci = eng._chunks(lay, eng.STATS_CHUNK)
        pf = np.asarray([self._pf[i] for i in slots], dtype=np.int64)
        pi = np.asarray([self._pi[i] for i in slots], dtype=np.int64)
        tf, ti = eng._pointer_tables(pf, pi)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        ncf, nci = int(cf.shape[0]), int(ci.shape[0])
        ws = torch.empty((eng.lib.plato_agg_entry_stats_workspace(k, ncf + nci) + 7) // 8,
                         dtype=torch.float64, device=eng.device)
        out = torch.empty((2 * k + 1) * n_e, dtype=torch.float64, device=eng.device)
        vf, vi = (None, None) if v is None else v
        n_i = lay.n_i64
        _lib.call("plato_agg_entry_stats", _ptr(tf), _ptr(ti) if n_i else None, k,
                  None if deltas else _ptr(self._base.f32), None if (deltas or not n_i) else _ptr(self._base.i64),
                  _ptr(vf), _ptr(vi) if (vf is not None and n_i) else None,
                  _ptr(cf), ncf, _ptr(ci) if nci else None, nci, n_e, lay.n_f32, n_i, _ptr(ws), _ptr(out),
                  _stream_handle(stream))
        res = out.cpu().numpy().reshape(2 * k + 1, n_e)
        if v is None:
            return None, res[k:2 * k].copy(), None
        return res[:k].copy(), res[k:2 * k].copy(), res[2 * k].copy()

    def entry_norms(self, slots: Sequence[int]) -> np.ndarray:
        """fp32 ``torch.linalg.norm`` of each (client, entry) delta in torch's CPU order.

        Bit-equal to the reference's ``torch.linalg.norm(-delta)``
        (fedatt_algorithm.py:39), by ``plato_agg_entry_norms_f32``; with
        ``FedAvgEngine.norms_long_threshold`` set, the long fp32 entries go to
        ``plato_agg_port_norms`` on a side stream instead (measured slower, off
        by default).  Returns ``[E, K]`` float32 (entries in layout order,
        clients in ``slots`` order).
        """
        slots = self._check_slots(slots)
        self._raw_only("entry_norms")
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        k, n_e = len(slots), len(lay.entries)
        ef, ei = eng._norm_tables(lay)  # one piece per entry, longest first
        long_ids = [] if eng.norms_long_threshold is None else sorted(
            (i for i, e in enumerate(lay.entries) if e.region == F32 and e.numel >= eng.norms_long_threshold),
            key=lambda i: -lay.entries[i].numel)
        if long_ids:
            ef = eng._norm_tables_without(lay, tuple(long_ids))
        pf = np.asarray([self._pf[i] for i in slots], dtype=np.int64)
        pi = np.asarray([self._pi[i] for i in slots], dtype=np.int64)
        tf, ti = eng._pointer_tables(pf, pi)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        out = torch.zeros(k * n_e, dtype=torch.float32, device=eng.device)
        n_i = lay.n_i64
        keep = ()
        if long_ids:  # the long chains first, on their own stream
            side = eng.side_stream()
            side.wait_stream(stream)
            base_f = _ptr(self._base.f32)
            xs = [int(pf[j]) + 4 * lay.entries[e].offset for e in long_ids for j in range(k)]
            bs = [base_f + 4 * lay.entries[e].offset for e in long_ids for j in range(k)]
            lens = np.asarray([lay.entries[e].numel for e in long_ids for _ in range(k)], dtype=np.uint32)
            n_max = int(lens.max())
            tab = np.asarray(xs + xs + bs + bs, dtype=np.int64)  # int64 tables unused (one fp32 segment)
            seg = np.zeros(1, dtype=[("flat", "<u8"), ("src", "<u8"), ("numel", "<u8"), ("region", "<u4"),
                                     ("flags", "<u4")])
            seg["numel"] = n_max
            v = len(xs)
            with torch.cuda.stream(side):
                dt = torch.from_numpy(tab).to(eng.device)
                dl = torch.from_numpy(lens.view(np.int32)).to(eng.device)
                ds = torch.from_numpy(seg.view(np.int64).copy()).to(eng.device)
                dn = torch.empty(v, dtype=torch.float32, device=eng.device)
                p8, n8 = dt.data_ptr(), 8 * v
                _lib.call("plato_agg_port_norms", p8, p8 + n8, p8 + 2 * n8, p8 + 3 * n8, v, dl.data_ptr(), ds.data_ptr(),
                          1, n_max, lay.n_f32, 0, dn.data_ptr(), None, _stream_handle(side))
                # scatter: vector (li, j) -> out[j * n_e + entry]
                idx = torch.from_numpy(np.asarray([j * n_e + e for e in long_ids for j in range(k)],
                                                  dtype=np.int64)).to(eng.device)
                out.index_copy_(0, idx, dn)
            keep = (dt, dl, ds, dn, idx)
        nef, nei = int(ef.shape[0]), int(ei.shape[0])
        if nef or nei:
            with self._timed("entry_norms", stream):
                _lib.call("plato_agg_entry_norms_f32", _ptr(tf), _ptr(ti) if n_i else None, k, _ptr(self._base.f32),
                          _ptr(self._base.i64) if n_i else None, _ptr(ef) if nef else None, nef,
                          _ptr(ei) if nei else None, nei, n_e, lay.n_f32, n_i, _ptr(out), _stream_handle(stream))
        if long_ids:
            stream.wait_stream(eng.side_stream())
        res = np.ascontiguousarray(out.cpu().numpy().reshape(k, n_e).T)
        self._resolve_timers()
        del keep
        return res

    def launch_entrywise(self, weights: np.ndarray, order: Sequence[int] | None = None, scale: float = 1.0,
                         noise: Mapping[str, torch.Tensor] | None = None, noise_scale: float = 0.0,
                         add_base: bool = True, deltas: bool = False, device: bool = False):
        """Weighted sum with a weight per (entry, client) (``plato_agg_fedavg_entrywise``).

        ``weights`` is ``[E, K]`` (entries in layout order, clients in
        ``order``), rounded to fp32 like torch's scalar multiply.  ``noise``
        is a state_dict of fp32 tensors added as ``noise * noise_scale``.
        ``device=True`` returns the device result ``(fp32 arena, int64
        entries as fp32)`` instead of scheduling the D2H for :meth:`result`.
        """
        order = list(range(np.shape(weights)[1])) if order is None else list(order)
        slots = self._check_slots(order)
        if not deltas and not self.has_baseline:
            raise ValueError("baseline not staged")
        if self.deltas and not deltas:
            if add_base:
                self._raw_only("launch_entrywise(add_base=True)")
            deltas = True  # the staged rows are the deltas the kernel would form
        if deltas and add_base:
            raise ValueError("add_base needs the baseline (deltas=False)")
        eng, lay = self.engine, self.layout
        k, n_e = len(slots), len(lay.entries)
        w = np.ascontiguousarray(np.asarray(weights, dtype=np.float64).astype(np.float32))
        if w.shape != (n_e, k):
            raise ValueError(f"weights must be [entries={n_e}, clients={k}], got {w.shape}")
        cf, ci = eng._chunks(lay, eng.ENTRYWISE_CHUNK)
        pf = np.asarray([self._pf[i] for i in slots], dtype=np.int64)
        pi = np.asarray([self._pi[i] for i in slots], dtype=np.int64)
        tf, ti = eng._pointer_tables(pf, pi)
        dw = torch.from_numpy(w).to(eng.device)
        nz = None
        nst = None
        if noise is not None:
            nz = DeviceArena(lay, eng.device, i64_dtype=torch.float32)
            lay.check_compatible(noise, "noise", "f32")
            nst = eng._f32_stager(lay)
            nst.put(noise, nz.f32, nz.i64)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        if nst is not None:
            nst.fence(stream)
        out_f = torch.empty(lay.row_f32, dtype=torch.float32, device=eng.device)
        out_i = torch.empty(lay.row_i64, dtype=torch.float32, device=eng.device)
        n_i = lay.n_i64
        ncf, nci = int(cf.shape[0]), int(ci.shape[0])
        _lib.call("plato_agg_fedavg_entrywise", _ptr(tf), _ptr(ti) if n_i else None, k, _ptr(dw), n_e,
                  _ptr(cf), ncf, _ptr(ci) if nci else None, nci,
                  None if deltas else _ptr(self._base.f32), None if (deltas or not n_i) else _ptr(self._base.i64),
                  None if nz is None else _ptr(nz.f32), None if (nz is None or not n_i) else _ptr(nz.i64),
                  float(scale), float(noise_scale), _lib.PLATO_AGG_ADD_BASE if add_base else 0,
                  _ptr(out_f), _ptr(out_i) if n_i else None, lay.n_f32, n_i, _stream_handle(stream))
        if device:
            # inputs stay referenced by the caller's stream order; nothing to fetch
            self._keep = (tf, ti, dw, nz)
            return out_f, out_i
        self._fetch(stream, out_f, out_i, (tf, ti, dw, nz))
        return None

    # ------------------------------------------- flattened-model reductions
    def _flat_segments(self, order: Sequence[int], neg_div_after_first: bool) -> torch.Tensor:
        """plato_agg_segment rows for the layout's entries in ``order`` (device, cached)."""
        lay, eng = self.layout, self.engine
        key = ("flat_segments", tuple(order), neg_div_after_first, str(eng.device))
        hit = lay._cache.get(key)
        if hit is None:
            rows = np.zeros((len(order), 4), dtype=np.uint64)
            flat = 0
            for j, idx in enumerate(order):
                e = lay.entries[idx]
                flags = 1 if (neg_div_after_first and j > 0) else 0
                region = 0 if e.region == F32 else 1
                rows[j, 0], rows[j, 1], rows[j, 2] = flat, e.offset, e.numel
                rows[j, 3] = np.uint64(region | (flags << 32))
                flat += e.numel
            hit = (torch.from_numpy(rows.view(np.int64).copy()).to(eng.device), flat)
            lay._cache[key] = hit
        return hit

    def _flatten(self, mode: int, segs, n_segs: int, n_flat: int, src_f: Sequence[int], src_i: Sequence[int],
                 base: tuple | None, lr: float, stream) -> tuple[torch.Tensor, int]:
        """K flat vectors (rows of a [K, stride] buffer, stride 64-aligned) from device arenas."""
        eng = self.engine
        k = len(src_f)
        stride = max(64, -(-n_flat // 64) * 64)
        out = torch.empty((k, stride), dtype=torch.float32, device=eng.device)
        ptrs = torch.from_numpy(np.asarray(list(src_f) + list(src_i) +
                                           [out.data_ptr() + r * stride * 4 for r in range(k)],
                                           dtype=np.int64)).to(eng.device)
        base_f, base_i = (None, None) if base is None else base
        _lib.call("plato_agg_flatten", mode, ptrs.data_ptr(), ptrs.data_ptr() + 8 * k, k, base_f, base_i,
                  segs.data_ptr(), n_segs, n_flat, float(lr), ptrs.data_ptr() + 16 * k, _stream_handle(stream))
        self._keep_flat = ptrs
        return out, stride

    def _fedadp_order(self):
        lay = self.layout
        order = fedadp_order(lay.keys())
        if order and lay.entries[order[0]].region != F32:
            raise ValueError("FedAdp: the first entry in name order is int64, so the reference flattens to "
                             "float64 (np.append) and takes float64 dots; the device path reproduces the "
                             "float32 case only")
        return order

    def fedadp_dots(self, grads: tuple[torch.Tensor, torch.Tensor], slots: Sequence[int], lr: float):
        """FedAdp's float32 reductions of process_grad's flattened vectors, bit-exact.

        ``grads`` is the device global gradient (fp32 arena, fp32 values of the
        int64 entries), e.g. :meth:`launch_entrywise` with ``device=True``.
        Returns ``(inner[K], g_sq, l_sq[K])`` as numpy float32: ``np.inner(g,
        loc_k)``, ``g.dot(g)``, ``loc_k.dot(loc_k)`` exactly as numpy's OpenBLAS
        forms them (examples/server_aggregation/fedadp/fedadp_server.py:91-99).
        The global gradient is flattened once (``plato_agg_flatten``, RAW); the
        clients' loc_k are gathered from their staged arenas inside
        ``plato_agg_fedadp_dots``, which runs the sdot chains with no flattened
        copies of the K deltas.
        """
        slots = self._check_slots(slots)
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        order = self._fedadp_order()
        segs, n_flat = self._flat_segments(order, True)
        # plato_agg_fedadp_dots' limits (csrc/fedadp.hip run_fedadp); beyond them the round-2 path
        if (len(order) >= self.FEDADP_MAX_SEGS or n_flat >= 1 << 30 or lay.n_f32 >= 1 << 30
                or lay.n_i64 >= 1 << 30 or len(slots) > 65535
                or self.fedadp_boundary_rows(len(order), lay.n_i64) >= self.FEDADP_MAX_BND):
            return self.fedadp_dots_flat(grads, slots, lr)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        g_flat, _ = self._flatten(_lib.PLATO_AGG_FLAT_RAW, segs, len(order), n_flat, [grads[0].data_ptr()],
                                  [grads[1].data_ptr()], None, lr, stream)
        k = len(slots)
        ptrs = torch.from_numpy(np.asarray([self._pf[i] for i in slots] + [self._pi[i] for i in slots],
                                           dtype=np.int64)).to(eng.device)
        xy = torch.empty(k + 1, dtype=torch.float32, device=eng.device)
        yy = torch.empty(k + 1, dtype=torch.float32, device=eng.device)
        # The workspace's layout-only tables (descriptors, boundary rows and their sources) depend on the
        # segment map alone (`segs`, cached on the layout): the engine keeps its last workspace, and its next
        # round of the same layout and K skips building them (PLATO_AGG_FEDADP_TABLES_READY).  Per engine,
        # not per layout: an engine runs one round at a time, while several engines (a client-split round's
        # devices, repeated devices in tests) may reduce the same layout concurrently.
        ws_key = (id(lay), lay.signature, tuple(order), k, segs.data_ptr())
        held = getattr(eng, "_fedadp_ws", None)
        if held is not None and held[0] == ws_key and held[1] is lay:
            ws, flags = held[2], _lib.PLATO_AGG_FEDADP_TABLES_READY
        else:
            eng._fedadp_ws = None  # one workspace per engine (K varies between async rounds)
            ws = torch.empty(-(-_lib.lib().plato_agg_fedadp_dots_workspace(k, 1, lay.n_i64, n_flat, len(order)) // 4),
                             dtype=torch.float32, device=eng.device)
            flags = 0
        n_i = lay.n_i64
        with self._timed("fedadp_dots", stream):
            # delta arenas: a null baseline selects the kernel that streams none (same values, same order)
            base_f = None if self.deltas else _ptr(self._base.f32)
            base_i = None if (self.deltas or not n_i) else _ptr(self._base.i64)
            _lib.call("plato_agg_fedadp_dots_ex", g_flat.data_ptr(), ptrs.data_ptr(), ptrs.data_ptr() + 8 * k, k,
                      base_f, base_i, segs.data_ptr(), len(order), n_flat,
                      lay.n_f32, n_i, float(lr), 1, ws.data_ptr(), xy.data_ptr(), yy.data_ptr(), _stream_handle(stream),
                      flags)
        xy_h, yy_h = xy.cpu().numpy(), yy.cpu().numpy()  # stream-ordered D2H (syncs this stream)
        eng._fedadp_ws = (ws_key, lay, ws)  # its tables are built (this stream has passed the call)
        self._resolve_timers()
        self._keep_flat = (g_flat, ptrs, ws)
        return xy_h[:k], xy_h[k], yy_h[:k]

    def fedadp_dots_flat(self, grads: tuple[torch.Tensor, torch.Tensor], slots: Sequence[int], lr: float,
                         batch_bytes: float = 32e9):
        """The same dots through materialised flat vectors (``plato_agg_flatten`` + ``plato_agg_sdot_shared``).

        The round-2 path, kept as an independent device cross-check of
        :meth:`fedadp_dots` (tests), for the before/after timing
        (scripts/bench_variant_paths.py), and for models beyond the fused
        kernel's limits (:meth:`fedadp_dots` falls back here).  On delta arenas
        the rows are flattened against a zero arena: x - 0 = x for the fp32
        deltas, and the int64 deltas are the exact int64 differences either way.
        """
        slots = self._check_slots(slots)
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        order = self._fedadp_order()
        segs, n_flat = self._flat_segments(order, True)
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        g_flat, stride = self._flatten(_lib.PLATO_AGG_FLAT_RAW, segs, len(order), n_flat, [grads[0].data_ptr()],
                                       [grads[1].data_ptr()], None, lr, stream)
        k = len(slots)
        # rows 0..k-1: g.loc_k and loc_k.loc_k; row k: g.g (the global gradient's squared norm),
        # which the last batch's launch forms alongside (with_xx)
        xy = torch.empty(k + 1, dtype=torch.float32, device=eng.device)
        yy = torch.empty(k + 1, dtype=torch.float32, device=eng.device)
        per = max(1, int(batch_bytes // (stride * 4)))
        ws = torch.empty(_lib.lib().plato_agg_sdot_shared_workspace(min(k, per), 1) // 4, dtype=torch.float32,
                         device=eng.device)
        zero = None
        if self.deltas:  # the rows already hold x - b
            zero = DeviceArena(lay, eng.device)
            zero.f32.zero_()
            zero.i64.zero_()
            base = (_ptr(zero.f32), _ptr(zero.i64))
        else:
            base = (_ptr(self._base.f32), _ptr(self._base.i64))
        keep = [zero]
        for s0 in range(0, k, per):
            part = slots[s0:s0 + per]
            locs, _ = self._flatten(_lib.PLATO_AGG_FLAT_DELTA, segs, len(order), n_flat,
                                    [self._pf[i] for i in part], [self._pi[i] for i in part], base, lr, stream)
            last = s0 + per >= k
            ys_h = [locs.data_ptr() + r * stride * 4 for r in range(len(part))]
            ys = torch.from_numpy(np.asarray(ys_h, dtype=np.int64)).to(eng.device)
            _lib.call("plato_agg_sdot_shared", g_flat.data_ptr(), ys.data_ptr(), len(ys_h), n_flat, int(last),
                      ws.data_ptr(), xy.data_ptr() + 4 * s0, yy.data_ptr() + 4 * s0, _stream_handle(stream))
            keep.append((locs, ys))
            if s0 + per < k:
                stream.synchronize()  # bound the flat buffers to one batch
                keep = [zero]
        stream.synchronize()
        xy_h, yy_h = xy.cpu().numpy(), yy.cpu().numpy()
        inner, g_sq, l_sq = xy_h[:k], xy_h[k], yy_h[:k]
        return inner, g_sq, l_sq

    def np_sumsq(self, slots: Sequence[int]) -> np.ndarray:
        """numpy's float32 ``np.sum(np.square(x - b))`` of every fp32 entry, per client, bit-exact.

        Polaris' per-layer squared deltas (examples/client_selection/polaris/
        polaris_server.py:78-81) in numpy's own order (``plato_agg_np_sumsq``).
        Returns ``[K, E]`` float32 (entries in layout order; int64 entries 0).
        """
        slots = self._check_slots(slots)
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        eng, lay = self.engine, self.layout
        key = ("np_sumsq_pieces", str(eng.device))
        hit = lay._cache.get(key)
        if hit is None:
            rows, first, n_chunks = [], [], 0
            for idx, e in enumerate(lay.entries):
                if e.region == F32 and e.numel:
                    rows.append((idx, e.offset, e.offset + e.numel, 0))
                    first.append(n_chunks)
                    n_chunks += -(-e.numel // 8192)
            pieces = np.asarray(rows, dtype=np.uint32).reshape(-1, 4)
            hit = (torch.from_numpy(pieces.view(np.int32).copy()).to(eng.device),
                   torch.from_numpy(np.asarray(first, dtype=np.uint32).view(np.int32)).to(eng.device),
                   pieces[:, 0].astype(np.int64), n_chunks)
            lay._cache[key] = hit
        pieces, first, entry_of, n_chunks = hit
        k, n_p = len(slots), int(entry_of.size)
        out = np.zeros((k, len(lay.entries)), dtype=np.float32)
        if n_p == 0:
            return out
        stream = torch.cuda.current_stream(eng.device)
        self.stager.fence(stream)
        tf = torch.from_numpy(np.asarray([self._pf[i] for i in slots], dtype=np.int64)).to(eng.device)
        ws = torch.empty(max(1, eng.lib.plato_agg_np_sumsq_workspace(k, n_chunks) // 4), dtype=torch.float32,
                         device=eng.device)
        dev_out = torch.empty((k, n_p), dtype=torch.float32, device=eng.device)
        with self._timed("np_sumsq", stream):
            # delta arenas: a null baseline selects the kernels that load none (the rows hold x - b)
            _lib.call("plato_agg_np_sumsq", tf.data_ptr(), k, None if self.deltas else _ptr(self._base.f32),
                      pieces.data_ptr(),
                      first.data_ptr(), n_p, n_chunks, ws.data_ptr(), dev_out.data_ptr(), _stream_handle(stream))
        out[:, entry_of] = dev_out.cpu().numpy()
        self._resolve_timers()
        return out

    PORT_NORMS_MAX_SEGS = 2048  # csrc/port.hip kMaxSegs
    FEDADP_MAX_SEGS = 1 << 22   # csrc/fedadp.hip run_fedadp
    FEDADP_MAX_BND = 1 << 22    # boundary-table rows (32-bit byte offsets of 1 KiB rows)

    @staticmethod
    def fedadp_boundary_rows(n_segs: int, n_i64: int) -> int:
        """csrc/fedadp.hip adp_max_bnd: boundary-table rows the kernel reserves per pair."""
        return 2 * (n_segs + n_i64 // 256 + 1)

    def model_similarities(self, reference: Mapping[str, torch.Tensor], slots: Sequence[int],
                           eps: float = 1e-8, threads: int | None = None, flat_norms: bool = False) -> list[np.float32]:
        """Port's cosine similarity of each client delta with ``baseline - reference``, bit-exact.

        ``F.cosine_similarity(current - previous, delta, dim=0)`` over the
        models flattened by ``torch.cat`` in state_dict order
        (examples/async/port/port_server.py:24-52), computed on the device in
        the order x86-64 PyTorch 2.10 uses on ``threads`` CPU threads (default
        ``torch.get_num_threads()``: what the reference's call would use in this
        process).  ``plato_agg_port_norms`` gathers ``current - previous`` and
        every client delta straight from the staged arenas for the vector norms
        (serial-chain bound) and stores the flattened vectors as it goes; the
        cascade cosine sums (``plato_agg_torch_cosine_sum``) then read those.
        ``flat_norms=True`` runs the round-2 path instead — ``plato_agg_flatten``,
        then ``plato_agg_entry_norms_f32`` over the flat rows — kept as a device
        cross-check.
        Returned as fp32 like the reference's 0-dim tensor.
        """
        if not self.has_baseline:
            raise ValueError("baseline not staged")
        slots = list(slots)
        for slot in slots:
            if not (0 <= slot < self.capacity and self.staged[slot]):
                raise ValueError(f"client slot {slot} was not staged")
        if not slots:
            return []
        slots = self._check_slots(slots)
        threads = torch.get_num_threads() if threads is None else int(threads)
        eng = self.engine
        lay = self.layout
        stream = torch.cuda.current_stream(eng.device)
        if isinstance(reference, DeviceArena):  # staged ahead by stage_reference
            if reference.layout is not lay:
                raise ValueError("reference arena was staged for another round / layout")
            prev = reference
        else:
            prev = self._stage_model(reference, "reference model", stream)
        self.stager.fence(stream)
        segs, n_flat = self._flat_segments(list(range(len(lay.entries))), False)
        n_segs = len(lay.entries)
        base = (_ptr(self._base.f32), _ptr(self._base.i64))
        stride = max(64, -(-n_flat // 64) * 64)
        k = len(slots)
        h = _stream_handle(stream)
        # plato_agg_port_norms keeps the segment map in LDS (<= PORT_NORMS_MAX_SEGS entries) and takes
        # n_flat < 2^31, n_f32 < 2^30: larger models take the flatten + entry_norms path (same bits)
        if n_segs > self.PORT_NORMS_MAX_SEGS or n_flat >= 1 << 31 or lay.n_f32 >= 1 << 30:
            flat_norms = True
        norms = torch.empty(k + 1, dtype=torch.float32, device=eng.device)
        ws = torch.empty(max(1, eng.lib.plato_agg_torch_cosine_workspace(k, threads) // 4), dtype=torch.float32,
                         device=eng.device)
        out = torch.empty(k, dtype=torch.float32, device=eng.device)
        if flat_norms:  # the round-2 path: flattened vectors, norms and sums over them
            cur, _ = self._flatten(_lib.PLATO_AGG_FLAT_CAST_DIFF, segs, n_segs, n_flat, [base[0]], [base[1]],
                                   (_ptr(prev.f32), _ptr(prev.i64)), 0.0, stream)
            # (delta arenas: the rows minus a zero arena, x - 0 = x, int64 differences cast once as before)
            zero = None
            if self.deltas:
                zero = DeviceArena(lay, eng.device)
                zero.f32.zero_()
                zero.i64.zero_()
            sub = (_ptr(zero.f32), _ptr(zero.i64)) if self.deltas else base
            deltas, _ = self._flatten(_lib.PLATO_AGG_FLAT_DELTA, segs, n_segs, n_flat, [self._pf[i] for i in slots],
                                      [self._pi[i] for i in slots], sub, 0.0, stream)
            rows = [cur.data_ptr()] + [deltas.data_ptr() + r * stride * 4 for r in range(k)]
            tab = torch.from_numpy(np.asarray(rows, dtype=np.int64)).to(eng.device)
            chunk = torch.from_numpy(np.asarray([[0, 0, n_flat, 0]], dtype=np.uint32).view(np.int32)).to(eng.device)
            # the rows are `stride` long (the padding past n_flat is read, never summed): declaring that length keeps
            # the one n_flat-long piece off the kernel's partial-last-float4 fallback (a per-wave path ~1.5x slower)
            _lib.call("plato_agg_entry_norms_f32", tab.data_ptr(), None, k + 1, None, None, chunk.data_ptr(), 1, None,
                      0, 1, stride, 0, norms.data_ptr(), h)
            _lib.call("plato_agg_torch_cosine_sum", cur.data_ptr(), tab.data_ptr() + 8, k, n_flat, norms.data_ptr(),
                      norms.data_ptr() + 4, float(eps), threads, ws.data_ptr(), out.data_ptr(), h)
            keep = (cur, deltas, tab, chunk, zero)
        else:  # norms straight from the arenas; the same kernel stores the flattened vectors for the sums
            flat = torch.empty((k + 1, stride), dtype=torch.float32, device=eng.device)
            vec = np.asarray([base[0]] + [self._pf[i] for i in slots]
                             + [base[1] or 0] + [self._pi[i] or 0 for i in slots]
                             # client vectors subtract the baseline, or nothing on delta arenas (null)
                             + [_ptr(prev.f32)] + [0 if self.deltas else base[0]] * k
                             + [_ptr(prev.i64) or 0] + [0 if self.deltas else (base[1] or 0)] * k
                             + [flat.data_ptr() + r * stride * 4 for r in range(k + 1)], dtype=np.int64)
            vt = torch.from_numpy(vec).to(eng.device)
            v8, n1 = vt.data_ptr(), 8 * (k + 1)
            scaled = torch.empty(stride, dtype=torch.float32, device=eng.device)
            args = (v8, v8 + n1, v8 + 2 * n1, v8 + 3 * n1, k + 1, None, segs.data_ptr(), n_segs, n_flat, lay.n_f32,
                    _lib.PLATO_AGG_PORT_CAST_FIRST, norms.data_ptr(), v8 + 4 * n1, h)
            with self._timed("port_norms", stream):
                if eng.port_variant is None:
                    _lib.call("plato_agg_port_norms", *args)
                else:
                    _lib.tune_call("plato_agg_tune_port_norms", eng.port_variant, *args)
            # current - previous over its norm once (not once per client), then the K cascade sums
            with self._timed("port_cosine", stream):
                _lib.call("plato_agg_scale_by_norm", flat.data_ptr(), n_flat, norms.data_ptr(), float(eps),
                          scaled.data_ptr(), h)
                _lib.call("plato_agg_torch_cosine_sum_scaled", scaled.data_ptr(), v8 + 4 * n1 + 8, k, n_flat,
                          norms.data_ptr() + 4, float(eps), threads, ws.data_ptr(), out.data_ptr(), h)
            keep = (vt, flat, scaled)
        stream.synchronize()
        self._resolve_timers()
        del keep
        self.last_norms = norms.cpu().numpy()
        return [np.float32(v) for v in out.cpu().numpy()]

    def ready(self) -> bool:
        return self.event is not None and self.event.query()

    def wait(self) -> None:
        """Block until the result is in host memory (releases the GIL: safe on a worker thread)."""
        if self.event is None:
            raise RuntimeError("launch() first")
        self.event.synchronize()

    def algorithmic_bytes(self) -> int:
        """HBM bytes of the launch: K client arenas + baseline read, result written."""
        return self.layout.algorithmic_bytes(self._k)

    def result(self) -> "OrderedDict[str, torch.Tensor]":
        if self.event is None:
            raise RuntimeError("launch() first")
        self.event.synchronize()
        if self._kernel_events is not None:
            e0, e1 = self._kernel_events
            self.timings["kernel_ms"] = e0.elapsed_time(e1)
            self.timings["d2h_ms"] = e1.elapsed_time(self.event)
        self.timings["total_ms"] = (time.perf_counter() - self._t0) * 1e3
        host_f, host_i = self._out[0], self._out[1]
        self._out = None
        return self.layout.unpack(host_f, host_i)


class _DecodedRound(AggregationRound):
    """A coded round's slots and baseline as fp32 rows of the promoted layout (AggregationRound.decoded)."""

    def __init__(self, parent: AggregationRound, layout: ArenaLayout, slots: Sequence[int]):
        eng = parent.engine
        self._parent = parent
        self.engine = eng
        self.layout = layout
        self.capacity = parent.capacity
        self.codec = "native"
        self.slab = ClientSlab(layout, len(slots), eng.device)
        self.stager = parent.stager
        self.staged = [False] * parent.capacity
        self._pf = [0] * parent.capacity
        self._pi = [0] * parent.capacity
        rows = self.slab.row_pointers(range(len(slots)))
        for r, slot in enumerate(slots):
            self._pf[slot], self._pi[slot] = int(rows[0][r]), int(rows[1][r])
            self.staged[slot] = True
        self._mv = [None] * parent.capacity
        self._level = None
        self.has_baseline = True
        self.event = None
        self._out = None
        self._t0 = parent._t0
        self._kernel_events = None
        self.timings = {}
        self._timers = []
        self._k = 0
        self._decoded = None
        self._own_base = DeviceArena(layout, eng.device)

    @property
    def _base(self) -> DeviceArena:
        return self._own_base

    def decoded(self) -> "AggregationRound":
        return self

    def _stage_model(self, state_dict, what: str, stream) -> DeviceArena:
        # staged in the model's own layout, then promoted like the baseline (counters cast to fp32)
        native = AggregationRound._stage_model(self._parent, state_dict, what, stream)
        out = DeviceArena(self.layout, self.engine.device)
        lay = self._parent.layout
        cf, ci = self.engine._chunks(lay, 4096)
        ncf, nci = int(cf.shape[0]), int(ci.shape[0])
        tab = torch.tensor([native.f32.data_ptr(), native.i64.data_ptr(), out.f32.data_ptr()], dtype=torch.int64,
                           device=self.engine.device)
        _lib.call("plato_agg_decode_rows", _lib.PLATO_AGG_DECODE["native"], tab.data_ptr(), tab.data_ptr() + 8, 1,
                  None, 0.0, _ptr(cf), ncf, _ptr(ci) if nci else None, nci, lay.row_f32, tab.data_ptr() + 16,
                  _stream_handle(stream))
        self._keep_model = (native, tab)
        return out


def cast_to_int64(src_f32: torch.Tensor, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """load_state_dict's fp32 -> int64 truncating copy, on the device."""
    if not src_f32.is_cuda or src_f32.dtype != torch.float32:
        raise ValueError("cast_to_int64 expects a CUDA float32 tensor")
    src = src_f32.contiguous()
    dst = torch.empty(src.shape, dtype=torch.int64, device=src.device)
    stream = stream or torch.cuda.current_stream(src.device)
    _lib.call("plato_agg_cast_f32_i64", _ptr(src), _ptr(dst), src.numel(), _stream_handle(stream))
    return dst

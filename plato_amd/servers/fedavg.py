"""FedAvg server hooks backed by the MI355X engine (drop-in for plato.servers.fedavg).

Plato's ``fedavg.Server._process_reports`` (plato/servers/fedavg.py:161-229)
prefers an ``aggregate_weights(updates, baseline_weights, weights_received)``
hook when the server has one (``:171-182``) and otherwise runs
``compute_weight_deltas -> aggregate_deltas -> update_weights`` (``:184-196``).
Both paths end in ``algorithm.load_weights``.  The mixins here plug into those
two hooks, so the orchestration, ``weights_received`` / ``weights_aggregated``
hooks, callbacks, testing and checkpointing of the reference stay untouched:

* :class:`FusedAggregationMixin` defines ``aggregate_weights``: one fused GPU
  pass returns exactly ``update_weights(aggregate_deltas(compute_weight_deltas(...)))``.
* :class:`DeltasAggregationMixin` only replaces ``aggregate_deltas``
  (``servers/fedavg.py:137-159``) for servers that keep their own delta logic.

Variants only change the per-client numbers (``aggregation_weights``); see
plato_amd/servers/variants.py.  Use :func:`make_server` to build a concrete
server class on top of the installed Plato (``import plato`` must work), or mix
the classes in by hand: ``class Server(FusedAggregationMixin, fedavg.Server)``.
"""

from __future__ import annotations

import asyncio
import concurrent.futures

from .. import tracing
from .. import weights as W
from ..arena import payload_codec
from ..engine import FedAvgEngine


class _EngineHolder:
    """Lazily created per-server GPU engine: one GPU, or every GPU of ``aggregation_devices``."""

    #: torch device string for the engine, e.g. "cuda:0" (None: current device)
    aggregation_device = None
    #: several devices ("cuda:0", "cuda:1", ... or ordinals): the model is
    #: bucket-sharded over them from this one server process (plato_amd.multi)
    aggregation_devices = None
    #: kernel variant override (tuning only; None = library default)
    aggregation_variant = None
    #: weights computed from the staged payloads (Port, FedAdp, Polaris): such
    #: rounds run on one GPU (the multi-GPU engine's first device) unless every
    #: reduction they need is per entry (``entry_local_weights``)
    needs_staged_round = False
    #: the staged-round weights reduce entry by entry (Polaris' per-layer sums):
    #: the round is sharded by whole entries over ``aggregation_devices``
    entry_local_weights = False
    #: FedAdp / Port: before the first round, check that this host's numpy / torch
    #: reduction order is the one the device reproduces (plato_amd.hostorder):
    #: "warn" logs a mismatch once and goes on, "strict" (or True) raises, False skips
    host_order_check = "warn"
    #: FedAdp / Port over several ``aggregation_devices``: split the whole-model reductions by client
    #: (``MultiDeviceEngine.clients``, every GPU reduces its own clients' chains).  Opt-in: the split's
    #: cross-device copies and RCCL all-gather have only run with repeated devices on a one-GPU box, so
    #: its parity on distinct GPUs is unpinned; the default runs such rounds on the first GPU.
    client_split_rounds = False
    #: arena alignment of the round layouts (plato_amd.arena.ALIGNMENTS): FedAdp's servers align
    #: every fp32 entry to its flattened position so the dot kernel reads whole lines
    arena_alignment = None
    #: stage each client as its delta x - b (FedAvgEngine.delta_arenas; FedAdp's servers): the
    #: subtraction runs behind each client's H2D (with stage_on_arrival: at arrival, against the
    #: server's current model), and the reductions that re-read the baseline per client stream none
    arena_deltas = False

    def aggregation_engine(self):
        eng = getattr(self, "_plato_amd_engine", None)
        if eng is None:
            devices = self.aggregation_devices
            if devices is not None and len(devices) > 1:
                from ..multi import MultiDeviceEngine

                eng = MultiDeviceEngine([f"cuda:{d}" if isinstance(d, int) else d for d in devices],
                                        variant=self.aggregation_variant)
            else:
                device = devices[0] if devices else self.aggregation_device
                device = f"cuda:{device}" if isinstance(device, int) else device
                eng = FedAvgEngine(device, variant=self.aggregation_variant)
            eng.layout_align = self.arena_alignment
            # one GPU, or every engine of the multi-GPU one (its buckets, entry shards, client-split devices
            # and first GPU): clients staged as deltas, at arrival against the server's current model
            eng.delta_arenas = bool(self.arena_deltas)
            self._plato_amd_engine = eng
        return eng

    def round_engine(self, codec: str):
        """The engine one round runs on.

        One GPU: its engine.  Several: parameter buckets for plain rounds of
        native / bf16 payloads; whole-entry shards (``MultiDeviceEngine.entries``)
        for QSGD payloads (per-entry scales) and entry-local staged weights
        (Polaris); for weights that reduce the whole flattened model serially
        per client (Port's similarity, FedAdp's dots) the first GPU, or, with
        ``client_split_rounds``, bucket-sharded staging with the reductions split
        by client (``MultiDeviceEngine.clients``; native payloads only).
        """
        eng = self.aggregation_engine()
        primary = getattr(eng, "primary", None)
        if primary is None:
            return eng
        if self.needs_staged_round and not self.entry_local_weights:
            return eng.clients if (codec == "native" and self.client_split_rounds) else primary
        if self.needs_staged_round or codec not in ("native", "bf16"):
            return eng.entries
        return eng

    def aggregation_executor(self) -> concurrent.futures.ThreadPoolExecutor:
        """One worker thread that packs and copies payloads, off the server's event loop."""
        ex = getattr(self, "_plato_amd_executor", None)
        if ex is None:
            ex = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="plato-amd-stage")
            self._plato_amd_executor = ex
        return ex

    async def _off_loop(self, fn, *args):
        return await asyncio.get_running_loop().run_in_executor(self.aggregation_executor(), fn, *args)

    async def _finish(self, rnd):
        """Wait for the round's result on the worker thread (a HIP event wait, no busy polling)."""
        await self._off_loop(rnd.wait)
        result = rnd.result()
        self._plato_amd_timings = dict(rnd.timings, bytes=rnd.algorithmic_bytes(),
                                       gpus=getattr(getattr(rnd, "engine", None), "world", 1))
        return result

    def aggregation_weights(self, updates):
        """Per-update (weights, second scalars or None), in ``updates`` order.

        FedAvg: ``n_i / N`` with ``self.total_samples = N`` set as the
        reference's aggregate_deltas does (``servers/fedavg.py:140``).
        """
        self.total_samples = sum(update.report.num_samples for update in updates)
        return W.fedavg([update.report.num_samples for update in updates]), None

    def get_logged_items(self) -> dict:
        """The reference's CSV items (``servers/fedavg.py:234-252``) plus the last aggregation's timings.

        ``aggregation_stage_ms`` (pack + H2D issue, host wall), ``aggregation_kernel_ms``
        (HIP events, max over GPUs), ``aggregation_d2h_ms``, ``aggregation_total_ms``
        (hook entry to result), ``aggregation_GBps`` (algorithmic bytes / kernel time)
        and ``aggregation_gpus``; list them in ``results.types`` to record them.
        ``aggregation_host_order_ok`` (FedAdp / Port): whether this host's numpy / torch reduction order
        matched the device's on the probe (False: the weights may differ from this host's reference in
        the last bits; None: not checked), so a "warn"-mode mismatch shows in the results, not only the log.
        """
        items = super().get_logged_items() if hasattr(super(), "get_logged_items") else {}
        t = getattr(self, "_plato_amd_timings", None) or {}
        kernel = t.get("kernel_ms")
        items.update({
            "aggregation_stage_ms": t.get("stage_ms"),
            "aggregation_kernel_ms": kernel,
            "aggregation_d2h_ms": t.get("d2h_ms"),
            "aggregation_total_ms": t.get("total_ms"),
            "aggregation_GBps": (t["bytes"] / (kernel * 1e-3) / 1e9) if kernel else None,
            "aggregation_gpus": t.get("gpus"),
            "aggregation_host_order_ok": getattr(self, "_plato_amd_host_order_ok", None),
        })
        return items


class FusedAggregationMixin(_EngineHolder):
    """``aggregate_weights`` hook: fused deltas -> weighted sum -> update on the GPU(s)."""

    async def aggregate_weights(self, updates, baseline_weights, weights_received):
        # bf16 payloads (model_quantize on the clients) stay bf16 on the device
        codec = payload_codec(weights_received[0])
        engine = self.round_engine(codec)
        try:
            rnd = engine.begin(baseline_weights, len(weights_received), codec)

            def stage():
                with tracing.range("plato_amd.stage"):
                    rnd.put_baseline(baseline_weights)
                    for slot, payload in enumerate(weights_received):
                        # payloads staged at arrival (WireIngestMixin.stage_on_arrival) are adopted in place
                        if not rnd.adopt(slot, payload):
                            rnd.put_client(slot, payload)

            # Pack + H2D run on a worker thread: the event loop keeps serving the
            # clients meanwhile (the reference yields per client, servers/fedavg.py:157).
            await self._off_loop(stage)
            # The weights may need the staged arenas (Port's similarity, FedAdp's dots,
            # Polaris' sums): those device reductions and their host syncs run on the
            # same worker thread, so the event loop is never blocked on the GPU.
            weights, scales = await self._off_loop(self._weights_on_round, rnd, updates)
            with tracing.range("plato_amd.launch"):
                rnd.launch(weights, scales)
            with tracing.range("plato_amd.fetch"):
                return await self._finish(rnd)
        finally:
            # also when a hook, a weight computation or a launch raised: the arrival slots and
            # the payload references they hold must not leak into the next round
            engine.release_arrivals()

    def _weights_on_round(self, rnd, updates):
        self._plato_amd_round = rnd
        try:
            return self.aggregation_weights(updates)
        finally:
            self._plato_amd_round = None


class DeltasAggregationMixin(_EngineHolder):
    """``aggregate_deltas`` hook: GPU weighted sum of already computed deltas."""

    async def aggregate_deltas(self, updates, deltas_received):
        weights, scales = self.aggregation_weights(updates)
        engine = self.round_engine("native")
        rnd = engine.begin(deltas_received[0], len(deltas_received))

        def stage():
            with tracing.range("plato_amd.stage"):
                for slot, delta in enumerate(deltas_received):
                    rnd.put_client(slot, delta, what="deltas_received")

        await self._off_loop(stage)
        with tracing.range("plato_amd.launch"):
            rnd.launch(weights, scales, deltas=True)
        with tracing.range("plato_amd.fetch"):
            return await self._finish(rnd)


def make_server(base=None, mixin=FusedAggregationMixin, name: str = "Server"):
    """Concrete server class = ``mixin`` + ``base`` (default: plato.servers.fedavg.Server)."""
    if base is None:
        try:
            from plato.servers import fedavg as plato_fedavg
        except ImportError as exc:  # pragma: no cover - depends on the install
            raise ImportError(
                "plato_amd.servers.make_server needs TL-System/plato importable "
                "(pip install plato-learn or add it to PYTHONPATH)"
            ) from exc
        base = plato_fedavg.Server
    return type(name, (mixin, base), {"__module__": __name__})


def __getattr__(name):
    # ``plato_amd.servers.fedavg.Server`` resolves against the installed Plato on
    # first use, so importing this module never requires Plato.
    if name == "Server":
        cls = make_server()
        globals()["Server"] = cls
        return cls
    raise AttributeError(name)

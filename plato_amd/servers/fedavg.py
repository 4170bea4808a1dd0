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

from .. import weights as W
from ..arena import payload_codec
from ..engine import FedAvgEngine


class _EngineHolder:
    """Lazily created per-server GPU engine (one process per GPU)."""

    #: torch device string for the engine, e.g. "cuda:0" (None: current device)
    aggregation_device = None
    #: kernel variant override (tuning only; None = library default)
    aggregation_variant = None

    def aggregation_engine(self) -> FedAvgEngine:
        eng = getattr(self, "_plato_amd_engine", None)
        if eng is None:
            eng = FedAvgEngine(self.aggregation_device, variant=self.aggregation_variant)
            self._plato_amd_engine = eng
        return eng

    def aggregation_weights(self, updates):
        """Per-update (weights, second scalars or None), in ``updates`` order.

        FedAvg: ``n_i / N`` with ``self.total_samples = N`` set as the
        reference's aggregate_deltas does (``servers/fedavg.py:140``).
        """
        self.total_samples = sum(update.report.num_samples for update in updates)
        return W.fedavg([update.report.num_samples for update in updates]), None


class FusedAggregationMixin(_EngineHolder):
    """``aggregate_weights`` hook: fused deltas -> weighted sum -> update on the GPU."""

    async def aggregate_weights(self, updates, baseline_weights, weights_received):
        engine = self.aggregation_engine()
        # bf16 payloads (model_quantize on the clients) stay bf16 on the device
        rnd = engine.begin(baseline_weights, len(weights_received), payload_codec(weights_received[0]))
        rnd.put_baseline(baseline_weights)
        for slot, payload in enumerate(weights_received):
            # payloads staged at arrival (WireIngestMixin.stage_on_arrival) are adopted in place
            if not rnd.adopt(slot, payload):
                rnd.put_client(slot, payload)
            # Yield to other tasks in the server between clients, as the
            # reference does per client (servers/fedavg.py:157).
            await asyncio.sleep(0)
        # weights may need the staged arenas (Port's similarity reduction)
        self._plato_amd_round = rnd
        try:
            weights, scales = self.aggregation_weights(updates)
        finally:
            self._plato_amd_round = None
        rnd.launch(weights, scales)
        while not rnd.ready():
            await asyncio.sleep(0)
        result = rnd.result()
        engine.release_arrivals()
        return result


class DeltasAggregationMixin(_EngineHolder):
    """``aggregate_deltas`` hook: GPU weighted sum of already computed deltas."""

    async def aggregate_deltas(self, updates, deltas_received):
        weights, scales = self.aggregation_weights(updates)
        engine = self.aggregation_engine()
        rnd = engine.begin(deltas_received[0], len(deltas_received))
        for slot, delta in enumerate(deltas_received):
            rnd.put_client(slot, delta, what="deltas_received")
            await asyncio.sleep(0)
        rnd.launch(weights, scales, deltas=True)
        while not rnd.ready():
            await asyncio.sleep(0)
        return rnd.result()


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

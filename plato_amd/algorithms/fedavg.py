"""GPU-backed FedAvg algorithm methods (drop-in for plato.algorithms.fedavg.Algorithm).

The reference's server-side algorithm object (plato/algorithms/fedavg.py:10-48)
computes deltas and applies them with torch CPU ops.  These mixins run the same
arithmetic through libplato_agg.so and return CPU ``OrderedDict``s with the
dtypes the reference returns:

* ``compute_weight_deltas`` (``:13-27``): ``x - b`` per client; int64 entries
  stay int64 (exact subtraction).
* ``update_weights`` (``:29-37``): ``b + avg`` in fp32 for every key.
* ``aggregate_weights`` (``algorithms/base.py:44-45``, FedAsync's
  ``fedasync_algorithm.py:9-20``): ``b * (1 - m) + x_0 * m``.

``extract_weights`` / ``load_weights`` stay the reference's (CPU state_dict),
so checkpointing and client-side use are unchanged.  Compose as
``class Algorithm(FedAvgAlgorithmMixin, plato.algorithms.fedavg.Algorithm)``.
"""

from __future__ import annotations

import numpy as np

from ..engine import FedAvgEngine


class _AlgorithmEngine:
    aggregation_device = None
    #: several devices: FedAtt's round is sharded by whole entries over them
    #: (plato_amd.multi.EntryShardedEngine); the other methods use the first
    aggregation_devices = None

    def aggregation_engine(self) -> FedAvgEngine:
        eng = getattr(self, "_plato_amd_engine", None)
        if eng is None:
            devices = self.aggregation_devices
            device = devices[0] if devices else self.aggregation_device
            eng = FedAvgEngine(f"cuda:{device}" if isinstance(device, int) else device)
            self._plato_amd_engine = eng
        return eng

    def entry_engine(self):
        """The engine of per-entry rounds: every device of ``aggregation_devices``, else the one engine."""
        devices = self.aggregation_devices
        if devices is None or len(devices) < 2:
            return self.aggregation_engine()
        multi = getattr(self, "_plato_amd_multi", None)
        if multi is None:
            from ..multi import MultiDeviceEngine

            multi = MultiDeviceEngine([f"cuda:{d}" if isinstance(d, int) else d for d in devices])
            self._plato_amd_multi = multi
        return multi.entries

    async def _off_loop(self, fn, *args):
        """Run ``fn`` on the algorithm's one aggregation worker thread (device work off the event loop)."""
        import asyncio
        import concurrent.futures

        ex = getattr(self, "_plato_amd_executor", None)
        if ex is None:
            ex = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="plato-amd-alg")
            self._plato_amd_executor = ex
        return await asyncio.get_running_loop().run_in_executor(ex, fn, *args)


class FedAvgAlgorithmMixin(_AlgorithmEngine):
    def compute_weight_deltas(self, baseline_weights, weights_received):
        return self.aggregation_engine().compute_weight_deltas(baseline_weights, weights_received)

    def update_weights(self, deltas):
        baseline_weights = self.extract_weights()
        return self.aggregation_engine().update_weights(baseline_weights, deltas)


class FedAsyncAlgorithmMixin(FedAvgAlgorithmMixin):
    async def aggregate_weights(self, baseline_weights, weights_received, mixing=0.9, **kwargs):
        return await self._off_loop(self.aggregation_engine().mix_weights, baseline_weights, weights_received[0],
                                    mixing)


class FedAttAlgorithmMixin(_AlgorithmEngine):
    """FedAtt's attentive aggregation on the GPU.

    examples/server_aggregation/fedatt/fedatt_algorithm.py:23-69:
    ``att[name] = softmax_i(|delta_i[name]|)`` per entry, then
    ``new = b + (-(sum_i -delta_i * att_i) * epsilon + randn * magnitude)``.

    * per-(client, entry) norms: ``plato_agg_entry_norms_f32``, which follows
      torch's CPU reduction order, so they equal the reference's fp32 values;
    * softmax with the same torch op (weights.fedatt_attention);
    * the noise is drawn on the host with ``torch.randn(shape)`` per key in
      baseline order — the reference's own RNG stream, so a seeded run gives
      the reference's bits;
    * ``plato_agg_fedavg_entrywise`` with ``W = -att``, ``scale = -epsilon``,
      ``noise_scale = magnitude``, plus the baseline (``update_weights``).

    ``epsilon`` / ``magnitude`` come from ``Config().algorithm`` like the
    reference (defaults 1.2 / 0.001) unless set on the class.
    """

    fedatt_epsilon = None
    fedatt_magnitude = None

    def _fedatt_param(self, name, default):
        value = getattr(self, f"fedatt_{name}")
        if value is not None:
            return value
        try:
            from plato.config import Config

            alg = Config().algorithm
            return getattr(alg, name) if hasattr(alg, name) else default
        except Exception:  # Plato not importable / not configured
            return default

    async def aggregate_weights(self, baseline_weights, weights_received, **kwargs):
        from collections import OrderedDict

        import torch

        from .. import weights as W

        from ..arena import payload_codec

        # per-(entry, client) norms and a per-entry weighted sum: whole entries shard over several GPUs
        engine = self.entry_engine()
        try:
            rnd = engine.begin(baseline_weights, len(weights_received), payload_codec(weights_received[0]))

            def stage_and_norms():
                rnd.put_baseline(baseline_weights)
                for slot, payload in enumerate(weights_received):
                    if not rnd.adopt(slot, payload):
                        rnd.put_client(slot, payload)
                # coded payloads (bf16 / QSGD): the dequantized rows, every entry float32 as the
                # reference's inbound processor hands them over; native: the round itself
                work = rnd.decoded()
                # the reference's fp32 norms bit for bit (torch's CPU reduction order)
                return work, work.entry_norms(range(len(weights_received)))

            # pack + H2D + the norms launch and its sync run on the worker thread, not the event loop
            work, norms = await self._off_loop(stage_and_norms)
            atts = W.fedatt_attention(norms)  # the reference's softmax
            epsilon = self._fedatt_param("epsilon", 1.2)
            magnitude = self._fedatt_param("magnitude", 0.001)
            # the reference's RNG stream: torch.randn per key in baseline order, on this thread
            noise = OrderedDict((name, torch.randn(weight.shape)) for name, weight in baseline_weights.items())
            await self._off_loop(lambda: work.launch_entrywise(-atts.astype(np.float64), scale=-epsilon, noise=noise,
                                                               noise_scale=magnitude, add_base=True))
            await self._off_loop(work.wait)  # a HIP event wait on the worker thread
            return work.result()
        finally:
            engine.release_arrivals()

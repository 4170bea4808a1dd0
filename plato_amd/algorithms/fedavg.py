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

from ..engine import FedAvgEngine


class _AlgorithmEngine:
    aggregation_device = None

    def aggregation_engine(self) -> FedAvgEngine:
        eng = getattr(self, "_plato_amd_engine", None)
        if eng is None:
            eng = FedAvgEngine(self.aggregation_device)
            self._plato_amd_engine = eng
        return eng


class FedAvgAlgorithmMixin(_AlgorithmEngine):
    def compute_weight_deltas(self, baseline_weights, weights_received):
        return self.aggregation_engine().compute_weight_deltas(baseline_weights, weights_received)

    def update_weights(self, deltas):
        baseline_weights = self.extract_weights()
        return self.aggregation_engine().update_weights(baseline_weights, deltas)


class FedAsyncAlgorithmMixin(FedAvgAlgorithmMixin):
    async def aggregate_weights(self, baseline_weights, weights_received, mixing=0.9, **kwargs):
        return self.aggregation_engine().mix_weights(baseline_weights, weights_received[0], mixing)

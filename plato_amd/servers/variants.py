"""FedAvg-family server variants on the same GPU kernel (weights differ only).

Each mixin overrides :meth:`aggregation_weights` with the reference variant's
per-client numbers (plato_amd/weights.py has the formulas and citations) and
inherits the fused ``aggregate_weights`` hook.  Compose with the reference's
own variant server when its other behaviour (client selection, saving models)
is wanted, e.g. ``class Server(PortWeights, FusedAggregationMixin, port_server.Server)``.
"""

from __future__ import annotations

import os

from .. import weights as W
from .fedavg import FusedAggregationMixin, _EngineHolder


def _config_server():
    try:
        from plato.config import Config

        return Config().server
    except Exception:  # Plato not importable: defaults below apply
        return None


def _cfg(name, default):
    server = _config_server()
    if server is not None and hasattr(server, name):
        return getattr(server, name)
    return default


class FedBuffWeights(_EngineHolder):
    """examples/async/fedbuff/fedbuff_server.py:31-50: every update weighs 1/K."""

    def aggregation_weights(self, updates):
        return W.fedbuff(len(updates)), None


class PortWeights(_EngineHolder):
    """examples/async/port/port_server.py:54-124 (+ staleness_function :134-144).

    The cosine-similarity term is 1.0 unless staleness > 1 and the global model
    of round ``current_round - 2`` exists on disk (``port_server.py:28-34``);
    that case needs the similarity reduction, which :meth:`port_similarities`
    computes on the GPU.
    """

    def port_previous_model_path(self):
        """Where the reference looks for the round-(r-2) global model (port_server.py:28-30)."""
        try:
            from plato.config import Config

            return f"{Config().params['model_path']}/model_{self.current_round - 2}.pth"
        except Exception:  # Plato not importable / not configured
            return None

    def port_similarities(self, updates):
        """1.0, or the fp32 cosine similarity computed on the GPU (port_server.py:24-52)."""
        path = self.port_previous_model_path()
        need = [i for i, u in enumerate(updates) if u.staleness > 1]
        if not need or path is None or not os.path.exists(path):
            return [1.0] * len(updates)
        rnd = getattr(self, "_plato_amd_round", None)
        if rnd is None:
            raise RuntimeError("Port similarities need the staged round (use the fused aggregate_weights hook)")
        import torch

        previous = torch.load(path, map_location="cpu", weights_only=True)
        sims = rnd.model_similarities(previous, need)
        out = [1.0] * len(updates)
        for i, sim in zip(need, sims):
            out[i] = sim
        return out

    #: Port hyper-parameters; None = Config().server.<name>, else the reference default
    similarity_weight = None
    staleness_weight = None
    staleness_bound = None

    def _port_param(self, name, default):
        value = getattr(self, name)
        return _cfg(name, default) if value is None else value

    def aggregation_weights(self, updates):
        self.total_samples = sum(u.report.num_samples for u in updates)
        return W.port(
            [u.report.num_samples for u in updates],
            [u.staleness for u in updates],
            similarities=self.port_similarities(updates),
            similarity_weight=self._port_param("similarity_weight", 1),
            staleness_weight=self._port_param("staleness_weight", 1),
            staleness_bound=self._port_param("staleness_bound", 10),
        ), None


class PiscesWeights(_EngineHolder):
    """examples/client_selection/pisces/pisces_server.py:73-100.

    ``delta * (n/N) * staleness_factor``: two successive fp32 multiplies, so
    the factor goes to the kernel's second-scalar slot.  Appends each update's
    staleness to ``self.client_staleness`` exactly like the reference.
    """

    def aggregation_weights(self, updates):
        self.total_samples = sum(u.report.num_samples for u in updates)
        exponent = getattr(self, "staleness_factor", _cfg("staleness_factor", 1))
        histories = []
        for update in updates:
            hist = self.client_staleness.setdefault(update.client_id, [])
            hist.append(update.staleness)
            histories.append(list(hist))
        first, second = W.pisces([u.report.num_samples for u in updates], histories, exponent)
        return first, second


class FedAsyncMixing(_EngineHolder):
    """examples/async/fedasync: ``b*(1-m) + x_0*m`` with staleness-adapted m."""

    mixing_hyperparam = 0.9
    adaptive_mixing = False

    async def aggregate_weights(self, updates, baseline_weights, weights_received):
        if self.adaptive_mixing:
            fn = _cfg("staleness_weighting_function", None)
            if fn is None:
                self.mixing_hyperparam = W.fedasync_mixing(self.mixing_hyperparam, updates[0].staleness)
            else:
                self.mixing_hyperparam = W.fedasync_mixing(
                    self.mixing_hyperparam, updates[0].staleness, fn.type,
                    getattr(fn, "a", 1), getattr(fn, "b", 0))
        return self.aggregation_engine().mix_weights(baseline_weights, weights_received[0],
                                                     self.mixing_hyperparam)


class GanDeltasAggregationMixin(_EngineHolder):
    """plato/servers/fedavg_gan.py:13-43: FedAvg of (generator, discriminator) delta pairs.

    The two sums are independent and use the same n_i/N weights, so both
    models go into one arena (keys prefixed per model) and one deltas-mode
    launch; the result is split back into the reference's (gen, disc) pair.
    """

    async def aggregate_deltas(self, updates, deltas_received):
        import asyncio
        from collections import OrderedDict

        weights, scales = self.aggregation_weights(updates)
        combined = []
        for gen, disc in deltas_received:
            d = OrderedDict((f"g.{n}", t) for n, t in gen.items())
            d.update((f"d.{n}", t) for n, t in disc.items())
            combined.append(d)
        engine = self.aggregation_engine()
        rnd = engine.begin(combined[0], len(combined))
        for slot, d in enumerate(combined):
            rnd.put_client(slot, d, what="deltas_received")
            await asyncio.sleep(0)
        rnd.launch(weights, scales, deltas=True)
        while not rnd.ready():
            await asyncio.sleep(0)
        avg = rnd.result()
        gen = {n[2:]: t for n, t in avg.items() if n.startswith("g.")}
        disc = {n[2:]: t for n, t in avg.items() if n.startswith("d.")}
        return gen, disc


class FedBuffServerMixin(FedBuffWeights, FusedAggregationMixin):
    pass


class PortServerMixin(PortWeights, FusedAggregationMixin):
    pass


class PiscesServerMixin(PiscesWeights, FusedAggregationMixin):
    pass

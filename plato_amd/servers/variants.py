"""FedAvg-family server variants on the same GPU kernel (weights differ only).

Each mixin overrides :meth:`aggregation_weights` with the reference variant's
per-client numbers (plato_amd/weights.py has the formulas and citations) and
inherits the fused ``aggregate_weights`` hook.  Compose with the reference's
own variant server when its other behaviour (client selection, saving models)
is wanted, e.g. ``class Server(PortWeights, FusedAggregationMixin, port_server.Server)``.
"""

from __future__ import annotations

import os

import numpy as np

from .. import hostorder
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
        threads = torch.get_num_threads() if self.port_threads is None else int(self.port_threads)
        check = hostorder.mode(self.host_order_check)
        if check:  # this host's F.cosine_similarity order (a mismatch warns; "strict" refuses)
            self._plato_amd_host_order_ok = hostorder.check_port(
                rnd.engine.device, threads, strict=check == "strict", align=getattr(rnd.engine, "layout_align", None),
                port_variant=getattr(rnd.engine, "port_variant", None))
        # coded payloads: the per-entry reductions run on the dequantized rows (model_dequantize semantics)
        sims = rnd.decoded().model_similarities(previous, need, threads=threads)
        out = [1.0] * len(updates)
        for i, sim in zip(need, sims):
            out[i] = sim
        return out

    needs_staged_round = True
    #: CPU threads whose reduction order F.cosine_similarity follows; None =
    #: torch.get_num_threads(), the pool the reference's call would use here
    port_threads = None

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
        engine = self.aggregation_engine()
        engine = getattr(engine, "primary", engine)  # one model-sized elementwise pass: one GPU
        # pack + H2D + kernel + D2H on the aggregation worker thread, not the event loop
        return await self._off_loop(engine.mix_weights, baseline_weights, weights_received[0],
                                    self.mixing_hyperparam)


class GanDeltasAggregationMixin(_EngineHolder):
    """plato/servers/fedavg_gan.py:13-43: FedAvg of (generator, discriminator) delta pairs.

    The two sums are independent and use the same n_i/N weights, so both
    models go into one arena (keys prefixed per model) and one deltas-mode
    launch; the result is split back into the reference's (gen, disc) pair.
    """

    async def aggregate_deltas(self, updates, deltas_received):
        from collections import OrderedDict

        weights, scales = self.aggregation_weights(updates)
        combined = []
        for gen, disc in deltas_received:
            d = OrderedDict((f"g.{n}", t) for n, t in gen.items())
            d.update((f"d.{n}", t) for n, t in disc.items())
            combined.append(d)
        engine = self.round_engine("native")
        rnd = engine.begin(combined[0], len(combined))

        def stage():
            for slot, d in enumerate(combined):
                rnd.put_client(slot, d, what="deltas_received")

        await self._off_loop(stage)
        rnd.launch(weights, scales, deltas=True)
        avg = await self._finish(rnd)
        gen = {n[2:]: t for n, t in avg.items() if n.startswith("g.")}
        disc = {n[2:]: t for n, t in avg.items() if n.startswith("d.")}
        return gen, disc


def _staged_round(server, who):
    rnd = getattr(server, "_plato_amd_round", None)
    if rnd is None:
        raise RuntimeError(f"{who} needs the staged round (use the fused aggregate_weights hook)")
    return rnd


def _config_attr(section, name, default):
    try:
        from plato.config import Config

        sec = getattr(Config(), section)
        return getattr(sec, name) if hasattr(sec, name) else default
    except Exception:  # Plato not importable / not configured
        return default


class FedAdpWeights(_EngineHolder):
    """examples/server_aggregation/fedadp/fedadp_server.py:38-133 on the staged round.

    The reference computes ``global_grads = sum_i delta_i * n_i/N`` (``:43-50``),
    the angle of every client's flattened delta with it (``:86-99``), smoothed
    per client into a contribution (``:101-120``), and averages the deltas
    with ``n_i exp(c_i) / sum`` (``:53-68``).  Here:

    1. ``global_grads`` = one ``fedavg_entrywise`` pass (no baseline added),
       left in HBM, bit-exact with the reference's;
    2. ``process_grad``'s flattening (sorted by ``name.lower()``, ``-x/lr``
       after the first entry) and numpy's float32 ``np.inner`` /
       ``np.linalg.norm`` in OpenBLAS's order (``AggregationRound.fedadp_dots``):
       the same float32 values the reference computes;
    3. the host runs the reference's scalar code (weights.fedadp_*), and the
       fused kernel does the final ``b + sum_i delta_i * w_i``.

    ``self.local_angles`` and ``self.adaptive_weighting`` are kept as the
    reference keeps them; ``self.selected_clients`` / ``self.current_round``
    come from the server.
    """

    needs_staged_round = True
    #: every fp32 entry at an arena offset congruent to its flattened position (arena.FEDADP_ALIGN):
    #: the dot kernel's gathers then read whole 128-byte lines
    arena_alignment = "fedadp"
    #: clients staged as deltas x - b (FedAvgEngine.delta_arenas): the dot kernel streams no baseline,
    #: 1.08 against 1.44 ms for 128 ResNet-18 clients, bitwise equal (profiles/r05zzk_delta_probe.log)
    arena_deltas = True

    #: FedAdp's alpha; None = Config().algorithm.alpha, else 5 (fedadp_server.py:112-114)
    fedadp_alpha = None
    #: learning rate of process_grad; None = Config().parameters.optimizer.lr
    fedadp_lr = None

    def aggregation_weights(self, updates):
        # coded payloads: global gradient and dots on the dequantized rows (every entry float32,
        # as model_dequantize hands them to the reference); the final FedAvg stays on the codes
        rnd = _staged_round(self, "FedAdp").decoded()
        if getattr(self, "local_angles", None) is None:
            self.local_angles = {}
        num_samples = [u.report.num_samples for u in updates]
        k = len(updates)
        lay = rnd.layout
        names = lay.keys()
        w1 = np.tile(np.asarray(W.fedavg(num_samples), dtype=np.float64), (len(names), 1))
        grads = rnd.launch_entrywise(w1, add_base=False, device=True)
        lr = self.fedadp_lr
        if lr is None:
            lr = _config_attr("parameters", "optimizer", None)
            lr = getattr(lr, "lr", None) if lr is not None else None
            if lr is None:
                raise ValueError("FedAdp needs parameters.optimizer.lr (or set fedadp_lr)")
        alpha = self.fedadp_alpha if self.fedadp_alpha is not None else _config_attr("algorithm", "alpha", 5)
        check = hostorder.mode(self.host_order_check)
        if check:  # this host's numpy sdot order (a mismatch warns; "strict" refuses)
            self._plato_amd_host_order_ok = hostorder.check_fedadp(
                rnd.engine.device, lr, strict=check == "strict", align=getattr(rnd.engine, "layout_align", None),
                deltas=bool(getattr(rnd, "deltas", False)))
        inner, g_sq, l_sq = rnd.fedadp_dots(grads, range(k), lr)
        angles = W.fedadp_angles_from_dots(inner, g_sq, l_sq)
        contribs = W.fedadp_contributions(angles, self.selected_clients, self.local_angles,
                                          self.current_round, alpha)
        self.adaptive_weighting = W.fedadp_weighting(contribs, num_samples)
        return self.adaptive_weighting, None


class PolarisWeights(_EngineHolder):
    """examples/client_selection/polaris/polaris_server.py:68-100 on the staged round.

    FedAvg weights, plus the per-client norm of the conv-layer deltas the
    reference records for its client-selection solver
    (``self.squared_deltas_current_round``, ``self.unexplored_clients``):
    each layer's ``np.sum(np.square(delta))`` in numpy's own float32 order on
    the device (``AggregationRound.np_sumsq``), then the reference's float32
    scalar code.  The solver itself (cvxopt/mosek, ``:129-186``) stays the
    reference's.
    """

    needs_staged_round = True
    entry_local_weights = True  # per-layer sums: sharded by whole entries over aggregation_devices
    #: clients staged as deltas x - b (FedAvgEngine.delta_arenas): the sums load no baseline, 0.918-0.921
    #: against 0.972-0.980 ms for 128 ResNet-18 clients, bitwise equal (profiles/r05zzzg_polaris_deltas.log)
    arena_deltas = True

    def aggregation_weights(self, updates):
        weights, scales = super().aggregation_weights(updates)  # FedAvg n_i/N, sets total_samples
        rnd = _staged_round(self, "Polaris")
        # numpy's float32 np.sum(np.square(delta)) per layer (coded payloads: on the dequantized rows)
        sums = rnd.decoded().np_sumsq(range(len(updates)))
        norms = W.polaris_delta_norms(sums, rnd.layout.keys())
        self.squared_deltas_current_round = np.zeros(self.number_of_client)
        sum_deltas_current_round = 0
        deltas_counter = 0
        for update, norm in zip(updates, norms):
            self.squared_deltas_current_round[update.client_id - 1] = norm
            if (update.client_id - 1) in self.unexplored_clients:
                self.unexplored_clients.remove(update.client_id - 1)
            sum_deltas_current_round += norm
            deltas_counter += 1
        avg_deltas_current_round = sum_deltas_current_round / deltas_counter
        expect_deltas = self.alpha * avg_deltas_current_round
        for client_counter in range(200):  # the reference's literal bound (polaris_server.py:96)
            if client_counter in self.unexplored_clients:
                self.squared_deltas_current_round[client_counter] = expect_deltas
        return weights, scales


class FedBuffServerMixin(FedBuffWeights, FusedAggregationMixin):
    pass


class PortServerMixin(PortWeights, FusedAggregationMixin):
    pass


class PiscesServerMixin(PiscesWeights, FusedAggregationMixin):
    pass


class FedAdpServerMixin(FedAdpWeights, FusedAggregationMixin):
    pass


class PolarisServerMixin(PolarisWeights, FusedAggregationMixin):
    pass


def rl_smart_weights(smart_weighting, k: int, has_int64: bool):
    """How the RL server's ``smart_weighting`` multiplies each kind of entry (rl_server.py:66-71).

    Returns ``(weights for fp32 entries, weights for int64 entries, float64?)``:
    ``delta * smart_weighting[i]`` for float entries — a float64 row of a
    [K, 1] array makes the product float64 (numpy promotion) and the in-place
    add then runs in float64; a float32 row or a scalar keeps torch's fp32
    chain — and ``delta * smart_weighting[i][0]`` (a scalar: fp32 chain) for
    int64 entries.
    """
    sw = np.asarray(smart_weighting)
    if sw.shape[0] != k:
        raise ValueError(f"smart_weighting has {sw.shape[0]} rows for {k} updates")
    if sw.ndim == 1:
        if has_int64:
            raise TypeError("the reference indexes smart_weighting[i][0] for int64 entries: a [K, m] array is needed")
        return [float(v) for v in sw], None, False
    if sw.ndim != 2 or sw.shape[1] != 1:
        raise ValueError("smart_weighting rows must hold one number ([K, 1]); wider rows broadcast per element")
    col = [float(v) for v in sw[:, 0]]
    return col, col, sw.dtype == np.float64


class RLDeltasAggregationMixin(_EngineHolder):
    """plato/utils/reinforcement_learning/rl_server.py:45-80: smart-weighted aggregate_deltas on the GPU.

    The agent handshake (``update_state``, ``agent.prep_agent_update``,
    ``update_action`` -> ``apply_action``) runs exactly as in the reference;
    the weighted sum of the deltas runs on the device with the reference's
    per-entry-type weight semantics (:func:`rl_smart_weights`): a float64
    action puts the fp32 entries on float64 arithmetic
    (``plato_agg_fedavg_w64``), while the int64 entries keep fp32 weights.
    Compose as ``class Server(RLDeltasAggregationMixin, MyRLServer)``.
    """

    async def aggregate_deltas(self, updates, deltas_received):
        self.update_state()
        num_samples = [update.report.num_samples for update in updates]
        self.total_samples = sum(num_samples)
        self.agent.num_samples = num_samples
        await self.agent.prep_agent_update()
        await self.update_action()

        engine = self.round_engine("native")
        engine = getattr(engine, "primary", engine)  # float64 weights: one device
        rnd = engine.begin(deltas_received[0], len(deltas_received))
        w, w_i64, f64 = rl_smart_weights(self.smart_weighting, len(deltas_received), rnd.layout.n_i64 > 0)

        def stage():
            for slot, delta in enumerate(deltas_received):
                rnd.put_client(slot, delta, what="deltas_received")

        await self._off_loop(stage)
        if f64:
            rnd.launch_w64(w, w_i64, deltas=True)
        else:
            rnd.launch(w, None, deltas=True)
        return await self._finish(rnd)


class HEHybridMixin(_EngineHolder):
    """plato/servers/fedavg_he.py:66-106: the plaintext half of hybrid FedAvg on the GPU.

    The CKKS half (tenseal vectors) stays the reference's; the unencrypted
    float64 vectors are summed by :meth:`FedAvgEngine.weighted_sum` with the
    reference's float64 promotion.  The reference's ``aggregate_weights``
    (``fedavg_he.py:50-64``) calls ``_fedavg_hybrid`` synchronously on the event
    loop; here the hybrid sum is formed first on the aggregation worker thread
    and the reference's method then picks it up, so its decrypt / serialize
    steps run unchanged.  Compose as ``class Server(HEHybridMixin, fedavg_he.Server)``.
    """

    async def aggregate_weights(self, updates, baseline_weights, weights_received):
        self._plato_amd_hybrid = await self._off_loop(self._fedavg_hybrid_device, updates)
        try:
            return await super().aggregate_weights(updates, baseline_weights, weights_received)
        finally:
            self._plato_amd_hybrid = None

    def _fedavg_hybrid(self, updates):
        done = getattr(self, "_plato_amd_hybrid", None)
        if done is not None:
            return done
        return self._fedavg_hybrid_device(updates)

    def _fedavg_hybrid_device(self, updates):
        from plato.utils import homo_enc

        weights_received = [homo_enc.deserialize_weights(update.payload, self.context) for update in updates]
        unencrypted_weights = [homo_enc.extract_encrypted_model(x)[0] for x in weights_received]
        encrypted_weights = [homo_enc.extract_encrypted_model(x)[1] for x in weights_received]
        indices = [homo_enc.extract_encrypted_model(x)[2] for x in weights_received]
        for i in range(1, len(indices)):
            assert indices[i] == indices[0]
        encrypt_indices = indices[0]
        self.total_samples = sum(update.report.num_samples for update in updates)
        factors = [update.report.num_samples / self.total_samples for update in updates]
        engine = self.aggregation_engine()
        engine = getattr(engine, "primary", engine)
        unencrypted_avg_update = engine.weighted_sum(unencrypted_weights, factors)
        encrypted_avg_update = self.trainer.zeros(encrypted_weights[0].size())
        for enc_w, factor in zip(encrypted_weights, factors):
            encrypted_avg_update += enc_w * factor
        if len(encrypt_indices) == 0:
            encrypted_avg_update = None
        return homo_enc.wrap_encrypted_model(unencrypted_avg_update, encrypted_avg_update, encrypt_indices)

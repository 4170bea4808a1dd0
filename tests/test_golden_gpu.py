"""GPU parity against the reference-generated golden fixtures (bit-exact).

Every case of tests/golden/fedavg_cases.json is replayed on the MI355X:
inputs are generated in HBM by plato_agg_fill_synth_* (restated by
oracle/synth.py, which the fixture generator fed to the reference), edge-value
overrides are written into the device arenas, weights come from the product's
host functions (plato_amd.weights), and the kernel output digests must equal
the reference's.  The server-plugin test drives the product's aggregate hooks
the way the reference's _process_reports does (plato/servers/fedavg.py:171-182).
"""

import asyncio
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from oracle import synth
from plato_amd import weights as W
from plato_amd.arena import ArenaLayout
from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine, cast_to_int64, fp32_weights
from plato_amd.synthetic import fill_baseline, fill_clients
from tests import golden_cases as G

pytestmark = pytest.mark.gpu
CASES = G.load_cases()
DEV = "cuda:0"


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine(DEV)


def _device_inputs(recipe):
    dev = torch.device(DEV)
    layout = ArenaLayout.from_shapes(G.model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    fill_baseline(base, seed)
    fill_clients(slab, base, seed, k)
    for tgt, region, idx, val in recipe.get("overrides", []):
        if region == "f32":
            v = torch.from_numpy(np.array([int(val, 16)], dtype=np.uint32).view(np.float32)).to(dev)
            (base.f32 if tgt == "base" else slab.f32[tgt])[idx : idx + 1].copy_(v)
        else:
            v = torch.tensor([int(val)], dtype=torch.int64, device=dev)
            (base.i64 if tgt == "base" else slab.i64[tgt])[idx : idx + 1].copy_(v)
    for dst, src, n in G.tied_ranges(recipe, layout):  # tied weights: one storage under two keys
        for arr in [base.f32, *slab.f32]:
            arr[dst:dst + n].copy_(arr[src:src + n])
    torch.cuda.synchronize()
    return layout, base, slab


def _launch(engine, layout, base, slab, order, weights, scales, deltas=False):
    dev = torch.device(DEV)
    pf, pi = slab.row_pointers(order)
    tf = torch.from_numpy(pf).to(dev)
    ti = torch.from_numpy(pi).to(dev)
    w = torch.from_numpy(fp32_weights(weights)).to(dev)
    s = None if scales is None else torch.from_numpy(fp32_weights(scales)).to(dev)
    out_f = torch.empty(layout.row_f32, device=dev)
    out_i = torch.empty(layout.row_i64, device=dev)
    engine.launch_fedavg(layout, tf, ti, w, s, len(order), None if deltas else base.f32,
                         None if deltas else base.i64, out_f, out_i)
    torch.cuda.synchronize()
    return out_f, out_i


NON_ASYNC = [c for c in CASES
             if c["recipe"].get("mode", "fedavg") not in ("fedasync", "gan") + G.PER_ENTRY_MODES + G.OWN_TEST_MODES
             and c["recipe"].get("codec") is None]
BF16 = [c for c in CASES if c["recipe"].get("codec") == "bf16"
        and G.plain_fedavg_weights(c["recipe"])]


@pytest.mark.parametrize("case", NON_ASYNC, ids=[c["recipe"]["name"] for c in NON_ASYNC])
def test_kernel_matches_reference(engine, case):
    recipe, exp = case["recipe"], case["expected"]
    layout, base, slab = _device_inputs(recipe)
    order = G.order_of(recipe)
    # Port with a stored stale model: the reference's own similarity values
    weights, scales = G.weights_for(recipe, W, G.reference_similarities(case))
    out_f, out_i = _launch(engine, layout, base, slab, order, weights, scales)
    got_f = out_f[: layout.n_f32].cpu().numpy()
    got_i = out_i[: layout.n_i64].cpu().numpy()
    assert G.sha(G.canon(got_f)) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(got_i)) == exp["updated_i64f_sha256"]
    # load_state_dict's truncating copy, on the device
    loaded = cast_to_int64(out_i[: layout.n_i64]).cpu().numpy() if layout.n_i64 else np.zeros(0, np.int64)
    assert G.sha(loaded) == exp["loaded_i64_sha256"]
    del slab, base
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["lenet5_k10_skewed", "resnet18_k16", "pisces_resnet18_k8",
                                  "resnet18_k5_int64_edges", "lenet5_k7_edge_values"])
def test_deltas_kernel_matches_reference_aggregate_deltas(engine, name):
    """aggregate_deltas alone: deltas formed on the device, summed by the deltas-mode kernel."""
    case = next(c for c in CASES if c["recipe"]["name"] == name)
    recipe, exp = case["recipe"], case["expected"]
    layout, base, slab = _device_inputs(recipe)
    from plato_amd import _lib

    h = torch.cuda.current_stream().cuda_stream
    for r in range(recipe["k"]):  # in place: row r <- row r - baseline
        _lib.call("plato_agg_compute_deltas", slab.f32[r].data_ptr(), slab.i64[r].data_ptr(),
                  base.f32.data_ptr(), base.i64.data_ptr(), slab.f32[r].data_ptr(), slab.i64[r].data_ptr(),
                  layout.n_f32, layout.n_i64, h)
    weights, scales = G.weights_for(recipe, W)
    out_f, out_i = _launch(engine, layout, base, slab, G.order_of(recipe), weights, scales, deltas=True)
    assert G.sha(G.canon(out_f[: layout.n_f32].cpu().numpy())) == exp["avg_f32_sha256"]
    assert G.sha(G.canon(out_i[: layout.n_i64].cpu().numpy())) == exp["avg_i64f_sha256"]


def test_full_arrays_small_cases(engine):
    full = G.load_full()
    for case in CASES:
        recipe = case["recipe"]
        if not recipe.get("full") or recipe.get("codec") or recipe.get("mode") in G.PER_ENTRY_MODES + G.OWN_TEST_MODES:
            continue
        layout, base, slab = _device_inputs(recipe)
        weights, scales = G.weights_for(recipe, W, G.reference_similarities(case))
        out_f, _ = _launch(engine, layout, base, slab, G.order_of(recipe), weights, scales)
        got = G.canon(out_f[: layout.n_f32].cpu().numpy())
        assert got.tobytes() == G.canon(full[f"{recipe['name']}/updated_f32"]).tobytes(), recipe["name"]


def _host_payloads(recipe):
    layout = ArenaLayout.from_shapes(G.model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    xs_f = [x[0] for x in xs]
    xs_i = [x[1] for x in xs]
    G.apply_overrides(bf, bi, xs_f, xs_i, recipe.get("overrides", []))
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [layout.unpack(torch.from_numpy(xs_f[c]), torch.from_numpy(xs_i[c])) for c in range(k)]
    return layout, baseline, payloads


def _updates(recipe, payloads):
    st = recipe.get("staleness", [0] * recipe["k"])
    return [types.SimpleNamespace(client_id=c + 1,
                                  report=types.SimpleNamespace(num_samples=recipe["num_samples"][c]),
                                  payload=payloads[c], staleness=st[c])
            for c in G.order_of(recipe)]


def _flat(layout, sd, region):
    return torch.cat([sd[e.name].reshape(-1).float() for e in layout.entries if e.region == region]).numpy() \
        if any(e.region == region for e in layout.entries) else np.zeros(0, np.float32)


@pytest.mark.parametrize("name,mixin", [
    ("resnet18_k16_permuted", "FusedAggregationMixin"),
    ("fedbuff_resnet18_k16", "FedBuffServerMixin"),
    ("port_resnet18_k16", "PortServerMixin"),
    ("pisces_resnet18_k8", "PiscesServerMixin"),
    ("lenet5_k7_edge_values", "DeltasAggregationMixin"),
    # async simulated wall time: updates in the order the reference's _process_clients formed them
    ("async_wall_resnet18_k12", "FusedAggregationMixin"),
    # cross-silo (fedavg_cs._process_reports dispatches to the same hooks)
    ("cross_silo_resnet18_k6", "FusedAggregationMixin"),
    ("cross_silo_lenet5_k4_edges", "DeltasAggregationMixin"),
])
def test_server_hooks_match_reference(name, mixin):
    """The product's Plato hooks, dispatched like _process_reports (servers/fedavg.py:171-196)."""
    from plato_amd.servers import fedavg as S
    from plato_amd.servers import variants as V

    case = next(c for c in CASES if c["recipe"]["name"] == name)
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    updates = _updates(recipe, payloads)
    base_cls = getattr(S, mixin, None) or getattr(V, mixin)

    class Server(base_cls):
        aggregation_device = DEV
        staleness_factor = 0.5  # Pisces exponent (golden config)
        staleness_weight = 3    # Port (golden config: similarity 1, staleness 3, bound 10)

        def __init__(self):
            self.client_staleness = {}
            self.current_round = 0

    server = Server()
    received = [u.payload for u in updates]
    if hasattr(server, "aggregate_weights"):
        updated = asyncio.run(server.aggregate_weights(updates, baseline, received))
    else:
        # the reference's own delta/update steps around the hook (algorithms/fedavg.py:23,35)
        deltas = [{n: p[n] - baseline[n] for n in p} for p in received]
        avg = asyncio.run(server.aggregate_deltas(updates, deltas))
        assert G.sha(G.canon(_flat(layout, avg, "f32"))) == exp["avg_f32_sha256"]
        updated = {n: baseline[n] + avg[n] for n in baseline}
    assert list(updated.keys()) == [e.name for e in layout.entries]
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    if recipe.get("mode") in ("fedavg", "port", "pisces", "cross_silo", "async_wall", None):
        assert server.total_samples == sum(recipe["num_samples"])


def test_fedasync_mixing_matches_reference():
    from plato_amd.servers.variants import FedAsyncMixing

    case = next(c for c in CASES if c["recipe"].get("mode") == "fedasync")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)

    class Server(FedAsyncMixing):
        aggregation_device = DEV
        mixing_hyperparam = 0.9
        adaptive_mixing = False

    server = Server()
    server.mixing_hyperparam = W.fedasync_mixing(0.9, recipe["staleness"][0], "hinge", 10, 4)
    updated = asyncio.run(server.aggregate_weights(_updates(recipe, payloads), baseline, payloads))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]


def _previous(recipe, layout):
    pv = recipe["previous"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, recipe["seed"])
    prev_f = synth.synth_f32(layout.n_f32, recipe["seed"], pv["stream"], pv["scale"], add=bf)
    prev_i = synth.synth_i64(layout.n_i64, recipe["seed"], pv["stream"], 3, add=bi)
    return layout.unpack(torch.from_numpy(prev_f), torch.from_numpy(prev_i))


# the similarity fixtures were generated with torch's default pool of the 8-CPU survey host
FIXTURE_TORCH_THREADS = 8


@pytest.mark.parametrize("name", ["port_similarity_lenet5_k8", "port_similarity_resnet18_k4"])
def test_device_similarities_match_reference(engine, name):
    """Flatten -> torch-order norms -> torch-order cascade sum == the reference's F.cosine_similarity bits."""
    case = next(c for c in CASES if c["recipe"]["name"] == name)
    recipe = case["recipe"]
    layout, baseline, payloads = _host_payloads(recipe)
    rnd = engine.begin(baseline, recipe["k"])
    rnd.put_baseline(baseline)
    for c in range(recipe["k"]):
        rnd.put_client(c, payloads[c])
    sims = rnd.model_similarities(_previous(recipe, layout), range(recipe["k"]), threads=FIXTURE_TORCH_THREADS)
    ref_sims = G.reference_similarities(case)
    st = recipe["staleness"]
    checked = 0
    for i in range(recipe["k"]):
        if st[i] > 1:  # the reference computed it
            assert np.float32(sims[i]).tobytes() == np.float32(ref_sims[i]).tobytes(), (i, sims[i], ref_sims[i])
            checked += 1
    assert checked
    # other thread counts: the oracle restatement of the same order
    from oracle import reductions as R

    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, recipe["seed"])
    pv = recipe["previous"]
    pf = synth.synth_f32(layout.n_f32, recipe["seed"], pv["stream"], pv["scale"], add=bf)
    pi = synth.synth_i64(layout.n_i64, recipe["seed"], pv["stream"], 3, add=bi)
    v = R.port_current_minus_previous(layout.entries, bf, bi, pf, pi)
    for threads in (1, 16):
        sims = rnd.model_similarities(_previous(recipe, layout), range(recipe["k"]), threads=threads)
        for i in range(recipe["k"]):
            xf, xi = synth.client_arena(bf, bi, recipe["seed"], i)
            d = R.port_delta(layout.entries, bf, bi, xf, xi)
            assert np.float32(sims[i]).tobytes() == R.torch_cosine(v, d, threads).tobytes(), (threads, i)


def test_port_server_with_stale_model_matches_reference(tmp_path):
    """PortServerMixin end to end with a stored round-(r-2) model: the reference's model bit for bit."""
    from plato_amd.servers.variants import PortServerMixin

    case = next(c for c in CASES if c["recipe"]["name"] == "port_similarity_lenet5_k8")
    recipe = case["recipe"]
    layout, baseline, payloads = _host_payloads(recipe)
    path = tmp_path / f"model_{recipe['current_round'] - 2}.pth"
    torch.save(_previous(recipe, layout), path)

    class Server(PortServerMixin):
        aggregation_device = DEV
        staleness_weight = 3
        current_round = recipe["current_round"]
        port_threads = FIXTURE_TORCH_THREADS

        def port_previous_model_path(self):
            return str(path)

    updated = asyncio.run(Server().aggregate_weights(_updates(recipe, payloads), baseline, payloads))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == case["expected"]["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == case["expected"]["updated_i64f_sha256"]


def test_wire_ingested_payloads_match_reference(engine):
    """Pickled payload bytes -> native ingest (pinned arenas) -> engine: reference digest."""
    import pickle

    from plato_amd import ingest

    case = next(c for c in CASES if c["recipe"]["name"] == "resnet18_k16_permuted")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    order = G.order_of(recipe)
    # one storage per tensor, like a client's model.state_dict() (views of one
    # arena would each pickle the whole arena)
    wire = [pickle.dumps(type(payloads[c])((n, t.clone()) for n, t in payloads[c].items())) for c in order]
    received = [ingest.loads(w, layout=layout, pin=True) for w in wire]
    assert all(isinstance(r, ingest.ArenaStateDict) for r in received)
    weights, _ = G.weights_for(recipe, W)
    updated = engine.aggregate_weights(baseline, received, weights)
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]


def test_zstd_compressed_payloads_match_reference(engine):
    """model_compress'd payloads -> native zstd + pickle ingest (zstd Processor) -> engine: reference digest."""
    from plato_amd import ingest
    from plato_amd.processors import zstd as zp

    if not ingest.zstd_available():
        pytest.skip("libzstd.so.1 absent")
    case = next(c for c in CASES if c["recipe"]["name"] == "resnet18_k16_permuted")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    order = G.order_of(recipe)
    client = zp.CompressProcessor(compression_level=1)
    wire = [client.process(type(payloads[c])((n, t.clone()) for n, t in payloads[c].items())) for c in order]
    server = zp.Processor(server_id=0, layout=layout)
    received = [server.process(w) for w in wire]
    assert all(isinstance(r, ingest.ArenaStateDict) and r.arena_f32.is_pinned() for r in received)
    weights, _ = G.weights_for(recipe, W)
    updated = engine.aggregate_weights(baseline, received, weights)
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]


def _bf16_payloads(recipe):
    layout, baseline, payloads = _host_payloads(recipe)
    # client side: Plato's model_quantize (.to(bfloat16)) of every entry
    return layout, baseline, [type(p)((n, t.to(torch.bfloat16)) for n, t in p.items()) for p in payloads]


@pytest.mark.parametrize("case", BF16, ids=[c["recipe"]["name"] for c in BF16])
def test_bf16_codec_device_resident_matches_reference(engine, case):
    """bf16 payloads kept bf16 in HBM, widened in registers == reference dequantize + FedAvg."""
    from plato_amd import _lib

    recipe, exp = case["recipe"], case["expected"]
    layout, base, slab32 = _device_inputs(recipe)
    slab = ClientSlab(layout, recipe["k"], torch.device(DEV), codec="bf16")
    slab.f32.copy_(slab32.f32.to(torch.bfloat16))          # model_quantize, on the device
    slab.i64.copy_(slab32.i64.to(torch.bfloat16))
    del slab32
    order = G.order_of(recipe)
    pf, pi = slab.row_pointers(order)
    tf, ti = torch.from_numpy(pf).to(DEV), torch.from_numpy(pi).to(DEV)
    weights, _ = G.weights_for(recipe, W)
    w = torch.from_numpy(fp32_weights(weights)).to(DEV)
    out_f = torch.empty(layout.row_f32, device=DEV)
    out_i = torch.empty(layout.row_i64, device=DEV)
    n_i = layout.n_i64
    for v in range(_lib.tune().plato_agg_tune_num_bf16_variants()):  # every variant, bit for bit
        out_f.fill_(float("nan"))
        _lib.tune_call("plato_agg_tune_fedavg_bf16", v, tf.data_ptr(), ti.data_ptr() if n_i else None, w.data_ptr(),
                  None, len(order), base.f32.data_ptr(), base.i64.data_ptr() if n_i else None, out_f.data_ptr(),
                  out_i.data_ptr() if n_i else None, layout.n_f32, n_i, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert G.sha(G.canon(out_f[: layout.n_f32].cpu().numpy())) == exp["updated_f32_sha256"], v
        assert G.sha(G.canon(out_i[: layout.n_i64].cpu().numpy())) == exp["updated_i64f_sha256"], v


@pytest.mark.parametrize("case", BF16, ids=[c["recipe"]["name"] for c in BF16])
def test_bf16_codec_host_and_wire_paths_match_reference(engine, case):
    import pickle

    from plato_amd import ingest

    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _bf16_payloads(recipe)
    weights, _ = G.weights_for(recipe, W)
    order = G.order_of(recipe)
    # host state_dicts (auto-detected codec)
    updated = engine.aggregate_weights(baseline, [payloads[c] for c in order], weights)
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    # from the wire: pickled bf16 payloads -> native ingest -> bf16 arenas
    wire = [pickle.dumps(type(payloads[c])((n, t.clone()) for n, t in payloads[c].items())) for c in order]
    received = [ingest.loads(b, layout=layout, pin=True) for b in wire]
    assert received[0].arena_f32.dtype == torch.bfloat16
    updated = engine.aggregate_weights(baseline, received, weights)
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]


def test_gan_deltas_match_reference():
    """GanDeltasAggregationMixin == fedavg_gan.Server.aggregate_deltas (servers/fedavg_gan.py:13-43)."""
    from collections import OrderedDict

    from plato_amd.servers.variants import GanDeltasAggregationMixin

    case = next(c for c in CASES if c["recipe"].get("mode") == "gan")
    recipe, exp = case["recipe"], case["expected"]
    k, seed = recipe["k"], recipe["seed"]
    parts = []
    for j, name in enumerate(recipe["models"]):
        layout = ArenaLayout.from_shapes(G.model_spec(name))
        bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed + j)
        base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
        deltas = []
        for c in range(k):
            xf, xi = synth.client_arena(bf, bi, seed + j, c)
            x = layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi))
            deltas.append(OrderedDict((n, x[n] - base[n]) for n in x))
        parts.append((layout, deltas))

    class Server(GanDeltasAggregationMixin):
        aggregation_device = DEV

    server = Server()
    updates = [types.SimpleNamespace(report=types.SimpleNamespace(num_samples=n)) for n in recipe["num_samples"]]
    gen, disc = asyncio.run(server.aggregate_deltas(updates, [(parts[0][1][c], parts[1][1][c]) for c in range(k)]))
    for tag, (layout, _), avg in (("gen", parts[0], gen), ("disc", parts[1], disc)):
        assert G.sha(G.canon(_flat(layout, avg, "f32"))) == exp[f"{tag}_avg_f32_sha256"]
        assert G.sha(G.canon(_flat(layout, avg, "i64"))) == exp[f"{tag}_avg_i64f_sha256"]
    assert server.total_samples == exp["total_samples"]


def test_weighted_sum_matches_sequential_loop(engine):
    """HE hybrid plaintext part (fedavg_he.py:88-98): avg += w_i * n_i/N, flat vectors."""
    from oracle import fedavg_oracle as ref

    rng = np.random.default_rng(3)
    vecs = [rng.standard_normal(100_003).astype(np.float32) for _ in range(7)]
    ns = [5, 100, 33, 2, 77, 9, 41]
    got = engine.weighted_sum([torch.from_numpy(v) for v in vecs], W.fedavg(ns)).numpy()
    exp, _ = ref.deltas_numpy(vecs, [np.zeros(0, np.int64)] * 7, ref.fedavg_weights(ns))
    assert got.tobytes() == exp.tobytes()


def _arrival_delta_keys(eng, kind: str, layout) -> list:
    """Per arrived payload: the key of the model its rows were turned into deltas against (None: weights)."""
    if kind == "single":
        return [hit[8] for hit in eng._arrivals.values()]
    if kind in ("multi", "clients"):
        return [hit[7] for hit in eng._arrivals.values()]
    ent = eng.entries
    parts = ent.plan(layout)[1]
    keys = []
    for _, _, subs in ent._arrivals.values():
        per = [ent._engines[g]._arrivals[id(sub)][8] for (g, _), sub in zip(parts, subs)]
        keys.append(None if any(k is None for k in per) else tuple(per))
    return keys


def _arrivals_of(eng, kind: str) -> dict:
    return eng.entries._arrivals if kind == "entry" else eng._arrivals


@pytest.mark.parametrize("engine_kind", ["single", "multi", "entry", "clients"])
@pytest.mark.parametrize("mode", ["weights", "deltas", "deltas_stale", "deltas_data_write"])
def test_stage_on_arrival_then_adopt_matches_reference(mode, engine_kind):
    """Payloads staged to HBM as they arrive (any arrival order), summed in updates order.

    "deltas": the server stages arrivals as deltas against its current model (arena_deltas), adopted by a
    round on that model; "deltas_stale": the model the arrivals were turned into deltas against is another
    one (other storage), so the round stages every payload again from its host tensors;
    "deltas_data_write": the arrivals were turned into deltas while the model held other values, written
    and then restored through ``.data`` (no version-counter bump: the keys still match), so only the
    device-side comparison of the two staged baselines makes the round stage the payloads again.
    ``engine_kind``: one GPU; the multi-GPU engine's bucket rounds, entry shards and client-split rounds
    (two repeated devices on a one-GPU box)."""
    import pickle

    from plato_amd.servers import FusedAggregationMixin, WireIngestMixin
    from plato_amd.staging import baseline_key

    case = next(c for c in CASES if c["recipe"]["name"] == "resnet18_k16_permuted")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)

    at_arrival = (OrderedDict((n, t.clone()) for n, t in baseline.items()) if mode == "deltas_stale"
                  else baseline)
    if mode == "deltas_data_write":
        saved = OrderedDict((n, t.clone()) for n, t in baseline.items())
        key0 = baseline_key(baseline)
        for t in baseline.values():
            t.data.add_(1)

    class Algo:
        def extract_weights(self):
            return at_arrival

    class Server(WireIngestMixin, FusedAggregationMixin):
        aggregation_device = DEV if engine_kind == "single" else None
        aggregation_devices = None if engine_kind == "single" else [DEV, DEV]
        needs_staged_round = engine_kind in ("entry", "clients")
        entry_local_weights = engine_kind == "entry"
        client_split_rounds = engine_kind == "clients"
        stage_on_arrival = True
        arena_deltas = mode != "weights"

        def __init__(self):
            self.algorithm = Algo()
            self.client_chunks, self.client_payload, self.training_clients = {}, {}, {}

    server = Server()
    arrived = {}
    for c in reversed(range(recipe["k"])):  # arrival order differs from the update order
        sid = f"s{c}"
        server.client_chunks[sid] = [pickle.dumps(type(payloads[c])((n, t.clone()) for n, t in payloads[c].items()))]
        server.client_payload[sid] = None
        server.training_clients[c + 1] = True
        asyncio.run(server._client_payload_arrived(sid, c + 1))
        arrived[c] = server.client_payload[sid]
    eng = server.aggregation_engine()
    if mode == "deltas_data_write":
        for n, t in baseline.items():
            t.data.copy_(saved[n])
        assert baseline_key(baseline) == key0  # the in-place writes left every key as it was
    keys = _arrival_delta_keys(eng, engine_kind, layout)
    assert len(keys) == recipe["k"]
    # the arrival rows hold deltas (keyed by the model they were formed against) exactly when asked
    assert all((key is not None) == (mode != "weights") for key in keys)
    updates = _updates(recipe, [arrived[c] for c in range(recipe["k"])])
    updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    assert len(_arrivals_of(eng, engine_kind)) == 0  # released after the round


RL = [c for c in CASES if c["recipe"].get("mode") in ("rl", "rl_f32")]


@pytest.mark.parametrize("case", RL, ids=[c["recipe"]["name"] for c in RL])
def test_rl_smart_weighting_matches_reference(case):
    """RLDeltasAggregationMixin == rl_server.RLServer.aggregate_deltas (float64 and float32 actions)."""
    from plato_amd.servers.variants import RLDeltasAggregationMixin

    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    updates = _updates(recipe, payloads)
    dtype = np.float64 if recipe["mode"] == "rl" else np.float32

    class Agent:
        num_samples = None

        async def prep_agent_update(self):
            return None

    class Server(RLDeltasAggregationMixin):
        aggregation_device = DEV
        agent = Agent()

        def update_state(self):
            self.state_updated = True

        async def update_action(self):
            self.smart_weighting = np.array([[float.fromhex(h)] for h in recipe["action"]], dtype=dtype)

    server = Server()
    deltas = [{n: p[n] - baseline[n] for n in p} for p in [u.payload for u in updates]]
    avg = asyncio.run(server.aggregate_deltas(updates, deltas))
    assert server.state_updated and server.agent.num_samples == [u.report.num_samples for u in updates]
    assert G.sha(G.canon(_flat(layout, avg, "f32"))) == exp["avg_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, avg, "i64"))) == exp["avg_i64f_sha256"]
    updated = {n: baseline[n] + avg[n] for n in baseline}  # the reference's update_weights
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert server.total_samples == exp["total_samples"]


HE = [c for c in CASES if c["recipe"].get("mode") == "he"]


@pytest.mark.parametrize("case", HE, ids=[c["recipe"]["name"] for c in HE])
def test_he_plaintext_half_matches_reference(engine, case):
    """fedavg_he._fedavg_hybrid's unencrypted sum: float64 vectors, float64 accumulation, on the GPU."""
    from tests.test_oracle import he_vectors

    recipe, exp = case["recipe"], case["expected"]
    vecs = he_vectors(recipe)
    got = engine.weighted_sum(vecs, W.fedavg(recipe["num_samples"]))
    assert got.dtype == torch.float64 and got.numel() == exp["n_unencrypted"]
    assert G.sha(np.ascontiguousarray(got.numpy())) == exp["unencrypted_avg_sha256"]


# ragged layouts for the gathered Port norms: int64 counters first, between and last; entries shorter than a
# 256-position gather iteration, entries straddling 2,048- / 4,096-position tiles, n % 8 tails of 0-7
PORT_SPECS = {
    "i64_first_tail5": [("n0", (), "i64"), ("a", (3,), "f32"), ("b", (5000,), "f32"), ("n1", (2,), "i64"),
                        ("c", (7, 9), "f32"), ("d", (4099,), "f32"), ("n2", (), "i64")],
    "tail0_big": [("w", (3, 4097), "f32"), ("n0", (), "i64"), ("b", (255,), "f32"), ("c", (2, 2049), "f32"),
                  ("n1", (), "i64"), ("e", (11,), "f32")],
    "tiny": [("a", (5,), "f32")],
    "i64_only_tail": [("a", (2048,), "f32"), ("n0", (3,), "i64")],
    # more entries than plato_agg_port_norms' 2,048-entry segment map: the engine takes the flatten path
    "many_entries": [(f"e{i}", (1 + i % 37,), "f32") if i % 11 else (f"n{i}", (), "i64") for i in range(2600)],
}


@pytest.mark.parametrize("spec", list(PORT_SPECS), ids=list(PORT_SPECS))
def test_port_norms_gathered_match_oracle(engine, spec):
    """plato_agg_port_norms (norms straight from the arenas) == the flatten + entry_norms path == the
    oracle's torch-order norm of torch.cat(...), bit for bit, including int64 counters (cast-first for
    current - previous, cast-once for the deltas) and every n % 8 tail."""
    from oracle import reductions as R

    layout = ArenaLayout.from_shapes(PORT_SPECS[spec])
    rng = np.random.default_rng(len(spec))
    k = 5
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(-2**40, 2**40, layout.n_i64)
    pf = (bf + rng.standard_normal(layout.n_f32).astype(np.float32) * 0.1).astype(np.float32)
    pi = bi + rng.integers(-2**35, 2**35, layout.n_i64)
    baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    previous = layout.unpack(torch.from_numpy(pf), torch.from_numpy(pi))
    clients = []
    for _ in range(k):
        xf = (bf + rng.standard_normal(layout.n_f32).astype(np.float32) * 0.01).astype(np.float32)
        xi = bi + rng.integers(-2**62, 2**62, layout.n_i64)  # wrapping int64 differences
        clients.append((xf, xi))
    rnd = engine.begin(baseline, k)
    rnd.put_baseline(baseline)
    for c, (xf, xi) in enumerate(clients):
        rnd.put_client(c, layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi)))
    sims = rnd.model_similarities(previous, range(k), threads=4)
    got = rnd.last_norms.copy()
    sims_flat = rnd.model_similarities(previous, range(k), threads=4, flat_norms=True)
    assert got.tobytes() == rnd.last_norms.tobytes()
    sims_staged = rnd.model_similarities(rnd.stage_reference(previous), range(k), threads=4)
    assert np.asarray(sims, np.float32).tobytes() == np.asarray(sims_staged, np.float32).tobytes()
    assert np.asarray(sims, np.float32).tobytes() == np.asarray(sims_flat, np.float32).tobytes()
    from plato_amd import _lib
    try:  # every tile / producer shape of the tuning library, bit for bit
        for variant in range(_lib.tune().plato_agg_tune_num_port_norms_variants()):
            engine.port_variant = variant
            sims_v = rnd.model_similarities(previous, range(k), threads=4)
            assert rnd.last_norms.tobytes() == got.tobytes(), variant
            assert np.asarray(sims_v, np.float32).tobytes() == np.asarray(sims, np.float32).tobytes(), variant
    finally:
        engine.port_variant = None
    v = R.port_current_minus_previous(layout.entries, bf, bi, pf, pi)
    want = [R.torch_norm(v)] + [R.torch_norm(R.port_delta(layout.entries, bf, bi, xf, xi)) for xf, xi in clients]
    assert got.tobytes() == np.asarray(want, np.float32).tobytes()

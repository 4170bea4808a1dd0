"""Multi-GPU engine in one server process (plato_amd.multi) against the reference fixtures.

``MultiDeviceEngine`` bucket-shards the arena over a device list; the result
must be bit-identical to the reference for any bucket count.  On a one-GPU
box the device list repeats cuda:0 (every bucket still gets its own arenas,
streams and copies, so the sharding, the per-bucket H2D/D2H assembly and the
pointer tables are all exercised); the RCCL communicator needs distinct GPUs
and runs when the box has them.
"""

import asyncio
import pickle
import types

import numpy as np
import pytest
import torch

from plato_amd import weights as W
from tests import golden_cases as G
from tests.test_golden_gpu import CASES, _bf16_payloads, _flat, _host_payloads, _updates

pytestmark = pytest.mark.gpu


def _devices(n):
    count = torch.cuda.device_count()
    return [f"cuda:{g % count}" for g in range(n)] if count >= 2 else ["cuda:0"] * n


def _case(name):
    return next(c for c in CASES if c["recipe"]["name"] == name)


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["resnet18_k16_permuted", "resnet18_k5_int64_edges", "lenet5_k7_edge_values",
                                  "C3_resnet50_200cls_k8", "resnet18_k1"])
def test_multi_device_hook_matches_reference(name, n):
    """FusedAggregationMixin with aggregation_devices: the reference digest for every bucket count."""
    from plato_amd.servers import FusedAggregationMixin

    case = _case(name)
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    updates = _updates(recipe, payloads)

    class Server(FusedAggregationMixin):
        aggregation_devices = _devices(n)

    server = Server()
    updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
    assert server.aggregation_engine().world == n
    assert list(updated.keys()) == [e.name for e in layout.entries]
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    assert server.total_samples == sum(recipe["num_samples"])
    items = server.get_logged_items()
    assert items["aggregation_gpus"] == n and items["aggregation_kernel_ms"] > 0
    assert items["aggregation_GBps"] > 0 and items["aggregation_total_ms"] >= items["aggregation_kernel_ms"]


@pytest.mark.parametrize("n", [2, 5])
def test_multi_device_deltas_and_variants(n):
    """aggregate_deltas (deltas mode), FedBuff and Pisces (second scalar) through the multi engine."""
    from plato_amd.servers import DeltasAggregationMixin
    from plato_amd.servers import variants as V

    for name, mixin in (("lenet5_k7_edge_values", DeltasAggregationMixin),
                        ("fedbuff_resnet18_k16", V.FedBuffServerMixin),
                        ("pisces_resnet18_k8", V.PiscesServerMixin)):
        case = _case(name)
        recipe, exp = case["recipe"], case["expected"]
        layout, baseline, payloads = _host_payloads(recipe)
        updates = _updates(recipe, payloads)

        class Server(mixin):
            aggregation_devices = _devices(n)
            staleness_factor = 0.5

            def __init__(self):
                self.client_staleness = {}
                self.current_round = 0

        server = Server()
        received = [u.payload for u in updates]
        if hasattr(server, "aggregate_weights"):
            updated = asyncio.run(server.aggregate_weights(updates, baseline, received))
        else:
            deltas = [{k: p[k] - baseline[k] for k in p} for p in received]
            avg = asyncio.run(server.aggregate_deltas(updates, deltas))
            assert G.sha(G.canon(_flat(layout, avg, "f32"))) == exp["avg_f32_sha256"], name
            updated = {k: baseline[k] + avg[k] for k in baseline}
        assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"], name
        assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"], name


@pytest.mark.parametrize("split", [False, True])
def test_multi_device_routes_staged_round_variants(split):
    """Port / FedAdp rounds run on GPU 0 by default; with client_split_rounds native payloads split their
    reductions by client, coded ones stay on GPU 0."""
    from plato_amd.servers import variants as V

    case = _case("port_resnet18_k16")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    updates = _updates(recipe, payloads)

    class Server(V.PortServerMixin):
        aggregation_devices = _devices(4)
        staleness_weight = 3
        client_split_rounds = split

        def __init__(self):
            self.current_round = 0

    server = Server()
    updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
    eng = server.aggregation_engine()
    assert server.round_engine("native") is (eng.clients if split else eng.primary)
    assert server.round_engine("qsgd") is eng.primary
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert server.get_logged_items()["aggregation_gpus"] == (4 if split else 1)


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["fedadp_lenet5_k6", "fedadp_resnet18_k8"])
def test_client_split_fedadp_matches_reference(name, n):
    """FedAdp over aggregation_devices: bucket-sharded staging and global gradient, dots split by client
    (client j's whole arena on device j mod n), final FedAvg bucket-sharded: the reference's weights,
    smoothed angles and model bit for bit, and every device used."""
    from plato_amd.servers.variants import FedAdpServerMixin
    from tests.test_per_entry_gpu import CASES as PE_CASES
    from tests.test_per_entry_gpu import _host

    recipe, exp = PE_CASES[name]["recipe"], PE_CASES[name]["expected"]
    layout, base, pays, _, updates = _host(recipe)

    class Server(FedAdpServerMixin):
        aggregation_devices = _devices(n)
        client_split_rounds = True
        fedadp_lr = 0.01

    server = Server()
    server.current_round = recipe["current_round"]
    server.selected_clients = [c + 1 for c in G.order_of(recipe)]
    server.local_angles = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    assert server.round_engine("native") is server.aggregation_engine().clients
    assert [float(x).hex() for x in server.adaptive_weighting] == exp["adaptive_weighting"]
    assert {str(c): "%08x" % np.float32(a).view(np.uint32) for c, a in server.local_angles.items()} == \
        exp["local_angles"]
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    items = server.get_logged_items()
    assert items["aggregation_gpus"] == n
    # one single-GPU engine per device holds its clients' arenas
    assert len(server.aggregation_engine()._client_engines) == n


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["port_similarity_lenet5_k8", "port_similarity_resnet18_k4"])
def test_client_split_port_matches_reference(tmp_path, name, n):
    """Port over aggregation_devices: similarities split by client, the reference's model bit for bit."""
    from plato_amd.servers.variants import PortServerMixin
    from tests.test_golden_gpu import FIXTURE_TORCH_THREADS, _previous

    case = _case(name)
    recipe = case["recipe"]
    layout, baseline, payloads = _host_payloads(recipe)
    path = tmp_path / f"model_{recipe['current_round'] - 2}.pth"
    torch.save(_previous(recipe, layout), path)

    class Server(PortServerMixin):
        aggregation_devices = _devices(n)
        client_split_rounds = True
        staleness_weight = 3
        current_round = recipe["current_round"]
        port_threads = FIXTURE_TORCH_THREADS

        def port_previous_model_path(self):
            return str(path)

    server = Server()
    updated = asyncio.run(server.aggregate_weights(_updates(recipe, payloads), baseline, payloads))
    assert server.round_engine("native") is server.aggregation_engine().clients
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == case["expected"]["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == case["expected"]["updated_i64f_sha256"]
    assert server.get_logged_items()["aggregation_gpus"] == n


@pytest.mark.parametrize("n", [2, 3])
def test_client_split_round_dots_equal_one_gpu(n):
    """The client-split round's FedAdp dots and Port similarities equal the one-GPU round's, bit for bit,
    on any client subset and order (ClientRound against AggregationRound on the same payloads)."""
    from plato_amd.engine import FedAvgEngine
    from plato_amd.multi import MultiDeviceEngine
    from tests.test_golden_gpu import _previous

    case = _case("port_similarity_resnet18_k4")
    recipe = case["recipe"]
    layout, baseline, payloads = _host_payloads(recipe)
    previous = _previous(recipe, layout)
    k = recipe["k"]
    one = FedAvgEngine("cuda:0").begin(baseline, k)
    one.put_baseline(baseline)
    multi = MultiDeviceEngine(_devices(n)).clients.begin(baseline, k)
    multi.put_baseline(baseline)
    for c in range(k):
        one.put_client(c, payloads[c])
        multi.put_client(c, payloads[c])
    w1 = np.tile(np.full(k, 1.0 / k), (len(layout.entries), 1))
    g1 = one.launch_entrywise(w1, add_base=False, device=True)
    gm = multi.launch_entrywise(w1, add_base=False, device=True)
    for gf, gi in gm:
        assert torch.equal(gf[: layout.n_f32].cpu(), g1[0][: layout.n_f32].cpu())
        assert torch.equal(gi[: layout.n_i64].cpu(), g1[1][: layout.n_i64].cpu())
    for slots in (list(range(k)), [k - 1, 0], [2]):
        a = one.fedadp_dots(g1, slots, 0.05)
        b = multi.fedadp_dots(gm, slots, 0.05)
        assert np.asarray(a[0]).tobytes() == np.asarray(b[0]).tobytes()
        assert np.float32(a[1]).tobytes() == np.float32(b[1]).tobytes()
        assert np.asarray(a[2]).tobytes() == np.asarray(b[2]).tobytes()
        sa = one.model_similarities(previous, slots, threads=4)
        sb = multi.model_similarities(previous, slots, threads=4)
        assert np.asarray(sa, np.float32).tobytes() == np.asarray(sb, np.float32).tobytes()
        assert one.last_norms.tobytes() == multi.last_norms.tobytes()


@pytest.mark.parametrize("name", ["bf16_codec_resnet18_k16", "bf16_codec_lenet5_k9"])
def test_multi_device_bf16_payloads(name):
    from plato_amd.multi import MultiDeviceEngine

    case = _case(name)
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _bf16_payloads(recipe)
    weights, _ = G.weights_for(recipe, W)
    eng = MultiDeviceEngine(_devices(3))
    updated = eng.aggregate_weights(baseline, [payloads[c] for c in G.order_of(recipe)], weights)
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]


def test_multi_device_wire_payloads_staged_on_arrival():
    """Native-ingested payloads prestaged bucket by bucket as they arrive, adopted in updates order."""
    from plato_amd import ingest
    from plato_amd.servers import FusedAggregationMixin, WireIngestMixin

    case = _case("resnet18_k16_permuted")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)

    class Algo:
        def extract_weights(self):
            return baseline

    class Server(WireIngestMixin, FusedAggregationMixin):
        aggregation_devices = _devices(4)
        stage_on_arrival = True

        def __init__(self):
            self.algorithm = Algo()
            self.client_chunks, self.client_payload, self.training_clients = {}, {}, {}

    server = Server()
    arrived = {}
    for c in reversed(range(recipe["k"])):
        sid = f"s{c}"
        server.client_chunks[sid] = [pickle.dumps(type(payloads[c])((n, t.clone()) for n, t in payloads[c].items()))]
        server.client_payload[sid] = None
        server.training_clients[c + 1] = True
        asyncio.run(server._client_payload_arrived(sid, c + 1))
        arrived[c] = server.client_payload[sid]
        assert isinstance(arrived[c], ingest.ArenaStateDict)
    eng = server.aggregation_engine()
    assert len(eng._arrivals) == recipe["k"]
    updates = _updates(recipe, [arrived[c] for c in range(recipe["k"])])
    updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    assert len(eng._arrivals) == 0


def test_multi_device_gather_leaves_the_model_on_every_gpu():
    from plato_amd.multi import MultiDeviceEngine

    case = _case("C3_resnet50_200cls_k8")
    recipe, exp = case["recipe"], case["expected"]
    layout, baseline, payloads = _host_payloads(recipe)
    weights, _ = G.weights_for(recipe, W)
    eng = MultiDeviceEngine(_devices(4))
    rnd = eng.begin(baseline, recipe["k"])
    rnd.put_baseline(baseline)
    for slot, c in enumerate(G.order_of(recipe)):
        rnd.put_client(slot, payloads[c])
    rnd.launch(weights, gather=True)
    host = rnd.result()
    flat = _flat(layout, host, "f32")
    assert G.sha(G.canon(flat)) == exp["updated_f32_sha256"]
    for g in range(eng.world):
        dev_f, dev_i = rnd.device_result(g)
        assert dev_f.device == eng.devices[g]
        assert np.array_equal(dev_f.cpu().numpy().view(np.uint32), flat.view(np.uint32))
        assert np.array_equal(dev_i.cpu().numpy().view(np.uint32), _flat(layout, host, "i64").view(np.uint32))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL communicator needs two or more GPUs")
def test_rccl_allgather_and_reduce_scatter_in_process():
    import ctypes

    from plato_amd import _lib
    from plato_amd.multi import MultiDeviceEngine

    n = torch.cuda.device_count()
    eng = MultiDeviceEngine([f"cuda:{g}" for g in range(n)])
    comm = eng.comm()
    assert comm is not None and _lib.lib().plato_agg_comm_size(comm) == n
    count = 1000
    send = [torch.full((count,), float(g + 1), device=f"cuda:{g}") for g in range(n)]
    recv = [torch.empty(count * n, device=f"cuda:{g}") for g in range(n)]
    streams = [torch.cuda.current_stream(g).cuda_stream for g in range(n)]
    arr = lambda xs: ctypes.cast((ctypes.c_void_p * n)(*xs), ctypes.c_void_p)  # noqa: E731
    _lib.call("plato_agg_comm_allgather_f32", comm, arr([t.data_ptr() for t in send]),
              arr([t.data_ptr() for t in recv]), count, arr(streams))
    for g in range(n):
        torch.cuda.synchronize(g)
        assert torch.equal(recv[g].cpu(), torch.arange(1, n + 1).float().repeat_interleave(count))
    part = [torch.full((count * n,), 1.0, device=f"cuda:{g}") for g in range(n)]
    out = [torch.empty(count, device=f"cuda:{g}") for g in range(n)]
    _lib.call("plato_agg_comm_reduce_scatter_f32", comm, arr([t.data_ptr() for t in part]),
              arr([t.data_ptr() for t in out]), count, arr(streams))
    for g in range(n):
        torch.cuda.synchronize(g)
        assert torch.all(out[g].cpu() == float(n))
    eng.close()


def test_rccl_refuses_repeated_devices():
    import ctypes

    from plato_amd import _lib

    arr = (ctypes.c_int * 2)(0, 0)
    handle = ctypes.c_void_p()
    with pytest.raises(ValueError, match="distinct"):
        _lib.call("plato_agg_comm_create", 2, ctypes.cast(arr, ctypes.c_void_p), ctypes.byref(handle))


def test_result_buffers_are_not_recycled_under_a_kept_result():
    """Pinned result buffers are pooled, but never reused while an earlier result is referenced."""
    from plato_amd.engine import FedAvgEngine

    case = _case("resnet18_k16")
    recipe = case["recipe"]
    layout, baseline, payloads = _host_payloads(recipe)
    eng = FedAvgEngine("cuda:0")
    weights, _ = G.weights_for(recipe, W)
    first = eng.aggregate_weights(baseline, payloads, weights)
    snapshot = {k: v.clone() for k, v in first.items()}
    for _ in range(3):
        eng.aggregate_weights(baseline, payloads[::-1], weights)
    for k in first:
        assert torch.equal(first[k], snapshot[k]), k
    ptrs = {eng.aggregate_weights(baseline, payloads, weights)[layout.entries[0].name].data_ptr() for _ in range(3)}
    assert len(ptrs) <= 2  # dropped results give their buffer back to the pool


# ------------------------------------------------------------ entry-aligned shards
# FedAtt, Polaris and QSGD payloads reduce entry by entry (fedatt_algorithm.py:23-69,
# polaris_server.py:68-100, model_dequantize_qsgd.py:34-60): over several devices their rounds
# are sharded by whole entries (MultiDeviceEngine.entries), each shard a single-GPU round over
# its entries.  Same reference digests at every shard count, including more shards than some
# models have large entries.
def _entry_host(name):
    from tests.test_per_entry_gpu import CASES as PE, _host

    return PE[name], _host(PE[name]["recipe"])


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["fedatt_resnet18_k8", "fedatt_lenet5_k6", "fedatt_qsgd_resnet18_k3"])
def test_entry_sharded_fedatt_matches_reference(name, n):
    from plato_amd.algorithms.fedavg import FedAttAlgorithmMixin
    from tests.test_per_entry_gpu import _coded, _hex_matrix

    case, (layout, base, pays, _, _) = _entry_host(name)
    recipe, exp = case["recipe"], case["expected"]
    if recipe.get("codec"):
        layout, base, pays, _ = _coded(recipe)

    class Algorithm(FedAttAlgorithmMixin):
        aggregation_devices = _devices(n)

    alg = Algorithm()
    eng = alg.entry_engine()
    assert eng.world == n
    rnd = eng.begin(base, recipe["k"], recipe.get("codec", "native"))
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    norms = rnd.decoded().entry_norms(range(recipe["k"]))
    assert norms.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_norms"]).view(np.uint32).tolist()
    torch.manual_seed(recipe["noise_seed"])
    updated = asyncio.run(alg.aggregate_weights(base, pays))
    assert list(updated) == layout.keys()
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("name", ["polaris_resnet18_k8", "polaris_bf16_resnet18_k4"])
def test_entry_sharded_polaris_matches_reference(name, n):
    from plato_amd.servers.variants import PolarisServerMixin
    from tests.test_per_entry_gpu import _coded

    case, (layout, base, pays, _, updates) = _entry_host(name)
    recipe, exp = case["recipe"], case["expected"]
    if recipe.get("codec"):
        layout, base, pays, updates = _coded(recipe)

    class Server(PolarisServerMixin):
        aggregation_devices = _devices(n)

    server = Server()
    server.number_of_client = 1024
    server.unexplored_clients = list(range(1024))
    server.alpha = 10
    assert server.round_engine(recipe.get("codec", "native")) is server.aggregation_engine().entries
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    want = {int(c): float.fromhex(v) for c, v in exp["squared_deltas"].items()}
    got = {i: float(v) for i, v in enumerate(server.squared_deltas_current_round) if v != 0}
    assert {c: v.hex() for c, v in got.items()} == {c: v.hex() for c, v in want.items()}
    assert server.get_logged_items()["aggregation_gpus"] == n


@pytest.mark.parametrize("n", [2, 3, 8])
def test_entry_sharded_qsgd_payloads_match_reference(n):
    from oracle import qsgd as Q
    from oracle import synth
    from plato_amd.arena import ArenaLayout
    from plato_amd.processors.qsgd import Processor
    from plato_amd.servers import FusedAggregationMixin

    cases = [c for c in G.load_cases() if c["recipe"].get("codec") == "qsgd" and c["recipe"]["name"].startswith("qsgd")]
    assert cases
    for case in cases:
        recipe, exp = case["recipe"], case["expected"]
        layout = ArenaLayout.from_shapes(G.model_spec(recipe["model"]))
        k, seed = recipe["k"], recipe["seed"]
        bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
        baseline = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
        proc = Processor()
        payloads = {c: proc.process(Q.client_wire(layout.entries, seed, c)[0]) for c in range(k)}
        updates = [types.SimpleNamespace(client_id=c + 1, report=types.SimpleNamespace(num_samples=recipe["num_samples"][c]),
                                         payload=payloads[c], staleness=0) for c in G.order_of(recipe)]

        class Server(FusedAggregationMixin):
            aggregation_devices = _devices(n)

        server = Server()
        assert server.round_engine("qsgd") is server.aggregation_engine().entries
        # half of the payloads arrive early and are prestaged shard by shard, the rest staged at aggregation
        eng = server.round_engine("qsgd")
        for u in updates[::2]:
            assert eng.prestage(u.payload, layout)
        updated = asyncio.run(server.aggregate_weights(updates, baseline, [u.payload for u in updates]))
        assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"], recipe["name"]
        assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"], recipe["name"]
        assert eng._arrivals == {}


def test_entry_sharded_round_rejects_whole_model_reductions():
    """Device-resident entrywise results (FedAdp's global gradient) stay on one GPU."""
    from tests.test_per_entry_gpu import CASES as PE, _host
    from plato_amd.multi import MultiDeviceEngine

    recipe = PE["fedadp_lenet5_k6"]["recipe"]
    layout, base, pays, _, _ = _host(recipe)
    eng = MultiDeviceEngine(_devices(2)).entries
    rnd = eng.begin(base, recipe["k"])
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    with pytest.raises(ValueError, match="one GPU"):
        rnd.launch_entrywise(np.ones((len(layout.entries), recipe["k"])), add_base=False, device=True)
    assert not hasattr(rnd, "fedadp_dots") and not hasattr(rnd, "model_similarities")


def test_entry_sharded_prestage_failure_keeps_no_slot():
    """A payload whose prestage fails on one shard leaves no arrival slot on the shards before it."""
    from tests.test_per_entry_gpu import CASES as PE, _host
    from plato_amd.arena import ArenaLayout
    from plato_amd.multi import MultiDeviceEngine

    recipe = PE["fedadp_lenet5_k6"]["recipe"]
    layout, base, pays, _, _ = _host(recipe)
    eng = MultiDeviceEngine(_devices(2)).entries
    lay = ArenaLayout.from_state_dict(base)
    assert eng.prestage(pays[0], lay)
    assert len(eng._engines[0]._arrivals) == 1 and len(eng._engines[1]._arrivals) == 1
    eng._engines[1].prestage = lambda payload, layout, baseline=None: False
    assert not eng.prestage(pays[1], lay)
    assert len(eng._engines[0]._arrivals) == 1  # only the first payload's slot
    assert id(pays[1]) not in eng._arrivals
    eng._release()
    assert eng._engines[0]._arrivals == {}

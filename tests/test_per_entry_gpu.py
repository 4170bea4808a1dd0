"""GPU parity of the per-entry kernels and the FedAtt / FedAdp / Polaris hooks.

* plato_agg_fedavg_entrywise vs oracle.entrywise_numpy: bit-exact, on a layout
  of awkward entry sizes and with chunk capacities small enough that entries
  span many chunks and chunks start/end inside float4 groups;
* plato_agg_entry_stats vs oracle.entry_stats_fp64: 1e-12 relative (both fp64,
  different summation order);
* plato_agg_entry_norms_f32 vs oracle.torch_cpu_norm_f32: bit-exact;
* the product hooks vs the reference fixtures: FedAtt bit-exact end to end,
  FedAdp bit-exact end to end (adaptive weights, smoothed angles, model: its
  float32 BLAS reductions run in numpy's OpenBLAS order, plato_agg_sdot_pairs),
  Polaris' model and norms bit-exact (numpy's pairwise sums, plato_agg_np_sumsq).
"""

import asyncio
import types
from collections import OrderedDict

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from plato_amd.arena import ArenaLayout
from plato_amd.engine import ClientSlab, FedAvgEngine
from tests import golden_cases as G

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
CASES = {c["recipe"]["name"]: c for c in G.load_cases()}

SPEC = [("a", (3,), "f32"), ("n0", (), "i64"), ("b", (1,), "f32"), ("c", (5, 7), "f32"), ("d", (64,), "f32"),
        ("n1", (4,), "i64"), ("e", (1000,), "f32"), ("f", (0,), "f32"), ("g", (4099,), "f32"), ("h", (2,), "f32"),
        ("n2", (), "i64"), ("big", (3, 4097), "f32")]


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine(DEV)


def _random_round(engine, k, seed):
    layout = ArenaLayout.from_shapes(SPEC)
    rng = np.random.default_rng(seed)
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(-1000, 1000, layout.n_i64)
    xs_f = [(bf + 0.01 * rng.standard_normal(layout.n_f32)).astype(np.float32) for _ in range(k)]
    xs_i = [bi + rng.integers(0, 9, layout.n_i64) for _ in range(k)]
    base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    pays = [layout.unpack(torch.from_numpy(xs_f[i]), torch.from_numpy(xs_i[i])) for i in range(k)]
    rnd = engine.begin(base, k)
    rnd.put_baseline(base)
    for i in range(k):
        rnd.put_client(i, pays[i])
    return layout, rnd, bf, bi, xs_f, xs_i, rng


@pytest.mark.parametrize("cap", [8, 20, 1024, 2048])
@pytest.mark.parametrize("noise,add_base", [(False, True), (True, True), (False, False)])
def test_entrywise_matches_oracle(engine, monkeypatch, cap, noise, add_base):
    monkeypatch.setattr(FedAvgEngine, "ENTRYWISE_CHUNK", cap)
    k = 5
    layout, rnd, bf, bi, xs_f, xs_i, rng = _random_round(engine, k, 10 + cap)
    w = rng.standard_normal((len(layout.entries), k))
    nz = nf = ni = None
    if noise:
        nf = rng.standard_normal(layout.n_f32).astype(np.float32)
        ni = rng.standard_normal(layout.n_i64).astype(np.float32)
        nz = layout.unpack(torch.from_numpy(nf), torch.from_numpy(ni))
    order = [3, 0, 4, 1, 2]
    rnd.launch_entrywise(w, order=order, scale=-1.2, noise=nz, noise_scale=0.001, add_base=add_base)
    got = rnd.result()
    exp_f, exp_i = ref.entrywise_numpy(layout.entries, bf, bi, [xs_f[i] for i in order], [xs_i[i] for i in order],
                                       w, -1.2, nf, ni, 0.001, add_base)
    got_f = torch.cat([got[e.name].reshape(-1) for e in layout.entries if e.region == "f32"]).numpy()
    got_i = torch.cat([got[e.name].reshape(-1) for e in layout.entries if e.region == "i64"]).numpy()
    assert got_f.tobytes() == exp_f.tobytes()
    assert got_i.tobytes() == exp_i.tobytes()


@pytest.mark.parametrize("cap", [4, 36, 4096])
def test_entry_stats_match_oracle(engine, monkeypatch, cap):
    monkeypatch.setattr(FedAvgEngine, "STATS_CHUNK", cap)
    k = 6
    layout, rnd, bf, bi, xs_f, xs_i, rng = _random_round(engine, k, 20 + cap)
    vf = rng.standard_normal(layout.row_f32).astype(np.float32)
    vi = rng.standard_normal(layout.row_i64).astype(np.float32)
    v = (torch.from_numpy(vf).to(DEV), torch.from_numpy(vi).to(DEV))
    dv, dd, vv = rnd.entry_stats(range(k), v=v)
    e_dv, e_dd, e_vv = ref.entry_stats_fp64(layout.entries, bf, bi, xs_f, xs_i, vf, vi)
    np.testing.assert_allclose(dd, e_dd, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(dv, e_dv, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(vv, e_vv, rtol=1e-12, atol=1e-300)
    assert dd[:, [i for i, e in enumerate(layout.entries) if e.numel == 0]].sum() == 0
    # without v: the d.d rows only, and the same values
    none_dv, dd2, none_vv = rnd.entry_stats(range(k))
    assert none_dv is None and none_vv is None and dd2.tobytes() == dd.tobytes()


@pytest.mark.parametrize("long_threshold,k", [(None, 7), (1 << 17, 7), (8, 7), (1, 7), (None, 97)])
def test_entry_norms_follow_torch_cpu_order(engine, monkeypatch, long_threshold, k):
    """Every entry's norm in torch's CPU order, whichever kernel takes it: the long entries through
    plato_agg_port_norms on the side stream (threshold 8 / 1: nearly every fp32 entry, ragged lengths,
    n % 8 tails, unaligned arena offsets), the rest through plato_agg_entry_norms_f32 (K = 97: two clients
    per workgroup, a one-client last group; empty and int64 entries)."""
    monkeypatch.setattr(engine, "norms_long_threshold", long_threshold)
    layout, rnd, bf, bi, xs_f, xs_i, _ = _random_round(engine, k, 5)
    got = rnd.entry_norms(range(k))
    for e_i, e in enumerate(layout.entries):
        if e.region == "f32":
            rows = np.stack([np.subtract(x[e.offset:e.offset + e.numel], bf[e.offset:e.offset + e.numel],
                                         dtype=np.float32) for x in xs_f])
        else:
            rows = np.stack([(x[e.offset:e.offset + e.numel] - bi[e.offset:e.offset + e.numel]).astype(np.float32)
                             for x in xs_i])
        exp = ref.torch_cpu_norm_f32(rows) if e.numel else np.zeros(k, np.float32)
        assert got[e_i].tobytes() == exp.tobytes(), e.name
        if e.numel:  # and the torch op itself, on this host
            t = torch.from_numpy(rows)
            assert got[e_i].tolist() == [torch.linalg.norm(-t[i]).item() for i in range(k)], e.name


RING_SPEC = [("a", (5,), "f32"), ("w", (33333,), "f32"), ("n", (), "i64"), ("v", (7,), "f32"),
             ("u", (160, 128), "f32"), ("t", (9,), "f32"), ("m", (3,), "i64"), ("z", (12290,), "f32")]


@pytest.mark.parametrize("k,deltas", [(5, False), (8, False), (3, True)])
def test_entry_norm_kernels_agree_bitwise(engine, k, deltas):
    """Every entry_norms kernel (LDS-DMA and register-staged producer / consumer shapes, per-wave) ==
    torch CPU order, across ring wrap-around, unaligned entry starts and both arena tails."""
    from plato_amd import _lib

    for spec in (RING_SPEC, RING_SPEC[:-1] + [("z", (12291,), "f32")]):  # n_f32 % 4 == 0 / == 3
        layout = ArenaLayout.from_shapes(spec)
        rng = np.random.default_rng(k)
        dev = torch.device(DEV)
        bf = rng.standard_normal(layout.row_f32).astype(np.float32)
        bi = rng.integers(-1000, 1000, max(layout.row_i64, 1))
        xs_f = np.stack([bf + 0.01 * rng.standard_normal(layout.row_f32).astype(np.float32) for _ in range(k)])
        xs_i = np.stack([bi + rng.integers(0, 9, bi.size) for _ in range(k)])
        xf = torch.from_numpy(xs_f).to(dev)
        xi = torch.from_numpy(xs_i).to(dev)
        tf = torch.tensor([xf[i].data_ptr() for i in range(k)], dtype=torch.int64, device=dev)
        ti = torch.tensor([xi[i].data_ptr() for i in range(k)], dtype=torch.int64, device=dev)
        b_f = torch.from_numpy(bf).to(dev)
        b_i = torch.from_numpy(bi).to(dev)
        ef, ei = engine._norm_tables(layout)
        n_e = len(layout.entries)
        outs = []
        for variant in range(_lib.tune().plato_agg_tune_num_entry_norms_variants()):
            out = torch.full((k * n_e,), float("nan"), device=dev)
            _lib.tune_call("plato_agg_tune_entry_norms", variant, tf.data_ptr(), ti.data_ptr(), k,
                      None if deltas else b_f.data_ptr(), None if deltas else b_i.data_ptr(), ef.data_ptr(),
                      ef.shape[0], ei.data_ptr(), ei.shape[0], n_e, layout.n_f32, layout.n_i64, out.data_ptr(),
                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy().reshape(k, n_e))
        for v in range(1, len(outs)):
            assert outs[0].tobytes() == outs[v].tobytes(), v
        for e_i, e in enumerate(layout.entries):
            if e.region == "f32":
                rows = xs_f[:, e.offset:e.offset + e.numel]
                if not deltas:
                    rows = np.subtract(rows, bf[e.offset:e.offset + e.numel], dtype=np.float32)
            else:
                rows = xs_i[:, e.offset:e.offset + e.numel]
                rows = (rows if deltas else rows - bi[e.offset:e.offset + e.numel]).astype(np.float32)
            assert outs[0][:, e_i].tobytes() == ref.torch_cpu_norm_f32(np.ascontiguousarray(rows)).tobytes(), e.name


@pytest.mark.parametrize("k,deltas", [(96, False), (97, False), (129, True), (193, False), (255, True)])
def test_entry_norms_default_from_k96_matches_oracle(engine, k, deltas):
    """The product entry point at K >= 96 (two clients of one entry per workgroup sharing the baseline
    tiles, four from K = 192, in one chain wave; a ragged K leaves a partial last group) == torch CPU
    order, both arena tails."""
    from plato_amd import _lib

    for spec in (RING_SPEC, RING_SPEC[:-1] + [("z", (12291,), "f32")]):
        layout = ArenaLayout.from_shapes(spec)
        rng = np.random.default_rng(k)
        dev = torch.device(DEV)
        bf = rng.standard_normal(layout.row_f32).astype(np.float32)
        bi = rng.integers(-1000, 1000, max(layout.row_i64, 1))
        xs_f = (bf + 0.01 * rng.standard_normal((k, layout.row_f32))).astype(np.float32)
        xs_i = bi + rng.integers(0, 9, (k, bi.size))
        xf = torch.from_numpy(xs_f).to(dev)
        xi = torch.from_numpy(xs_i).to(dev)
        tf = torch.tensor([xf[i].data_ptr() for i in range(k)], dtype=torch.int64, device=dev)
        ti = torch.tensor([xi[i].data_ptr() for i in range(k)], dtype=torch.int64, device=dev)
        b_f = torch.from_numpy(bf).to(dev)
        b_i = torch.from_numpy(bi).to(dev)
        ef, ei = engine._norm_tables(layout)
        n_e = len(layout.entries)
        out = torch.full((k * n_e,), float("nan"), device=dev)
        _lib.call("plato_agg_entry_norms_f32", tf.data_ptr(), ti.data_ptr(), k, None if deltas else b_f.data_ptr(),
                  None if deltas else b_i.data_ptr(), ef.data_ptr(), ef.shape[0], ei.data_ptr(), ei.shape[0], n_e,
                  layout.n_f32, layout.n_i64, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        got = out.cpu().numpy().reshape(k, n_e)
        for e_i, e in enumerate(layout.entries):
            if e.region == "f32":
                rows = xs_f[:, e.offset:e.offset + e.numel]
                if not deltas:
                    rows = np.subtract(rows, bf[e.offset:e.offset + e.numel], dtype=np.float32)
            else:
                rows = xs_i[:, e.offset:e.offset + e.numel]
                rows = (rows if deltas else rows - bi[e.offset:e.offset + e.numel]).astype(np.float32)
            assert got[:, e_i].tobytes() == ref.torch_cpu_norm_f32(np.ascontiguousarray(rows)).tobytes(), e.name


# ------------------------------------------------------------------ hooks vs reference
def _host(recipe):
    layout, base, pays, arenas = G.host_state_dicts(recipe)
    st = recipe.get("staleness", [0] * recipe["k"])
    updates = [types.SimpleNamespace(client_id=c + 1, report=types.SimpleNamespace(num_samples=recipe["num_samples"][c]),
                                     payload=p, staleness=st[c]) for c, p in zip(G.order_of(recipe), pays)]
    return layout, base, pays, arenas, updates


def _flat(layout, sd, region):
    parts = [sd[e.name].reshape(-1).float() for e in layout.entries if e.region == region]
    return torch.cat(parts).numpy() if parts else np.zeros(0, np.float32)


def _hex_matrix(rows):
    return np.array([[G.hexf(h) for h in row] for row in rows], dtype=np.float32)


@pytest.mark.parametrize("name", ["fedatt_lenet5_k6", "fedatt_resnet18_k8"])
def test_fedatt_algorithm_is_bit_exact(engine, name):
    from plato_amd.algorithms.fedavg import FedAttAlgorithmMixin

    recipe, exp = CASES[name]["recipe"], CASES[name]["expected"]
    layout, base, pays, _, _ = _host(recipe)

    class Algorithm(FedAttAlgorithmMixin):
        aggregation_device = DEV

    alg = Algorithm()
    alg._plato_amd_engine = engine
    # the device norms equal the reference's fp32 values
    rnd = engine.begin(base, recipe["k"])
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    norms = rnd.entry_norms(range(recipe["k"]))
    assert norms.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_norms"]).view(np.uint32).tolist()
    torch.manual_seed(recipe["noise_seed"])
    updated = asyncio.run(alg.aggregate_weights(base, pays))
    assert list(updated) == layout.keys()
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == exp["updated_i64f_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]


@pytest.mark.parametrize("deltas", [True, False])
@pytest.mark.parametrize("align", [None, "fedadp"])
@pytest.mark.parametrize("name", ["fedadp_lenet5_k6", "fedadp_resnet18_k8"])
def test_fedadp_server_matches_reference(name, align, deltas):
    """The product path (FedAdpServerMixin: arenas aligned to the flattened positions, clients staged as
    their deltas) and the packed layout / weight arenas give the reference's weights, angles and model
    bit for bit."""
    from plato_amd.servers.variants import FedAdpServerMixin

    recipe, exp = CASES[name]["recipe"], CASES[name]["expected"]
    layout, base, pays, (bf, bi, xs_f, xs_i), updates = _host(recipe)

    class Server(FedAdpServerMixin):
        aggregation_device = DEV
        fedadp_lr = 0.01
        arena_alignment = align
        arena_deltas = deltas

    server = Server()
    engine = server.aggregation_engine()
    assert engine.layout_align == align
    assert engine.delta_arenas is deltas
    server.current_round = recipe["current_round"]
    server.selected_clients = [c + 1 for c in G.order_of(recipe)]
    server.local_angles = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    # the adaptive weights and smoothed angles: the reference's bits (numpy's float32 BLAS order on the device)
    assert [float(x).hex() for x in server.adaptive_weighting] == exp["adaptive_weighting"]
    assert {str(c): "%08x" % np.float32(a).view(np.uint32) for c, a in server.local_angles.items()} == \
        exp["local_angles"]
    # the model: the reference's digest
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    ref_w = [float.fromhex(h) for h in exp["adaptive_weighting"]]

    # global gradient (deltas pass, no baseline) bit-exact; model bit-exact given the reference's weights;
    # the materialised-flatten cross-check reads weight arenas
    engine.delta_arenas = False
    rnd = engine.begin(base, recipe["k"])
    assert rnd.layout.align == align
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    w1 = np.tile(np.asarray([u.report.num_samples for u in updates], dtype=np.float64)
                 / sum(u.report.num_samples for u in updates), (len(layout.entries), 1))
    g_f, g_i = rnd.launch_entrywise(w1, add_base=False, device=True)
    g_model = rnd.layout.unpack(g_f.cpu(), g_i.cpu())  # (the aligned arena has padding between entries)
    assert G.sha(G.canon(_flat(layout, g_model, "f32"))) == exp["global_grads_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, g_model, "i64"))) == exp["global_grads_i64f_sha256"]
    # the fused gather kernel against the materialised-flatten path, whole and in batches of 1 and 3
    # clients (g.g rides with the last batch), and on client subsets and orders
    whole = rnd.fedadp_dots((g_f, g_i), range(recipe["k"]), 0.01)
    stride_bytes = -(-(layout.n_f32 + layout.n_i64) // 64) * 64 * 4
    for per in (1e12, 1, 3):
        parts = rnd.fedadp_dots_flat((g_f, g_i), range(recipe["k"]), 0.01, batch_bytes=per * stride_bytes)
        assert np.asarray(parts[0]).tobytes() == np.asarray(whole[0]).tobytes()
        assert np.float32(parts[1]).tobytes() == np.float32(whole[1]).tobytes()
        assert np.asarray(parts[2]).tobytes() == np.asarray(whole[2]).tobytes()
    sub = [recipe["k"] - 1, 0, 2]
    part = rnd.fedadp_dots((g_f, g_i), sub, 0.01)
    assert np.asarray(part[0]).tobytes() == np.asarray(whole[0])[sub].tobytes()
    assert np.asarray(part[2]).tobytes() == np.asarray(whole[2])[sub].tobytes()
    rnd.launch(ref_w)
    again = rnd.result()
    assert G.sha(G.canon(_flat(layout, again, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, again, "i64"))) == exp["loaded_i64_sha256"]


@pytest.mark.parametrize("deltas", [True, False])
def test_fedadp_server_with_arrival_staging_matches_reference(deltas):
    """FedAdp through the wire path: payloads parsed natively and staged to HBM as they arrive (turned
    into deltas against the server's current model when arena_deltas), then the FedAdp round adopts them —
    the reference's adaptive weights and model bit for bit."""
    import pickle

    from plato_amd.servers import WireIngestMixin
    from plato_amd.servers.variants import FedAdpServerMixin

    name = "fedadp_resnet18_k8"
    recipe, exp = CASES[name]["recipe"], CASES[name]["expected"]
    layout, base, pays, _, updates = _host(recipe)

    class Algo:
        def extract_weights(self):
            return base

    class Server(WireIngestMixin, FedAdpServerMixin):
        aggregation_device = DEV
        fedadp_lr = 0.01
        stage_on_arrival = True
        arena_deltas = deltas

        def __init__(self):
            self.algorithm = Algo()
            self.client_chunks, self.client_payload, self.training_clients = {}, {}, {}

    server = Server()
    arrived = {}
    for c in reversed(range(recipe["k"])):  # arrival order differs from the update order
        sid = f"s{c}"
        server.client_chunks[sid] = [pickle.dumps(type(pays[c])((n, t.clone()) for n, t in pays[c].items()))]
        server.client_payload[sid] = None
        server.training_clients[c + 1] = True
        asyncio.run(server._client_payload_arrived(sid, c + 1))
        arrived[c] = server.client_payload[sid]
    eng = server.aggregation_engine()
    assert eng.delta_arenas is deltas
    assert len(eng._arrivals) == recipe["k"]
    assert all((hit[8] is not None) == deltas for hit in eng._arrivals.values())
    for c, u in enumerate(updates):
        u.payload = arrived[c]
    server.current_round = recipe["current_round"]
    server.selected_clients = [c + 1 for c in G.order_of(recipe)]
    server.local_angles = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    import unittest.mock as um

    from plato_amd.engine import AggregationRound

    adopted = []
    orig_adopt = AggregationRound.adopt

    def spy(rnd, slot, payload):
        ok = orig_adopt(rnd, slot, payload)
        adopted.append(ok)
        return ok

    with um.patch.object(AggregationRound, "adopt", spy):
        updated = asyncio.run(server.aggregate_weights(updates, base, [u.payload for u in updates]))
    assert adopted and all(adopted)  # every payload came from its arrival row
    assert [float(x).hex() for x in server.adaptive_weighting] == exp["adaptive_weighting"]
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    assert len(eng._arrivals) == 0  # released after the round


@pytest.mark.parametrize("name", ["fedadp_lenet5_k6", "fedadp_resnet18_k8"])
def test_delta_round_matches_weight_round(name):
    """A round whose clients are staged as deltas (FedAvgEngine.delta_arenas: put_client and adopt turn each
    slot into x - b in place) gives the weight round's global gradient, FedAdp dots and FedAvg result bit
    for bit, refuses the reductions that need the clients' weights, and needs the baseline first."""
    recipe = CASES[name]["recipe"]
    layout, base, pays, _, updates = _host(recipe)
    k = recipe["k"]
    w1 = np.tile(np.asarray([u.report.num_samples for u in updates], dtype=np.float64)
                 / sum(u.report.num_samples for u in updates), (len(layout.entries), 1))
    weights = [float(u.report.num_samples) / sum(x.report.num_samples for x in updates) for u in updates]
    got = {}
    for deltas in (False, True):
        eng = FedAvgEngine(DEV)
        eng.layout_align = "fedadp"
        eng.delta_arenas = deltas
        rnd = eng.begin(base, k)
        assert rnd.deltas is deltas
        if deltas:
            with pytest.raises(ValueError, match="baseline"):
                rnd.put_client(0, pays[0])
        rnd.put_baseline(base)
        for i, p in enumerate(pays):
            if i == 1 and deltas:  # one slot through the arrival path: prestaged weights, converted at adopt
                assert eng.prestage(p, rnd.layout) and rnd.adopt(i, p)
            elif i == 2 and deltas:  # and one turned into its delta at arrival against the same model
                assert eng.prestage(p, rnd.layout, baseline=base)
                assert eng._arrivals[id(p)][8] is not None and rnd.adopt(i, p)
            else:
                rnd.put_client(i, p)
        g_f, g_i = rnd.launch_entrywise(w1, add_base=False, device=True)
        dots = rnd.fedadp_dots((g_f, g_i), range(k), 0.01)
        # the fallback past the dot kernel's limits: on delta arenas it flattens the deltas
        dots_flat = rnd.fedadp_dots_flat((g_f, g_i), range(k), 0.01)
        rnd.launch(weights)
        res = rnd.result()
        g_model = rnd.layout.unpack(g_f.cpu(), g_i.cpu())  # (the aligned arena has padding between entries)
        sumsq = rnd.np_sumsq(range(k))  # Polaris' sums: on delta arenas with a null baseline
        # Port's similarities against another model: gathered (null subtrahends) and flat-norms paths
        other = OrderedDict((n_, (t_ * 0.5 if t_.is_floating_point() else t_)) for n_, t_ in base.items())
        sims = [np.asarray(rnd.model_similarities(other, range(k), threads=4, flat_norms=f)).tobytes()
                for f in (False, True)]
        got[deltas] = (sims, sumsq.tobytes(), _flat(layout, g_model, "f32").tobytes(),
                       _flat(layout, g_model, "i64").tobytes(),
                       [np.asarray(d).tobytes() for d in dots], [np.asarray(d).tobytes() for d in dots_flat],
                       _flat(layout, res, "f32").tobytes(),
                       _flat(layout, res, "i64").tobytes())
        if deltas:
            for call in (lambda: rnd.entry_norms(range(k)),
                         lambda: rnd.launch_entrywise(w1, add_base=True)):
                with pytest.raises(ValueError, match="deltas"):
                    call()
            with pytest.raises(ValueError, match="deltas"):
                rnd.put_baseline(base)
        eng.release_arrivals()
    assert got[True] == got[False]


def test_polaris_server_matches_reference(engine):
    from plato_amd.servers.variants import PolarisServerMixin

    recipe, exp = CASES["polaris_resnet18_k8"]["recipe"], CASES["polaris_resnet18_k8"]["expected"]
    layout, base, pays, _, updates = _host(recipe)

    class Server(PolarisServerMixin):
        aggregation_device = DEV

    server = Server()
    server._plato_amd_engine = engine
    server.number_of_client = 1024
    server.unexplored_clients = list(range(1024))
    server.alpha = 10
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    assert server.total_samples == exp["total_samples"]
    want = {int(c): float.fromhex(v) for c, v in exp["squared_deltas"].items()}
    got = {i: float(v) for i, v in enumerate(server.squared_deltas_current_round) if v != 0}
    assert set(got) == set(want)
    # numpy's float32 pairwise sums on the device: the reference's bits, expected fill included
    assert {c: v.hex() for c, v in got.items()} == {c: v.hex() for c, v in want.items()}
    assert sorted(set(range(1024)) - set(server.unexplored_clients)) == sorted(c for c in G.order_of(recipe))


@pytest.mark.parametrize("deltas", [False, True])
def test_fedadp_layout_tables_reused_across_rounds(deltas):
    """The second round of one layout and K reuses the workspace's layout-only tables
    (plato_agg_fedadp_dots_ex, PLATO_AGG_FEDADP_TABLES_READY) and gives the first round's dots bit for bit;
    another K builds them again; both equal the flatten + sdot path."""
    from plato_amd import _lib

    recipe = CASES["fedadp_resnet18_k8"]["recipe"]
    _, base, pays, _, _ = _host(recipe)
    k = recipe["k"]
    engine = FedAvgEngine(DEV)
    engine.layout_align = "fedadp"
    engine.delta_arenas = deltas
    seen = []
    real = _lib.call

    def spy(name, *args):
        if name == "plato_agg_fedadp_dots_ex":
            seen.append(args[-1])
        return real(name, *args)

    got = []
    for kk in (k, k, k - 3, k - 3):
        rnd = engine.begin(base, kk)
        rnd.put_baseline(base)
        for i in range(kk):
            rnd.put_client(i, pays[i])
        w1 = np.tile(np.full(kk, 1.0 / kk), (len(rnd.layout.entries), 1))
        grads = rnd.launch_entrywise(w1, add_base=False, device=True)
        _lib.call = spy
        try:
            dots = rnd.fedadp_dots(grads, range(kk), 0.01)
        finally:
            _lib.call = real
        want = rnd.fedadp_dots_flat(grads, range(kk), 0.01)
        assert [np.asarray(d).tobytes() for d in dots] == [np.asarray(d).tobytes() for d in want]
        got.append([np.asarray(d).tobytes() for d in dots])
        engine.release_arrivals()
    assert seen == [0, _lib.PLATO_AGG_FEDADP_TABLES_READY, 0, _lib.PLATO_AGG_FEDADP_TABLES_READY]
    assert got[0] == got[1] and got[2] == got[3]


@pytest.mark.parametrize("odd", [False, True])
@pytest.mark.parametrize("align", [None, "fedadp"])
@pytest.mark.parametrize("name", ["fedadp_lenet5_k6", "fedadp_resnet18_k8"])
def test_fedadp_dots_tile_shapes_agree_bitwise(name, align, odd):
    """Every tile shape of the fused gather + sdot kernel (tuning library) equals the flatten + sdot path,
    on packed and on FedAdp-aligned arenas; ``odd``: one client fewer (the two-client kernel's last
    workgroup then holds one client)."""
    from plato_amd import _lib

    recipe = CASES[name]["recipe"]
    layout, base, pays, _, updates = _host(recipe)
    k = recipe["k"] - (1 if odd else 0)
    pays = pays[:k]
    engine = FedAvgEngine(DEV)
    engine.layout_align = align
    rnd = engine.begin(base, k)
    layout = rnd.layout
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    w1 = np.tile(np.full(k, 1.0 / k), (len(layout.entries), 1))
    grads = rnd.launch_entrywise(w1, add_base=False, device=True)
    want = rnd.fedadp_dots_flat(grads, range(k), 0.01)
    rnd.fedadp_dots(grads, range(k), 0.01)
    g_flat, ptrs, ws = rnd._keep_flat
    order = rnd._fedadp_order()
    segs, n_flat = rnd._flat_segments(order, True)
    dev = torch.device(DEV)
    # delta arenas (the delta variants, null baseline): compute_weight_deltas of every staged slot
    dslab = ClientSlab(layout, k, dev)
    h = torch.cuda.current_stream().cuda_stream
    for i in range(k):
        _lib.call("plato_agg_compute_deltas", rnd._pf[i], rnd._pi[i], engine._base.f32.data_ptr(),
                  engine._base.i64.data_ptr(), dslab.f32[i].data_ptr(), dslab.i64[i].data_ptr(), layout.n_f32,
                  layout.n_i64, h)
    dpf, dpi = dslab.row_pointers(range(k))
    dptrs = torch.from_numpy(np.concatenate([dpf, dpi]).astype(np.int64)).to(dev)
    n_delta = 0
    for v in range(_lib.tune().plato_agg_tune_num_fedadp_variants()):
        if _lib.tune().plato_agg_tune_fedadp_is_probe(v):  # timing probes: wrong results by design
            continue
        delta = bool(_lib.tune().plato_agg_tune_fedadp_is_delta(v))
        n_delta += delta
        p = dptrs if delta else ptrs
        xy = torch.full((k + 1,), float("nan"), device=dev)
        yy = torch.full((k + 1,), float("nan"), device=dev)
        _lib.tune_call("plato_agg_tune_fedadp_dots", v, g_flat.data_ptr(), p.data_ptr(), p.data_ptr() + 8 * k, k,
                       None if delta else engine._base.f32.data_ptr(), None if delta else engine._base.i64.data_ptr(),
                       segs.data_ptr(), len(order), n_flat, layout.n_f32, layout.n_i64, 0.01, 1, ws.data_ptr(),
                       xy.data_ptr(), yy.data_ptr(), h)
        torch.cuda.synchronize()
        assert xy.cpu().numpy()[:k].tobytes() == np.asarray(want[0]).tobytes(), v
        assert xy.cpu().numpy()[k:].tobytes() == np.float32(want[1]).tobytes(), v
        assert yy.cpu().numpy()[:k].tobytes() == np.asarray(want[2]).tobytes(), v
    assert n_delta >= 1


# ------------------------------------------------------- coded payloads reaching the variants
# The reference dequantizes bf16 / QSGD payloads in its inbound processor before FedAtt, FedAdp,
# Polaris or Port run (plato/processors/model_dequantize.py:15-18, model_dequantize_qsgd.py:34-60);
# the engine keeps the codes in HBM and runs those reductions on rows decoded once per round
# (AggregationRound.decoded).  Fixtures: the reference's own servers on the dequantized payloads.
def _coded(recipe):
    layout, base, _, _ = G.host_state_dicts(recipe)
    pays = G.coded_payloads(recipe)
    st = recipe.get("staleness", [0] * recipe["k"])
    updates = [types.SimpleNamespace(client_id=c + 1, report=types.SimpleNamespace(num_samples=recipe["num_samples"][c]),
                                     payload=p, staleness=st[c]) for c, p in zip(G.order_of(recipe), pays)]
    return layout, base, pays, updates


@pytest.mark.parametrize("name", ["fedatt_bf16_lenet5_k5", "fedatt_qsgd_resnet18_k3"])
def test_fedatt_coded_payloads_match_reference(engine, name):
    from plato_amd.algorithms.fedavg import FedAttAlgorithmMixin

    recipe, exp = CASES[name]["recipe"], CASES[name]["expected"]
    layout, base, pays, _ = _coded(recipe)

    class Algorithm(FedAttAlgorithmMixin):
        aggregation_device = DEV

    alg = Algorithm()
    alg._plato_amd_engine = engine
    rnd = engine.begin(base, recipe["k"], recipe["codec"])
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
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]


@pytest.mark.parametrize("name", ["fedadp_bf16_resnet18_k4", "fedadp_qsgd_lenet5_k5"])
def test_fedadp_coded_payloads_match_reference(engine, name):
    from plato_amd.servers.variants import FedAdpServerMixin

    recipe, exp = CASES[name]["recipe"], CASES[name]["expected"]
    layout, base, pays, updates = _coded(recipe)

    class Server(FedAdpServerMixin):
        aggregation_device = DEV
        fedadp_lr = 0.01

    server = Server()
    server._plato_amd_engine = engine
    server.current_round = recipe["current_round"]
    server.selected_clients = [c + 1 for c in G.order_of(recipe)]
    server.local_angles = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    assert [float(x).hex() for x in server.adaptive_weighting] == exp["adaptive_weighting"]
    assert {str(c): "%08x" % np.float32(a).view(np.uint32) for c, a in server.local_angles.items()} == \
        exp["local_angles"]
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    # the global gradient on the decoded rows: the reference's digests
    rnd = engine.begin(base, recipe["k"], recipe["codec"])
    rnd.put_baseline(base)
    for i, p in enumerate(pays):
        rnd.put_client(i, p)
    work = rnd.decoded()
    w1 = np.tile(np.asarray([u.report.num_samples for u in updates], dtype=np.float64)
                 / sum(u.report.num_samples for u in updates), (len(layout.entries), 1))
    g_f, _ = work.launch_entrywise(w1, add_base=False, device=True)
    g = g_f.cpu().numpy()
    assert G.sha(G.canon(g[: layout.n_f32])) == exp["global_grads_f32_sha256"]
    assert G.sha(G.canon(g[layout.row_f32: layout.row_f32 + layout.n_i64])) == exp["global_grads_i64f_sha256"]


def test_polaris_coded_payloads_match_reference(engine):
    from plato_amd.servers.variants import PolarisServerMixin

    recipe, exp = CASES["polaris_bf16_resnet18_k4"]["recipe"], CASES["polaris_bf16_resnet18_k4"]["expected"]
    layout, base, pays, updates = _coded(recipe)

    class Server(PolarisServerMixin):
        aggregation_device = DEV

    server = Server()
    server._plato_amd_engine = engine
    server.number_of_client = 1024
    server.unexplored_clients = list(range(1024))
    server.alpha = 10
    updated = asyncio.run(server.aggregate_weights(updates, base, pays))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(_flat(layout, updated, "i64"))) == exp["loaded_i64_sha256"]
    want = {int(c): float.fromhex(v) for c, v in exp["squared_deltas"].items()}
    got = {i: float(v) for i, v in enumerate(server.squared_deltas_current_round) if v != 0}
    assert {c: v.hex() for c, v in got.items()} == {c: v.hex() for c, v in want.items()}


def test_port_coded_payloads_with_stale_model_match_reference(tmp_path):
    from oracle import synth
    from plato_amd.servers.variants import PortServerMixin

    case = CASES["port_similarity_qsgd_lenet5_k6"]
    recipe = case["recipe"]
    layout, base, pays, updates = _coded(recipe)
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, recipe["seed"])
    pv = recipe["previous"]
    prev = layout.unpack(torch.from_numpy(synth.synth_f32(layout.n_f32, recipe["seed"], pv["stream"], pv["scale"],
                                                          add=bf)),
                         torch.from_numpy(synth.synth_i64(layout.n_i64, recipe["seed"], pv["stream"], 3, add=bi)))
    path = tmp_path / "model_prev.pth"
    torch.save(prev, path)

    class Server(PortServerMixin):
        aggregation_device = DEV
        staleness_weight = 3
        current_round = recipe["current_round"]
        port_threads = 8  # the fixture host's torch pool

        def port_previous_model_path(self):
            return str(path)

    updated = asyncio.run(Server().aggregate_weights(updates, base, pays))
    assert G.sha(G.canon(_flat(layout, updated, "f32"))) == case["expected"]["updated_f32_sha256"]
    assert G.sha(G.canon(_flat(layout, updated, "i64"))) == case["expected"]["updated_i64f_sha256"]


def _many_entries(n_entries, seed):
    """A model of n_entries small entries (1-300 elements, every 13th an int64 counter), names in
    scrambled order so that FedAdp's name order reorders the arena."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n_entries)
    spec = []
    for i in range(n_entries):
        name = f"m{perm[i]:05d}"
        if i % 13 == 5:
            spec.append((name + ".num_batches_tracked", (), "i64"))
        else:
            spec.append((name + ".weight", (int(rng.integers(1, 300)),), "f32"))
    # name order must start with an fp32 entry (the float32 case the device reproduces)
    first = min(range(n_entries), key=lambda i: spec[i][0].lower())
    spec[first] = (spec[first][0].replace(".num_batches_tracked", ".weight"), (7,), "f32")
    return ArenaLayout.from_shapes(spec)


@pytest.mark.parametrize("deltas", [False, True], ids=["weight_arenas", "delta_arenas"])
@pytest.mark.parametrize("n_entries", [300, 2600])
def test_fedadp_dots_many_entries_match_oracle(engine, n_entries, deltas):
    """More entries than the round-3 kernel's 2,048-entry segment map: every boundary group goes through
    the boundary table; the dots equal numpy's sdot order (oracle) and the flatten + sdot path bit for bit.
    ``delta_arenas``: the clients staged as deltas (FedAdp's servers' default), where the fallback to the
    flat path for models past the fused kernel's limits flattens the delta rows against a zero arena."""
    from oracle import fedavg_oracle as FO
    from oracle import reductions as R

    if deltas:
        from plato_amd.engine import FedAvgEngine

        engine = FedAvgEngine(engine.device)
        engine.delta_arenas = True
    layout = _many_entries(n_entries, n_entries)
    rng = np.random.default_rng(7)
    k, lr = 3, 0.03
    bf = rng.standard_normal(layout.n_f32).astype(np.float32)
    bi = rng.integers(-2**40, 2**40, layout.n_i64)
    xs = [((bf + 0.01 * rng.standard_normal(layout.n_f32)).astype(np.float32), bi + rng.integers(-50, 50, layout.n_i64))
          for _ in range(k)]
    base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    rnd = engine.begin(base, k)
    rnd.put_baseline(base)
    for i, (xf, xi) in enumerate(xs):
        rnd.put_client(i, layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi)))
    w1 = np.tile(np.full(k, 1.0 / k), (len(layout.entries), 1))
    g_f, g_i = rnd.launch_entrywise(w1, add_base=False, device=True)
    inner, g_sq, l_sq = rnd.fedadp_dots((g_f, g_i), range(k), lr)
    flat = rnd.fedadp_dots_flat((g_f, g_i), range(k), lr)
    # a layout past the fused kernel's limits routes to the flat path (limit lowered to force it)
    calls = []
    orig = rnd.fedadp_dots_flat
    rnd.fedadp_dots_flat = lambda *a, **kw: calls.append(1) or orig(*a, **kw)
    rnd.FEDADP_MAX_SEGS = n_entries
    routed = rnd.fedadp_dots((g_f, g_i), range(k), lr)
    assert calls and np.asarray(routed[0]).tobytes() == np.asarray(flat[0]).tobytes()
    assert np.asarray(inner).tobytes() == np.asarray(flat[0]).tobytes()
    assert np.float32(g_sq).tobytes() == np.float32(flat[1]).tobytes()
    assert np.asarray(l_sq).tobytes() == np.asarray(flat[2]).tobytes()
    # the oracle: process_grad in numpy / torch semantics, then sdot_k_SKYLAKEX's order
    gh = layout.unpack(g_f[: layout.row_f32].cpu(), g_i[: max(1, layout.n_i64)].cpu())
    g = FO.fedadp_flatten(gh, lr)
    assert R.sdot(g, g).tobytes() == np.float32(g_sq).tobytes()
    for i, (xf, xi) in enumerate(xs):
        delta = {e.name: (layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi))[e.name] - base[e.name])
                 for e in layout.entries}
        loc = FO.fedadp_flatten(delta, lr)
        assert loc.dtype == np.float32 and loc.size == layout.n_f32 + layout.n_i64
        assert R.sdot(g, loc).tobytes() == np.float32(inner[i]).tobytes(), i
        assert R.sdot(loc, loc).tobytes() == np.float32(l_sq[i]).tobytes(), i

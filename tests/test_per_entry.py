"""Per-entry variants (FedAtt, FedAdp, Polaris) on the CPU: oracle pinned to the reference.

The fixtures (tests/golden/make_golden.py) were produced by the reference's
own fedatt_algorithm / fedadp_server / polaris_server.  Here:

* the oracle's torch/numpy restatements reproduce them bit for bit;
* the kernel contract's restatement (oracle.entrywise_numpy) with the
  reference's attention weights reproduces FedAtt's model bit for bit;
* FedAtt's norms follow torch's CPU order (bit-exact); FedAdp's float32
  BLAS reductions are restated in numpy's OpenBLAS order (oracle/reductions.c,
  tests/test_reductions.py: bit-exact); Polaris' norms are fp64 per-entry
  sums (plato_agg_entry_stats), within the tolerance written below;
* the chunk tables the kernels walk cover every element exactly once.
"""

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from plato_amd import weights as W
from plato_amd.arena import ArenaLayout
from tests import golden_cases as G

CASES = {c["recipe"]["name"]: c for c in G.load_cases()}
FEDATT = [n for n, c in CASES.items() if c["recipe"].get("mode") == "fedatt"]
FEDADP = [n for n, c in CASES.items() if c["recipe"].get("mode") == "fedadp"]
POLARIS = [n for n, c in CASES.items() if c["recipe"].get("mode") == "polaris"]
LR = 0.01  # parameters.optimizer.lr of the fixture config


def _hex_matrix(rows):
    return np.array([[G.hexf(h) for h in row] for row in rows], dtype=np.float32)


# ------------------------------------------------------------------ chunks
@pytest.mark.parametrize("model,cap", [("lenet5", 4), ("lenet5", 8), ("lenet5", 1024), ("resnet18", 1024),
                                       ("resnet18", 4096), ("resnet18", 1 << 32)])
def test_chunk_tables_cover_each_element_once(model, cap):
    layout = ArenaLayout.from_shapes(G.model_spec(model))
    cf, ci = layout.chunk_tables(cap)
    for table, region, n in ((cf, "f32", layout.n_f32), (ci, "i64", layout.n_i64)):
        owner = np.full(n, -1)
        assert list(table[:, 0]) == sorted(table[:, 0])
        for entry, begin, end, _ in table:
            e = layout.entries[entry]
            assert e.region == region and e.offset <= begin < end <= e.offset + e.numel
            if region == "f32":
                assert end - begin <= cap
                if cap > layout.n_f32:
                    assert (begin, end) == (e.offset, e.offset + e.numel)  # one piece per entry
                assert int(begin) // cap == (int(end) - 1) // cap  # never crosses a cap boundary
            assert (owner[begin:end] == -1).all()
            owner[begin:end] = entry
        assert (owner == ref.entry_index(layout.entries, region, n)).all()


def test_chunk_tables_skip_empty_entries_and_validate_cap():
    layout = ArenaLayout.from_shapes([("a", (0,), "f32"), ("b", (5,), "f32"), ("c", (), "i64")])
    cf, ci = layout.chunk_tables(4)
    assert cf.tolist() == [[1, 0, 4, 0], [1, 4, 5, 0]]
    assert ci.tolist() == [[2, 0, 1, 0]]
    with pytest.raises(ValueError):
        layout.chunk_tables(6)


# ------------------------------------------------------------------ FedAtt
@pytest.mark.parametrize("name", FEDATT)
def test_fedatt_oracle_reproduces_reference(name):
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, _ = G.host_state_dicts(recipe)
    torch.manual_seed(recipe["noise_seed"])
    upd, norms, atts = ref.fedatt_torch(base, pays)
    assert norms.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_norms"]).view(np.uint32).tolist()
    assert atts.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_atts"]).view(np.uint32).tolist()
    flat = torch.cat([upd[e.name].reshape(-1) for e in layout.entries if e.region == "f32"]).numpy()
    assert G.sha(G.canon(flat)) == exp["updated_f32_sha256"]


@pytest.mark.parametrize("name", FEDATT)
def test_fedatt_kernel_contract_with_reference_attention_is_bit_exact(name):
    """entrywise_numpy (the kernel's contract) + the reference's atts + its noise stream."""
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, arenas = G.host_state_dicts(recipe)
    entries, bf, bi, xs_f, xs_i, split = G.oracle_arenas(recipe, layout, *arenas)
    torch.manual_seed(recipe["noise_seed"])
    noise = {n: torch.randn(t.shape) for n, t in base.items()}
    nf = np.zeros(max([e.offset + e.numel for e in entries if e.region == "f32"] + [0]), dtype=np.float32)
    for e in entries:
        if e.region == "f32":
            nf[e.offset:e.offset + e.numel] = noise[e.name].reshape(-1).numpy()
    ni = np.array([noise[e.name].item() for e in entries if e.region == "i64"], dtype=np.float32)
    atts = _hex_matrix(exp["fedatt_atts"])
    new_f, new_i = ref.entrywise_numpy(entries, bf, bi, xs_f, xs_i, -atts.astype(np.float64),
                                       scale=-1.2, noise_f=nf, noise_i=ni, noise_scale=0.001)
    new_f, new_i = split(new_f, new_i)
    assert G.sha(G.canon(new_f)) == exp["updated_f32_sha256"]
    assert G.sha(G.canon(new_i)) == exp["updated_i64f_sha256"]
    assert G.sha(ref.trunc_to_int64(new_i)) == exp["loaded_i64_sha256"]


@pytest.mark.parametrize("name", FEDATT)
def test_fedatt_torch_order_norms_are_bit_exact(name):
    """The norm order plato_agg_entry_norms_f32 implements (oracle.torch_cpu_norm_f32)
    gives the reference's fp32 norms bit for bit, and weights.fedatt_attention its softmax."""
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, _, _, arenas = G.host_state_dicts(recipe)
    entries, bf, bi, xs_f, xs_i, _ = G.oracle_arenas(recipe, layout, *arenas)
    norms = np.zeros((len(entries), recipe["k"]), dtype=np.float32)
    for e_i, e in enumerate(entries):
        if e.region == "f32":
            rows = np.stack([np.subtract(x[e.offset:e.offset + e.numel], bf[e.offset:e.offset + e.numel],
                                         dtype=np.float32) for x in xs_f])
        else:
            rows = np.stack([(x[e.offset:e.offset + e.numel] - bi[e.offset:e.offset + e.numel]).astype(np.float32)
                             for x in xs_i])
        norms[e_i] = ref.torch_cpu_norm_f32(rows)
    assert norms.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_norms"]).view(np.uint32).tolist()
    atts = W.fedatt_attention(norms)
    assert atts.view(np.uint32).tolist() == _hex_matrix(exp["fedatt_atts"]).view(np.uint32).tolist()


def test_fedatt_fp64_norms_differ_from_torch_order():
    """Why the device follows torch's order: a correctly rounded norm of a 2.4M-element
    ResNet-18 tensor is ~3e-5 away from torch's fp32 value (fixture fedatt_resnet18_k8)."""
    case = CASES["fedatt_resnet18_k8"]
    layout, _, _, (bf, bi, xs_f, xs_i) = G.host_state_dicts(case["recipe"])
    _, dd, _ = ref.entry_stats_fp64(layout.entries, bf, bi, xs_f[:1], xs_i[:1])
    exp = _hex_matrix(case["expected"]["fedatt_norms"])[:, 0].astype(np.float64)
    rel = np.abs(np.sqrt(dd[0]) - exp) / np.maximum(exp, 1e-30)
    assert rel.max() > 1e-5


# ------------------------------------------------------------------ FedAdp
def _fedadp_inputs(recipe):
    layout, base, pays, arenas = G.host_state_dicts(recipe)
    order = G.order_of(recipe)
    ns = [recipe["num_samples"][c] for c in order]
    deltas = [{n: x[n] - base[n] for n in x} for x in pays]
    return layout, base, pays, arenas, ns, deltas


@pytest.mark.parametrize("name", FEDADP)
def test_fedadp_oracle_reproduces_reference(name):
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, arenas, ns, deltas = _fedadp_inputs(recipe)
    _, bf, bi, xs_f, xs_i, split = G.oracle_arenas(recipe, layout, *arenas)
    w1 = ref.fedavg_weights(ns)
    d_f = [np.subtract(x, bf, dtype=np.float32) for x in xs_f]
    d_i = [x - bi for x in xs_i]
    g_f, g_i = split(*ref.deltas_numpy(d_f, d_i, w1))
    assert G.sha(G.canon(g_f)) == exp["global_grads_f32_sha256"]
    assert G.sha(G.canon(g_i)) == exp["global_grads_i64f_sha256"]
    grads = layout.unpack(torch.from_numpy(g_f), torch.from_numpy(g_i))
    angles = ref.fedadp_angles_numpy(grads, deltas, LR)
    selected = [c + 1 for c in G.order_of(recipe)]
    local = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    contribs = W.fedadp_contributions(angles, selected, local, recipe["current_round"])
    assert {str(c): "%08x" % np.float32(a).view(np.uint32) for c, a in local.items()} == exp["local_angles"]
    aw = W.fedadp_weighting(contribs, ns)
    assert [float(x).hex() for x in aw] == exp["adaptive_weighting"]
    new_f, new_i = split(*ref.fedavg_numpy(bf, bi, xs_f, xs_i, aw))
    assert G.sha(G.canon(new_f)) == exp["updated_f32_sha256"]
    assert G.sha(ref.trunc_to_int64(new_i)) == exp["loaded_i64_sha256"]


# ------------------------------------------------------------------ Polaris
@pytest.mark.parametrize("name", POLARIS)
def test_polaris_norms(name):
    """Oracle restatement bit-exact; fp64 per-entry sums within 1e-5 relative."""
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, (bf, bi, xs_f, xs_i) = G.host_state_dicts(recipe)
    deltas = [{n: x[n] - base[n] for n in x} for x in pays]
    want = {int(k): float.fromhex(v) for k, v in exp["squared_deltas"].items()}
    ids = [c for c in G.order_of(recipe)]  # client_id - 1
    exact = ref.polaris_norms_numpy(deltas)
    assert [float(v).hex() for v in exact] == [float(want[c]).hex() for c in ids]
    entries, bf, bi, xs_f, xs_i, _ = G.oracle_arenas(recipe, layout, bf, bi, xs_f, xs_i)
    _, dd, _ = ref.entry_stats_fp64(entries, bf, bi, xs_f, xs_i)
    approx = W.polaris_delta_norms(dd, layout.keys())
    np.testing.assert_allclose(np.array(approx, dtype=np.float64), [want[c] for c in ids], rtol=1e-5)
    # the unexplored clients (all others below 200) get alpha * mean
    expect = 10 * sum(exact) / len(exact)
    others = [v for c, v in want.items() if c not in ids]
    assert others and all(v == np.float64(expect) for v in others)

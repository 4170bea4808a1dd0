"""The C restatements of the variant servers' float32 reductions (oracle/reductions.c).

Pinned two ways, on the CPU:
* against the libraries the reference calls, on this host: numpy's
  ``np.inner`` / ``np.linalg.norm`` (FedAdp) and torch's
  ``F.cosine_similarity`` (Port), over ragged sizes and thread counts;
* against the reference-generated fixtures: Port's similarities and FedAdp's
  adaptive weights, bit for bit.
"""

import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fedavg_oracle as ref
from oracle import reductions as R
from oracle import synth
from plato_amd import weights as W
from tests import golden_cases as G

pytestmark = pytest.mark.skipif(not os.path.exists(R.LIB_PATH), reason="oracle library not built")
CASES = {c["recipe"]["name"]: c for c in G.load_cases()}
SIZES = list(range(1, 70)) + [127, 128, 129, 1000, 32767, 32768, 40001, 65537, 262147]


def _openblas_arch():
    try:
        import threadpoolctl

        for info in threadpoolctl.threadpool_info():
            if info.get("internal_api") == "openblas":
                return info.get("architecture")
    except Exception:  # pragma: no cover
        return None
    return None


SKX_LIKE = ("SkylakeX", "Cooperlake", "SapphireRapids")


@pytest.mark.skipif(_openblas_arch() not in SKX_LIKE, reason="numpy's OpenBLAS picked another CPU kernel here")
def test_sdot_restatement_equals_numpy_inner_and_norm():
    import threadpoolctl

    rng = np.random.default_rng(3)
    for n in SIZES:
        x = rng.standard_normal(n).astype(np.float32)
        y = (rng.standard_normal(n) * 1e-3).astype(np.float32)
        for threads in (1, 4):
            with threadpoolctl.threadpool_limits(threads, user_api="blas"):
                assert R.sdot(x, y) == np.float32(np.inner(x, y)), (n, threads)
                assert R.np_norm(y) == np.linalg.norm(y), (n, threads)


@pytest.mark.parametrize("threads", [1, 2, 3, 8, 16])
def test_torch_reductions_restatement_equals_torch(threads):
    rng = np.random.default_rng(threads)
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for n in SIZES + [1 << 20, (1 << 20) + 5]:
            a = (rng.standard_normal(n) * 1e-2).astype(np.float32)
            b = (rng.standard_normal(n) * 3e-2).astype(np.float32) + a
            ta, tb = torch.from_numpy(a), torch.from_numpy(b)
            assert R.torch_norm(a) == np.float32(torch.linalg.vector_norm(ta).item()), n
            assert R.torch_sum(b, threads) == np.float32(tb.sum().item()), n
            assert R.torch_cosine(a, b, threads) == np.float32(F.cosine_similarity(ta, tb, dim=0).item()), n
    finally:
        torch.set_num_threads(old)


def _port_vectors(recipe):
    from plato_amd.arena import ArenaLayout

    layout = ArenaLayout.from_shapes(G.model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    pv = recipe["previous"]
    pf = synth.synth_f32(layout.n_f32, seed, pv["stream"], pv["scale"], add=bf)
    pi = synth.synth_i64(layout.n_i64, seed, pv["stream"], 3, add=bi)
    v = R.port_current_minus_previous(layout.entries, bf, bi, pf, pi)
    ds = []
    for c in G.order_of(recipe):
        xf, xi = synth.client_arena(bf, bi, seed, c)
        ds.append(R.port_delta(layout.entries, bf, bi, xf, xi))
    return v, ds


# the fixtures were generated with torch's default pool on the 8-CPU survey host
FIXTURE_TORCH_THREADS = 8


@pytest.mark.parametrize("name", ["port_similarity_lenet5_k8", "port_similarity_resnet18_k4"])
def test_port_similarity_restatement_reproduces_reference_bits(name):
    case = CASES[name]
    recipe = case["recipe"]
    v, ds = _port_vectors(recipe)
    sims = G.reference_similarities(case)
    st = [recipe["staleness"][c] for c in G.order_of(recipe)]
    checked = 0
    for i, s in enumerate(sims):
        if st[i] <= 1:
            continue
        got = R.torch_cosine(v, ds[i], FIXTURE_TORCH_THREADS)
        assert got.tobytes() == np.float32(s).tobytes(), (i, got, s)
        checked += 1
    assert checked


LR = 0.01  # parameters.optimizer.lr of the FedAdp fixture config


@pytest.mark.parametrize("name", ["fedadp_lenet5_k6", "fedadp_resnet18_k8"])
def test_fedadp_weights_from_restated_dots_reproduce_reference_bits(name):
    case = CASES[name]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, (bf, bi, xs_f, xs_i) = G.host_state_dicts(recipe)
    ns = [recipe["num_samples"][c] for c in G.order_of(recipe)]
    d_f = [np.subtract(x, bf, dtype=np.float32) for x in xs_f]
    g_f, g_i = ref.deltas_numpy(d_f, [x - bi for x in xs_i], ref.fedavg_weights(ns))
    grads = layout.unpack(torch.from_numpy(g_f), torch.from_numpy(g_i))
    g = ref.fedadp_flatten(grads, LR)
    inner, l_sq = [], []
    for x in pays:
        loc = ref.fedadp_flatten({n: x[n] - base[n] for n in x}, LR)
        inner.append(R.sdot(g, loc))
        l_sq.append(R.sdot(loc, loc))
    angles = W.fedadp_angles_from_dots(inner, R.sdot(g, g), l_sq)
    selected = [c + 1 for c in G.order_of(recipe)]
    local = {int(c): np.float32(float.fromhex(a)) for c, a in recipe.get("local_angles", {}).items()}
    contribs = W.fedadp_contributions(angles, selected, local, recipe["current_round"])
    aw = W.fedadp_weighting(contribs, ns)
    assert [float(x).hex() for x in aw] == exp["adaptive_weighting"]
    assert {str(c): "%08x" % np.float32(a).view(np.uint32) for c, a in local.items()} == exp["local_angles"]


def test_numpy_sum_restatement_equals_np_sum_of_squares():
    rng = np.random.default_rng(11)
    for shape in [(1,), (7,), (8,), (100,), (129,), (8192,), (8193,), (20000,), (100003,), (64, 3, 3, 3),
                  (512, 256, 3, 3)]:
        d = (rng.standard_normal(shape) * 1e-2).astype(np.float32)
        assert R.np_sum(np.square(d).ravel()) == np.sum(np.square(d)), shape


def test_polaris_norms_from_restated_sums_reproduce_reference_bits():
    case = CASES["polaris_resnet18_k8"]
    recipe, exp = case["recipe"], case["expected"]
    layout, base, pays, (bf, bi, xs_f, xs_i) = G.host_state_dicts(recipe)
    names = layout.keys()
    got = {}
    for c, x in zip(G.order_of(recipe), pays):
        sums = np.zeros(len(names), dtype=np.float32)
        for e_i, e in enumerate(layout.entries):
            if e.region == "f32" and "conv" in e.name:
                d = np.subtract(x[e.name].numpy(), base[e.name].numpy(), dtype=np.float32)
                sums[e_i] = R.np_sum(np.square(d).ravel())
        got[c] = W.polaris_delta_norms(sums[None, :], names)[0]
    want = {int(c): float.fromhex(v) for c, v in exp["squared_deltas"].items()}
    assert {c: float(v).hex() for c, v in got.items()} == {c: float(want[c]).hex() for c in got}
    # unexplored clients get alpha * the mean norm, accumulated like the reference (float32 norms)
    total = 0
    for c in got:
        total += got[c]
    expect = 10 * (total / len(got))  # alpha of the fixture config
    assert all(float(want[c]).hex() == float(expect).hex() for c in want if c not in got)

"""Loading and replaying the reference-generated golden cases (tests/golden/).

A case = recipe (model, K, seed, num_samples, order, staleness, overrides,
mode) + what the reference produced (SHA-256 of its outputs, samples, and full
arrays for small cases).  ``weights_for`` derives the per-client numbers a
recipe implies, either with the product's host functions (plato_amd.weights)
or the oracle's restatement, so both sides get pinned.
"""

from __future__ import annotations

import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
CANON_NAN = np.uint32(0x7FC00000)


def load_cases():
    with open(os.path.join(GOLDEN, "fedavg_cases.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        # async simulated wall time: the update order is what the reference's
        # _process_clients produced (heap pops + stale sweep); replay it
        if c["recipe"].get("mode") == "async_wall":
            c["recipe"] = dict(c["recipe"], order=c["expected"]["updates_order"])
    return cases


def load_full():
    return np.load(os.path.join(GOLDEN, "fedavg_full_small.npz"), allow_pickle=False)


def load_known_answer():
    with open(os.path.join(GOLDEN, "known_answer_fedavg_tests.json")) as f:
        return json.load(f)


def load_shapes(name):
    with open(os.path.join(GOLDEN, f"shapes_{name}.json")) as f:
        return [(k, tuple(s), r) for k, s, r in json.load(f)]


def canon(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32).copy()
    a.view(np.uint32)[np.isnan(a)] = CANON_NAN
    return a


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def hexf(bits: str) -> np.float32:
    return np.array([int(bits, 16)], dtype=np.uint32).view(np.float32)[0]


def order_of(recipe):
    return recipe.get("order", list(range(recipe["k"])))


def reference_similarities(case):
    """Port similarities the reference computed: 1.0 or np.float32 (from fp32 hex)."""
    sims = case["expected"].get("port_similarities")
    if sims is None:
        return None
    return [s if isinstance(s, float) else hexf(s) for s in sims]


def weights_for(recipe, impl, similarities=None):
    """(weights, scales) in update order.  ``impl`` is plato_amd.weights or an oracle shim."""
    order = order_of(recipe)
    ns = [recipe["num_samples"][c] for c in order]
    st = [recipe.get("staleness", [0] * recipe["k"])[c] for c in order]
    mode = recipe.get("mode", "fedavg")
    if mode in ("fedavg", "polaris", "cross_silo", "async_wall"):  # plain FedAvg weights
        return impl.fedavg(ns), None
    if mode == "fedbuff":
        return impl.fedbuff(len(ns)), None
    if mode == "port":
        return impl.port(ns, st, similarities, similarity_weight=1, staleness_weight=3,
                         staleness_bound=10), None
    if mode == "pisces":
        first, second = impl.pisces(ns, [[s] for s in st], 0.5)
        return first, second
    raise ValueError(mode)


def plain_fedavg_weights(recipe) -> bool:
    """The case's expected model follows from weights_for() alone (no staged-round reduction:
    FedAtt / FedAdp, or Port with a stale model on disk, have their own tests)."""
    return recipe.get("mode", "fedavg") not in ("fedatt", "fedadp") and "previous" not in recipe


def fedasync_mixing(recipe, impl):
    st = recipe.get("staleness", [0])[0]
    return impl.fedasync_mixing(0.9, st, "hinge", 10, 4)


def model_spec(name):
    from plato_amd import workloads

    return {
        "lenet5": lambda: workloads.lenet5(10),
        "resnet18": lambda: workloads.resnet(18, 10),
        "resnet50_200": lambda: workloads.resnet(50, 200),
        # C5: the layouts of the HuggingFace modules the generator built (shapes_*.json, recorded with the case)
        "vit_large_hf": lambda: load_shapes("vit_large_hf"),
        "gpt2_medium_hf": lambda: load_shapes("gpt2_medium_hf"),
    }[name]()


def apply_overrides(bf, bi, xs_f, xs_i, overrides):
    for tgt, region, idx, val in overrides:
        if region == "f32":
            arr = bf if tgt == "base" else xs_f[tgt]
            arr.view(np.uint32)[idx] = np.uint32(int(val, 16))
        else:
            arr = bi if tgt == "base" else xs_i[tgt]
            arr[idx] = np.int64(int(val))


def tied_ranges(recipe, layout):
    """[(dst_offset, src_offset, numel)] of the recipe's tied fp32 entries (``tied``: [[dst, src]] names).

    A model with tied weights (GPT-2's lm_head and transformer.wte) lists both keys in its state_dict
    over one storage, so the server's baseline and every client's payload hold the same values under
    both: the generator copies src's values over dst's in the baseline and in every client."""
    out = []
    for dst, src in recipe.get("tied", []):
        d, s = layout[dst], layout[src]
        assert d.numel == s.numel and d.region == s.region == "f32"
        out.append((d.offset, s.offset, d.numel))
    return out


def apply_tied(bf, xs_f, ranges):
    for dst, src, n in ranges:
        for arr in [bf, *xs_f]:
            arr[dst:dst + n] = arr[src:src + n]


def case_size(recipe):
    from plato_amd import workloads

    return recipe["k"] * workloads.numel(model_spec(recipe["model"]))


# modes whose weights depend on reductions over the deltas (own tests)
PER_ENTRY_MODES = ("fedatt", "fedadp")
# modes with their own arithmetic (float64 weights / vectors): own tests
OWN_TEST_MODES = ("rl", "rl_f32", "he")


def host_state_dicts(recipe):
    """(layout, baseline, payloads in update order) as CPU state_dicts from the counter generator.

    For a coded recipe the payloads are what the reference's inbound processor hands the server
    (model_dequantize / model_dequantize_qsgd): every entry float32, the counters too; the arrays in
    the last item are then float32 for both regions.  ``coded_payloads`` gives the wire-side form.
    """
    import torch

    from oracle import synth
    from plato_amd.arena import ArenaLayout

    layout = ArenaLayout.from_shapes(model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    codec = recipe.get("codec")
    if codec == "bf16":
        from oracle import fedavg_oracle as ref

        xs = [(ref.bf16_roundtrip(xf), ref.bf16_roundtrip(xi)) for xf, xi in xs]
    elif codec == "qsgd":
        from oracle import qsgd

        xs = [qsgd.dequantize_regions(layout.entries, *qsgd.client_wire(layout.entries, seed, c)[1:])
              for c in range(k)]
    base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    pays = [layout.unpack(torch.from_numpy(xs[c][0]), torch.from_numpy(xs[c][1])) for c in order_of(recipe)]
    return layout, base, pays, (bf, bi, [xs[c][0] for c in order_of(recipe)], [xs[c][1] for c in order_of(recipe)])


def coded_payloads(recipe):
    """The payloads of a coded recipe as the server receives them, in update order: bf16 state_dicts
    (model_quantize's .to(bfloat16) of every entry) or QSGD payloads parsed by the product processor."""
    import torch

    from oracle import synth
    from plato_amd.arena import ArenaLayout

    layout = ArenaLayout.from_shapes(model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    if recipe["codec"] == "bf16":
        bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
        xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
        pays = [layout.unpack(torch.from_numpy(xf), torch.from_numpy(xi)) for xf, xi in xs]
        pays = [type(p)((n, t.to(torch.bfloat16)) for n, t in p.items()) for p in pays]
    else:
        from oracle import qsgd
        from plato_amd.processors.qsgd import Processor

        proc = Processor()
        pays = [proc.process(qsgd.client_wire(layout.entries, seed, c)[0]) for c in range(k)]
    return [pays[c] for c in order_of(recipe)]


def oracle_arenas(recipe, layout, bf, bi, xs_f, xs_i):
    """The arenas the kernel-contract restatements compute on, and how to split their results.

    Native recipes: as given.  Coded recipes: the reference reduces dequantized payloads whose
    counters are float32, so a counter's delta is float32(x) - float32(b); the device runs those
    rounds on ``layout.promoted()`` rows (AggregationRound.decoded), and so does the oracle here:
    entries all fp32, the counters after the padded fp32 region, the baseline's cast with RNE.
    Returns ``(entries, bf, bi, xs_f, xs_i, split)``; ``split(flat_f32, flat_i64)`` gives the
    results as (fp32 region, counter values) of the original layout.
    """
    if not recipe.get("codec"):
        return layout.entries, bf, bi, xs_f, xs_i, lambda f, i: (f, i)
    play = layout.promoted()
    n_f, n_i, row = layout.n_f32, layout.n_i64, layout.row_f32

    def prom(f, i):
        out = np.zeros(play.n_f32, dtype=np.float32)
        out[:n_f] = f
        out[row:row + n_i] = np.asarray(i).astype(np.float32)
        return out

    empty = np.zeros(0, dtype=np.int64)
    return (play.entries, prom(bf, bi), empty, [prom(f, i) for f, i in zip(xs_f, xs_i)], [empty] * len(xs_f),
            lambda f, i: (f[:n_f], f[row:row + n_i]))

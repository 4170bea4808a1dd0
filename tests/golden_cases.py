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


def fedasync_mixing(recipe, impl):
    st = recipe.get("staleness", [0])[0]
    return impl.fedasync_mixing(0.9, st, "hinge", 10, 4)


def model_spec(name):
    from plato_amd import workloads

    return {
        "lenet5": lambda: workloads.lenet5(10),
        "resnet18": lambda: workloads.resnet(18, 10),
        "resnet50_200": lambda: workloads.resnet(50, 200),
    }[name]()


def apply_overrides(bf, bi, xs_f, xs_i, overrides):
    for tgt, region, idx, val in overrides:
        if region == "f32":
            arr = bf if tgt == "base" else xs_f[tgt]
            arr.view(np.uint32)[idx] = np.uint32(int(val, 16))
        else:
            arr = bi if tgt == "base" else xs_i[tgt]
            arr[idx] = np.int64(int(val))


def case_size(recipe):
    from plato_amd import workloads

    return recipe["k"] * workloads.numel(model_spec(recipe["model"]))


# modes whose weights depend on reductions over the deltas (own tests)
PER_ENTRY_MODES = ("fedatt", "fedadp")
# modes with their own arithmetic (float64 weights / vectors): own tests
OWN_TEST_MODES = ("rl", "rl_f32", "he")


def host_state_dicts(recipe):
    """(layout, baseline, payloads in update order) as CPU state_dicts from the counter generator."""
    import torch

    from oracle import synth
    from plato_amd.arena import ArenaLayout

    layout = ArenaLayout.from_shapes(model_spec(recipe["model"]))
    k, seed = recipe["k"], recipe["seed"]
    bf, bi = synth.baseline_arena(layout.n_f32, layout.n_i64, seed)
    xs = [synth.client_arena(bf, bi, seed, c) for c in range(k)]
    base = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    pays = [layout.unpack(torch.from_numpy(xs[c][0]), torch.from_numpy(xs[c][1])) for c in order_of(recipe)]
    return layout, base, pays, (bf, bi, [xs[c][0] for c in order_of(recipe)], [xs[c][1] for c in order_of(recipe)])

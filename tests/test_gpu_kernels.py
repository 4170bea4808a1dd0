"""GPU parity of the HIP FedAvg kernels against the CPU oracle (bit-exact).

Inputs are generated on the device by ``plato_agg_fill_synth_*`` and on the
host by the numpy restatement ``oracle/synth.py``; the tests first check the
two generators agree bit for bit, then compare every kernel's output with the
oracle's sequential fp32 restatement (``oracle/fedavg_oracle.py``).
"""

import numpy as np
import pytest
import torch

from oracle import fedavg_oracle as ref
from oracle import synth
from plato_amd import _lib, workloads
from plato_amd.arena import ArenaLayout
from plato_amd.engine import ClientSlab, DeviceArena, FedAvgEngine
from plato_amd.synthetic import fill_baseline, fill_clients
from tests.helpers import bits_equal, first_mismatch, host_inputs

pytestmark = pytest.mark.gpu


def _device_case(spec, k, seed):
    dev = torch.device("cuda:0")
    layout = ArenaLayout.from_shapes(spec)
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    fill_baseline(base, seed)
    fill_clients(slab, base, seed, k)
    return layout, base, slab


def _run(engine, layout, base, slab, k, weights, scales=None, deltas_mode=False, variant=None):
    dev = base.f32.device
    pf, pi = slab.row_pointers(range(k))
    tf = torch.from_numpy(pf).to(dev)
    ti = torch.from_numpy(pi).to(dev)
    w = torch.from_numpy(ref.fp32(weights)).to(dev)
    s = None if scales is None else torch.from_numpy(ref.fp32(scales)).to(dev)
    out_f = torch.full((layout.row_f32,), float("nan"), device=dev)
    out_i = torch.full((layout.row_i64,), float("nan"), device=dev)
    engine.variant = variant
    engine.launch_fedavg(layout, tf, ti, w, s, k, None if deltas_mode else base.f32,
                         None if deltas_mode else base.i64, out_f, out_i)
    torch.cuda.synchronize()
    return out_f[: layout.n_f32].cpu().numpy(), out_i[: layout.n_i64].cpu().numpy()


@pytest.fixture(scope="module")
def engine():
    return FedAvgEngine("cuda:0")


def test_generator_matches_oracle():
    layout, base, slab = _device_case(workloads.lenet5(), 3, seed=7)
    bf, bi, xs_f, _ = host_inputs(layout.n_f32, layout.n_i64, 7, 3)
    assert bits_equal(base.f32[: layout.n_f32].cpu().numpy(), bf)
    for c in range(3):
        assert bits_equal(slab.f32[c, : layout.n_f32].cpu().numpy(), xs_f[c])
    # int64 generator on a ResNet arena
    layout, base, slab = _device_case(workloads.resnet(18), 2, seed=3)
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, 3, 2)
    assert np.array_equal(base.i64[: layout.n_i64].cpu().numpy(), bi)
    assert np.array_equal(slab.i64[1, : layout.n_i64].cpu().numpy(), xs_i[1])


@pytest.mark.parametrize(
    "model,k,seed",
    [("lenet5", 10, 1), ("resnet18", 16, 2), ("resnet18", 13, 3), ("lenet5", 1, 4)],
)
def test_fedavg_weights_bit_exact(engine, model, k, seed):
    spec = workloads.lenet5() if model == "lenet5" else workloads.resnet(18)
    layout, base, slab = _device_case(spec, k, seed)
    ns = synth.num_samples(k, seed)
    weights = ref.fedavg_weights(ns)
    got_f, got_i = _run(engine, layout, base, slab, k, weights)
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, seed, k)
    exp_f, exp_i = ref.fedavg_numpy(bf, bi, xs_f, xs_i, weights)
    assert bits_equal(got_f, exp_f), first_mismatch(got_f, exp_f)
    assert bits_equal(got_i, exp_i), first_mismatch(got_i, exp_i)


def test_all_variants_identical(engine):
    spec = workloads.resnet(18)
    k, seed = 11, 5
    layout, base, slab = _device_case(spec, k, seed)
    weights = ref.fedavg_weights(synth.num_samples(k, seed))
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, seed, k)
    exp_f, exp_i = ref.fedavg_numpy(bf, bi, xs_f, xs_i, weights)
    for v in range(_lib.tune().plato_agg_tune_num_variants()):
        got_f, got_i = _run(engine, layout, base, slab, k, weights, variant=v)
        assert bits_equal(got_f, exp_f), (v, first_mismatch(got_f, exp_f))
        assert bits_equal(got_i, exp_i), v
    engine.variant = None


def test_deltas_mode_and_two_scales(engine):
    spec = workloads.lenet5()
    k, seed = 9, 6
    layout, base, slab = _device_case(spec, k, seed)
    weights = ref.fedavg_weights(synth.num_samples(k, seed))
    scales = [1.0 / (1 + 0.37 * i) ** 0.5 for i in range(k)]
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, seed, k)
    got_f, got_i = _run(engine, layout, base, slab, k, weights, scales=scales, deltas_mode=True)
    exp_f, exp_i = ref.deltas_numpy(xs_f, xs_i, weights, scales)
    assert bits_equal(got_f, exp_f), first_mismatch(got_f, exp_f)
    got_f, _ = _run(engine, layout, base, slab, k, weights, scales=scales)
    exp_f, _ = ref.fedavg_numpy(bf, bi, xs_f, xs_i, weights, scales)
    assert bits_equal(got_f, exp_f), first_mismatch(got_f, exp_f)


def test_engine_host_path_matches_torch_ops(engine):
    """aggregate_weights on CPU state_dicts == the reference's torch op sequence."""
    spec = workloads.resnet(18)
    k, seed = 5, 9
    layout = ArenaLayout.from_shapes(spec)
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, seed, k)
    base_sd = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [layout.unpack(torch.from_numpy(xs_f[c]), torch.from_numpy(xs_i[c])) for c in range(k)]
    ns = synth.num_samples(k, seed)
    got = engine.aggregate_weights(base_sd, payloads, ref.fedavg_weights(ns))
    exp = ref.fedavg_torch_ops(base_sd, payloads, num_samples=ns)
    assert list(got.keys()) == list(exp.keys())
    for name in exp:
        assert got[name].dtype == exp[name].dtype, name
        assert torch.equal(got[name].view(torch.int32), exp[name].view(torch.int32)), name


def test_cast_and_mix(engine):
    from plato_amd.engine import cast_to_int64

    vals = np.array([5.9999, -0.5, -7.99, 1e10, 2.0**63, -(2.0**63), np.nan, np.inf, 0.0, -3.0],
                    dtype=np.float32)
    got = cast_to_int64(torch.from_numpy(vals).cuda()).cpu().numpy()
    assert np.array_equal(got, ref.trunc_to_int64(vals))
    layout = ArenaLayout.from_shapes(workloads.resnet(18))
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, 4, 1)
    base_sd = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    recv = layout.unpack(torch.from_numpy(xs_f[0]), torch.from_numpy(xs_i[0]))
    got = engine.mix_weights(base_sd, recv, 0.9 * 0.6)
    exp_f, exp_i = ref.mix_numpy(bf, bi, xs_f[0], xs_i[0], 0.9 * 0.6)
    got_f = torch.cat([got[e.name].reshape(-1) for e in layout.entries if e.region == "f32"]).numpy()
    assert bits_equal(got_f, exp_f), first_mismatch(got_f, exp_f)


def test_compute_deltas_and_update(engine):
    layout = ArenaLayout.from_shapes(workloads.lenet5())
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, 8, 3)
    base_sd = layout.unpack(torch.from_numpy(bf), torch.from_numpy(bi))
    payloads = [layout.unpack(torch.from_numpy(xs_f[c]), torch.from_numpy(xs_i[c])) for c in range(3)]
    deltas = engine.compute_weight_deltas(base_sd, payloads)
    for c in range(3):
        for name, t in deltas[c].items():
            assert torch.equal(t, payloads[c][name] - base_sd[name]), name
    ns = [100, 250, 40]
    avg = engine.aggregate_deltas(deltas, ref.fedavg_weights(ns))
    upd = engine.update_weights(base_sd, avg)
    exp = ref.fedavg_torch_ops(base_sd, payloads, num_samples=ns)
    for name in exp:
        assert torch.equal(upd[name], exp[name]), name


@pytest.mark.parametrize("groups", [1000, 4096, 777777])
def test_split_launch_ranges_bit_exact(engine, groups):
    """Arenas beyond one launch's 4 GiB reach run as consecutive ranges; emulate with a small range."""
    spec = workloads.resnet(18)
    k, seed = 7, 12
    layout, base, slab = _device_case(spec, k, seed)
    weights = ref.fedavg_weights(synth.num_samples(k, seed))
    scales = [1.0 / (1 + 0.11 * i) for i in range(k)]
    bf, bi, xs_f, xs_i = host_inputs(layout.n_f32, layout.n_i64, seed, k)
    lib = _lib.tune()
    lib.plato_agg_tune_set_launch_groups(groups)
    try:
        for v in (0, 6, 5):  # variant 0 = the default kernel, from the tuning library whose split is lowered
            got_f, got_i = _run(engine, layout, base, slab, k, weights, scales=scales, variant=v)
            exp_f, exp_i = ref.fedavg_numpy(bf, bi, xs_f, xs_i, weights, scales)
            assert bits_equal(got_f, exp_f), (v, first_mismatch(got_f, exp_f))
            assert bits_equal(got_i, exp_i), v
        # bf16 payloads take the same split
        slab16 = ClientSlab(layout, k, base.f32.device, codec="bf16")
        slab16.f32.copy_(slab.f32.to(torch.bfloat16))
        slab16.i64.copy_(slab.i64.to(torch.bfloat16))
        pf, pi = slab16.row_pointers(range(k))
        dev = base.f32.device
        tf, ti = torch.from_numpy(pf).to(dev), torch.from_numpy(pi).to(dev)
        w = torch.from_numpy(ref.fp32(weights)).to(dev)
        out_f = torch.full((layout.row_f32,), float("nan"), device=dev)
        out_i = torch.full((layout.row_i64,), float("nan"), device=dev)
        _lib.tune_call("plato_agg_fedavg_weights_bf16", tf.data_ptr(), ti.data_ptr(), w.data_ptr(), None, k,
                       base.f32.data_ptr(), base.i64.data_ptr(), out_f.data_ptr(), out_i.data_ptr(),
                  layout.n_f32, layout.n_i64, torch.cuda.current_stream().cuda_stream)
        lib.plato_agg_tune_set_launch_groups(0)
        ref_f = torch.full_like(out_f, float("nan"))
        ref_i = torch.full_like(out_i, float("nan"))
        _lib.call("plato_agg_fedavg_weights_bf16", tf.data_ptr(), ti.data_ptr(), w.data_ptr(), None, k,
                  base.f32.data_ptr(), base.i64.data_ptr(), ref_f.data_ptr(), ref_i.data_ptr(),
                  layout.n_f32, layout.n_i64, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(out_f[: layout.n_f32].view(torch.int32), ref_f[: layout.n_f32].view(torch.int32))
        assert torch.equal(out_i[: layout.n_i64].view(torch.int32), ref_i[: layout.n_i64].view(torch.int32))
    finally:
        lib.plato_agg_tune_set_launch_groups(0)
        engine.variant = None


def test_arena_beyond_4gib_one_launch_call(engine):
    """A 1.1 G-parameter fp32 arena (4.4 GB per client) through the public entry point; sampled check."""
    n = (1 << 30) + 12345  # > 4 GiB of fp32, with a ragged tail
    layout = ArenaLayout.from_shapes([("w", (n,), "f32"), ("c", (3,), "i64")])
    k, seed = 2, 21
    dev = torch.device("cuda:0")
    base = DeviceArena(layout, dev)
    slab = ClientSlab(layout, k, dev)
    fill_baseline(base, seed)
    fill_clients(slab, base, seed, k)
    weights = [0.25, 0.75]
    got_f, got_i = _run(engine, layout, base, slab, k, weights)
    rng = np.random.default_rng(0)
    idx = np.unique(np.concatenate([rng.integers(0, n, 4096), np.arange(n - 64, n),
                                    np.arange((1 << 30) - 64, (1 << 30) + 64)]))
    bf = base.f32[: n].cpu().numpy()[idx]
    xs = [slab.f32[c, : n].cpu().numpy()[idx] for c in range(k)]
    exp_f, _ = ref.fedavg_numpy(bf, np.zeros(0, np.int64), xs, [np.zeros(0, np.int64)] * k, weights)
    assert bits_equal(got_f[idx], exp_f)
    del slab, base
    torch.cuda.empty_cache()

"""Host staging on the CPU: native pack == the arena layout, tracing no-ops, result-pool accounting."""

import numpy as np
import pytest
import torch

from plato_amd import ingest, tracing, workloads
from plato_amd.arena import ArenaLayout
from plato_amd.staging import HostPacker, _in_use

pytestmark = pytest.mark.skipif(not __import__("os").path.exists(ingest.LIB_PATH), reason="ingest lib not built")


def _state_dict(layout, seed, dtype_f=torch.float32, dtype_i=torch.int64):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for e in layout.entries:
        if e.region == "f32":
            out[e.name] = torch.randn(e.shape, generator=g).to(dtype_f)
        else:
            out[e.name] = torch.randint(0, 1000, e.shape, generator=g).to(dtype_i)
    return out


@pytest.mark.parametrize("model", ["lenet5", "resnet18"])
def test_native_pack_equals_layout_pack(model):
    spec = workloads.lenet5() if model == "lenet5" else workloads.resnet(18)
    layout = ArenaLayout.from_shapes(spec)
    sd = _state_dict(layout, 1)
    # one non-contiguous entry: packed through a contiguous copy
    name = next(e.name for e in layout.entries if len(e.shape) == 2 or len(e.shape) == 4)
    sd[name] = sd[name].clone().transpose(0, -1).contiguous().transpose(0, -1)
    assert not sd[name].is_contiguous()
    exp_f = torch.empty(layout.row_f32)
    exp_i = torch.empty(layout.row_i64, dtype=torch.int64)
    layout.pack(sd, exp_f, exp_i)
    got_f = torch.full((layout.row_f32,), float("nan"))
    got_i = torch.full((layout.row_i64,), -1, dtype=torch.int64)
    HostPacker(layout).pack(sd, got_f, got_i)
    assert torch.equal(got_f[: layout.n_f32], exp_f[: layout.n_f32])
    assert torch.equal(got_i[: layout.n_i64], exp_i[: layout.n_i64])


def test_native_pack_bf16_codec_and_errors():
    layout = ArenaLayout.from_shapes(workloads.lenet5())
    sd = _state_dict(layout, 2, torch.bfloat16, torch.bfloat16)
    out_f = torch.empty(layout.row_f32, dtype=torch.bfloat16)
    out_i = torch.empty(layout.row_i64, dtype=torch.bfloat16)
    HostPacker(layout, "bf16").pack(sd, out_f, out_i)
    flat = torch.cat([sd[e.name].reshape(-1) for e in layout.entries if e.region == "f32"])
    assert torch.equal(out_f[: layout.n_f32], flat)
    bad = dict(sd)
    first = layout.entries[0].name
    bad[first] = bad[first].reshape(-1)[:-1]
    with pytest.raises(ValueError):
        HostPacker(layout, "bf16").pack(bad, out_f, out_i)
    with pytest.raises(ValueError):
        HostPacker(layout).pack(sd, out_f, out_i)  # bf16 tensors into a native layout


def test_pack_refuses_pieces_outside_the_destination():
    import ctypes

    lib = ingest.lib()
    src = np.arange(16, dtype=np.uint8)
    dst = np.zeros(8, dtype=np.uint8)
    ptrs = (ctypes.c_uint64 * 1)(src.ctypes.data)
    nbytes = (ctypes.c_uint64 * 1)(16)
    offs = (ctypes.c_uint64 * 1)(0)
    rc = lib.plato_ingest_pack(ptrs, nbytes, offs, 1, dst.ctypes.data, dst.size, 1)
    assert rc == -5 and not dst.any()


def test_tracing_ranges_nest_without_a_profiler():
    with tracing.range("outer"):
        with tracing.range("inner"):
            pass


def test_result_pool_use_count():
    t = torch.empty(64)
    assert not _in_use(t)
    v = t[3:9]
    assert _in_use(t)
    del v
    assert not _in_use(t)


def test_baseline_key_follows_storage_and_in_place_writes():
    """staging.baseline_key (delta arenas at arrival): equal for the same model's state_dict taken twice,
    different after an in-place write (load_state_dict's copy_) or for a copy of the same values."""
    from plato_amd.staging import baseline_key

    model = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.BatchNorm1d(3))
    k0 = baseline_key(model.state_dict())
    assert baseline_key(model.state_dict()) == k0  # fresh tensor objects, same storage and versions
    clone = {n: t.clone() for n, t in model.state_dict().items()}
    assert baseline_key(clone) != k0  # same values elsewhere: another model as far as arrivals go
    model.load_state_dict({n: t + 1 if t.is_floating_point() else t for n, t in clone.items()})
    assert baseline_key(model.state_dict()) != k0  # written in place: the version counters moved
    with torch.inference_mode():
        frozen = {"w": torch.ones(3)}
    assert baseline_key(frozen) is None  # inference tensors keep no version counter: no key, no arrival deltas

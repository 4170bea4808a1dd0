"""Arena layouts (plato_amd.arena): packed and FedAdp-aligned, on the CPU."""

import numpy as np
import pytest
import torch

from plato_amd import workloads
from plato_amd.arena import F32, FEDADP_ALIGN, I64, ArenaLayout, fedadp_order
from plato_amd.staging import HostPacker


def _flat_positions(layout):
    pos, flat = {}, 0
    for i in fedadp_order(layout.keys()):
        e = layout.entries[i]
        pos[e.name] = flat
        flat += e.numel
    return pos


def test_fedadp_alignment_puts_entries_on_their_flat_position_mod_32():
    packed = ArenaLayout.from_shapes(workloads.resnet(18))
    lay = packed.aligned("fedadp")
    pos = _flat_positions(lay)
    for e in lay.entries:
        if e.region == F32:
            assert (e.offset - pos[e.name]) % FEDADP_ALIGN == 0, e.name
    f32 = sorted((e for e in lay.entries if e.region == F32), key=lambda e: e.offset)
    for a, b in zip(f32, f32[1:]):  # no overlap, padding < FEDADP_ALIGN between consecutive entries
        assert a.offset + a.numel <= b.offset < a.offset + a.numel + FEDADP_ALIGN
    assert lay.n_f32_data == packed.n_f32 and lay.n_f32 >= packed.n_f32
    assert lay.n_f32 - packed.n_f32 < FEDADP_ALIGN * len(f32)
    assert lay.algorithmic_bytes(128) == packed.algorithmic_bytes(128)  # padding is not model data
    assert [e.offset for e in lay.entries if e.region == I64] == [e.offset for e in packed.entries if e.region == I64]
    assert lay.signature != packed.signature and lay.aligned(None).signature == packed.signature
    assert not lay.packed and packed.packed


def test_aligned_pack_unpack_round_trip():
    spec = [("Zeta.w", (5, 3), "f32"), ("a.n", (), "i64"), ("b", (33,), "f32"), ("A", (7,), "f32"),
            ("c.n", (2,), "i64"), ("d", (64,), "f32")]
    lay = ArenaLayout.from_shapes(spec, align="fedadp")
    rng = np.random.default_rng(0)
    sd = {}
    for name, shape, region in spec:
        sd[name] = (torch.from_numpy(rng.standard_normal(shape).astype(np.float32)) if region == F32
                    else torch.from_numpy(rng.integers(0, 99, shape)))
    f = torch.full((lay.row_f32,), float("nan"))
    i = torch.zeros(lay.row_i64, dtype=torch.int64)
    lay.pack(sd, f, i)
    back = lay.unpack(f, i)
    for name in sd:
        assert torch.equal(back[name], sd[name]), name
    # the native packer (the stager's) agrees
    f2 = torch.full((lay.row_f32,), float("nan"))
    i2 = torch.zeros(lay.row_i64, dtype=torch.int64)
    HostPacker(lay, "native").pack(sd, f2, i2)
    for name in sd:
        assert torch.equal(lay.unpack(f2, i2)[name], sd[name]), name


def test_from_state_dict_alignment_matches_from_shapes():
    spec = workloads.resnet(18)
    sd = {n: torch.zeros(s, dtype=torch.float32 if r == F32 else torch.int64) for n, s, r in spec}
    a = ArenaLayout.from_state_dict(sd, align="fedadp")
    b = ArenaLayout.from_shapes(spec, align="fedadp")
    assert [(e.name, e.offset) for e in a.entries] == [(e.name, e.offset) for e in b.entries]
    with pytest.raises(ValueError):
        ArenaLayout.from_shapes(spec, align="sideways")


def test_padding_mask_ignores_only_alignment_padding():
    """Two stagings of one model agree on the entries; their padding may hold different host bytes
    (AggregationRound._arrival_base_matches compares the arrival baseline with the round's outside it)."""
    from collections import OrderedDict

    from plato_amd.arena import same_f32_bits

    sd = OrderedDict([("w", torch.zeros(50)), ("n", torch.zeros(4, dtype=torch.int64)), ("b", torch.zeros(70)),
                      ("c", torch.zeros(33))])
    assert ArenaLayout.from_state_dict(sd).f32_padding("cpu") is None  # packed: nothing to mask
    lay = ArenaLayout.from_state_dict(sd, align="fedadp")
    pad = lay.f32_padding("cpu")
    assert int((~pad).sum()) == lay.n_f32_data and pad.numel() == lay.n_f32
    a = torch.randn(lay.n_f32)
    b = a.clone()
    b[pad] = 123.0
    assert same_f32_bits(a, b, pad) and not same_f32_bits(a, b, None)
    for name in ("w", "b", "c"):
        e = lay._by_name[name]
        for at in (e.offset, e.offset + e.numel - 1):
            c = b.clone()
            c[at] = -c[at] if c[at] != 0 else 1.0
            assert not same_f32_bits(a, c, pad)

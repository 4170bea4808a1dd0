"""QSGD inbound processor (host side): wire parsing, payload object, layout checks.

The wire format is the reference's (plato/processors/model_quantize_qsgd.py:130-139,
restated by oracle/qsgd.py and pinned there against the reference's own
dequantize processor through the qsgd_codec_* fixtures, tests/test_oracle.py).
"""

import pickle

import numpy as np
import pytest
import torch

from oracle import qsgd as Q
from plato_amd.arena import ArenaLayout, payload_codec
from plato_amd.processors.qsgd import Processor, QsgdPayload, parse_layer
from tests import golden_cases as G


def _wire(model="lenet5", seed=3, client=0):
    layout = ArenaLayout.from_shapes(G.model_spec(model))
    wire, cf, ci, mv = Q.client_wire(layout.entries, seed, client)
    return layout, wire, cf, ci, mv


def test_parse_layer_header():
    codes = np.arange(24, dtype=np.uint8)
    blob = Q.encode_layer(codes, np.float32(0.75), (2, 3, 4))
    max_v, shape, start, n = parse_layer(blob)
    assert (max_v, shape, start, n) == (0.75, (2, 3, 4), 16, 24)
    assert parse_layer(Q.encode_layer(np.array([200], np.uint8), 3.0, ()))[1:] == ((), 10, 1)
    with pytest.raises(ValueError):
        parse_layer(blob[:-1])          # truncated codes
    with pytest.raises(ValueError):
        parse_layer(blob[:8])           # truncated header


def test_processor_gathers_codes_in_arena_order():
    layout, wire, cf, ci, mv = _wire()
    payload = Processor(pin=False).process(wire)
    assert isinstance(payload, QsgdPayload) and payload_codec(payload) == "qsgd"
    assert list(payload) == layout.keys()
    layout.check_compatible(payload, "payload", "qsgd")
    hf = torch.empty(layout.row_f32, dtype=torch.uint8)
    hi = torch.empty(layout.row_i64, dtype=torch.uint8)
    layout.pack(payload, hf, hi)
    assert hf[: layout.n_f32].numpy().tobytes() == cf.tobytes()
    assert hi[: layout.n_i64].numpy().tobytes() == ci.tobytes()
    assert payload.max_v_array(layout.keys()).tobytes() == mv.tobytes()
    assert payload.level == 64


def test_payload_pickles_for_size_accounting():
    """servers/base.py:839-846 re-pickles payloads to log their size."""
    _, wire, *_ = _wire()
    payload = Processor(pin=False).process(wire)
    back = pickle.loads(pickle.dumps(payload))
    assert isinstance(back, QsgdPayload) and back.max_v == payload.max_v and back.shapes == payload.shapes
    assert all(torch.equal(back[n], payload[n]) for n in payload)


def test_layout_rejects_wrong_shapes():
    layout, wire, *_ = _wire()
    payload = Processor(pin=False).process(wire)
    name = layout.keys()[0]
    payload.shapes[name] = (1,) + tuple(payload.shapes[name])[1:] + (0,)
    with pytest.raises(ValueError):
        layout.check_compatible(payload, "payload", "qsgd")


def test_oracle_decode_matches_torch_ops_of_the_reference():
    """decode_layer == the reference's op sequence (int64 tensor * float / int), on all 256 codes."""
    codes = np.arange(256, dtype=np.uint8)
    for max_v in (np.float32(0.0371), np.float32(1e-30), np.float32(3.4e38)):
        blob = Q.encode_layer(codes, max_v, (256,))
        zeta = torch.tensor([c if c < 128 else -(c - 128) for c in range(256)])
        expected = (zeta * struct_f32(blob) / 63).numpy()
        assert Q.decode_layer(blob).tobytes() == expected.tobytes()


def struct_f32(blob):
    import struct

    return struct.unpack("!f", blob[0:4])[0]

"""TEST INFRASTRUCTURE ONLY — QSGD wire format and dequantization, restated.

Never imported by the product path.  Plato's QSGD processors
(plato/processors/model_quantize_qsgd.py:95-139 on the client,
plato/processors/model_dequantize_qsgd.py:34-60 on the server) send each
state_dict entry as

    !f max_v | !I numel | !h ndim | ndim x !h size | numel x 1 byte

(big-endian header; one byte per element: bit 7 = sign, bits 0-6 = |zeta|,
zeta in [-127, 127]) and dequantize with torch ops on an int64 tensor:
``zeta * max_v / (level - 1)``, i.e. in fp32 ``fp32(fp32(fp32(z) * m) / (level - 1))``.

The client's quantizer draws from ``random.seed()`` (OS entropy), so the
fixtures use synthetic codes from the counter generator (oracle/synth.py)
encoded in this format, and the reference's own dequantize processor decodes
them (tests/golden/make_golden.py).
"""

from __future__ import annotations

import struct

import numpy as np

from . import synth

LEVEL = 64  # the processors' default quantization_level


def encode_layer(codes: np.ndarray, max_v: float, shape) -> bytes:
    """One entry in the wire format of model_quantize_qsgd.py:130-139."""
    out = struct.pack("!f", float(max_v)) + struct.pack("!I", int(codes.size)) + struct.pack("!h", len(shape))
    for dim in shape:
        out += struct.pack("!h", int(dim))
    return out + np.ascontiguousarray(codes, dtype=np.uint8).tobytes()


def decode_layer(blob: bytes, level: int = LEVEL) -> np.ndarray:
    """model_dequantize_qsgd.py:34-60 restated with numpy (same fp32 roundings)."""
    max_v = struct.unpack("!f", blob[0:4])[0]
    numel = struct.unpack("!I", blob[4:8])[0]
    ndim = struct.unpack("!h", blob[8:10])[0]
    shape = [struct.unpack("!h", blob[10 + 2 * i:12 + 2 * i])[0] for i in range(ndim)]
    raw = np.frombuffer(blob, dtype=np.uint8, count=numel, offset=10 + 2 * ndim).astype(np.int64)
    zeta = np.where(raw >= 128, -(raw - 128), raw)
    with np.errstate(over="ignore"):  # torch overflows to inf the same way
        prod = np.multiply(zeta.astype(np.float32), np.float32(max_v), dtype=np.float32)
    return np.divide(prod, np.float32(level - 1), dtype=np.float32).reshape(shape)


def synth_codes(n: int, seed: int, stream: int) -> np.ndarray:
    """Synthetic code bytes (uniform over 0..255: every sign/magnitude, incl. -0 = 0x80)."""
    return synth.synth_i64(n, seed, stream, 256).astype(np.uint8)


def synth_max_v(n_entries: int, seed: int, client: int) -> np.ndarray:
    """Per-entry max_v of client ``client``: (1024 + r) * 2^-15, r in [0, 1024) (exact fp32)."""
    r = synth.synth_i64(n_entries, seed, 3000 + client, 1024)
    return ((1024 + r).astype(np.float32) * np.float32(2.0**-15)).astype(np.float32)


def client_wire(entries, seed: int, client: int):
    """(wire dict name -> bytes, codes_f32-region, codes_i64-region, max_v per entry) of one client."""
    n_f = sum(e.numel for e in entries if e.region == "f32")
    n_i = sum(e.numel for e in entries if e.region == "i64")
    cf = synth_codes(n_f, seed, 1000 + client)
    ci = synth_codes(n_i, seed, 2000 + client)
    mv = synth_max_v(len(entries), seed, client)
    wire = {}
    for e_i, e in enumerate(entries):
        src = cf if e.region == "f32" else ci
        wire[e.name] = encode_layer(src[e.offset:e.offset + e.numel], mv[e_i], e.shape)
    return wire, cf, ci, mv


def dequantize_regions(entries, cf, ci, mv, level: int = LEVEL):
    """Flat fp32 values of both regions (the int64 entries dequantize to fp32 too)."""
    out = []
    for region, codes in (("f32", cf), ("i64", ci)):
        vals = np.zeros(codes.size, dtype=np.float32)
        for e_i, e in enumerate(entries):
            if e.region != region:
                continue
            blob = encode_layer(codes[e.offset:e.offset + e.numel], mv[e_i], e.shape)
            vals[e.offset:e.offset + e.numel] = decode_layer(blob, level).reshape(-1)
        out.append(vals)
    return out[0], out[1]

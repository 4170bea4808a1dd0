"""TEST INFRASTRUCTURE ONLY — never imported by the product path (plato_amd/).

Bit-exact numpy restatement of the counter-based synthetic payload generator
that libplato_agg.so exposes as ``plato_agg_fill_synth_f32/_i64``
(include/plato_agg.h).  The golden fixtures under tests/golden/ were made by
feeding these inputs to the reference's own aggregation code
(tests/golden/make_golden.py), so the GPU tests can regenerate the same inputs
on the device and compare against the fixtures without shipping tensors.

    key    = splitmix64(seed ^ (stream * 0xD1B54A32D192ED03))
    h(e)   = splitmix64(key + e)                       (all mod 2^64)
    f32:   r = (int32)(h >> 40) - 2^23 ;  v = fp32(r) * 2^scale_log2  (exact)
           out = fp32(add + v)                         (one RNE fp32 add)
    i64:   out = add + (int64)(h % modulus)
"""

from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_STREAM = 0xD1B54A32D192ED03
_MASK = (1 << 64) - 1


def splitmix64_int(z: int) -> int:
    """Scalar (Python int) splitmix64."""
    z = (z + 0x9E3779B97F4A7C15) & _MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
    return z ^ (z >> 31)


def synth_key(seed: int, stream: int) -> int:
    return splitmix64_int((seed ^ ((stream * _STREAM) & _MASK)) & _MASK)


def _hashes(n: int, seed: int, stream: int, start: int = 0) -> np.ndarray:
    key = np.uint64(synth_key(seed, stream))
    with np.errstate(over="ignore"):
        z = np.arange(start, start + n, dtype=np.uint64) + key
        z = z + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def synth_f32(n: int, seed: int, stream: int, scale_log2: int, add: np.ndarray | None = None,
              start: int = 0) -> np.ndarray:
    h = _hashes(n, seed, stream, start)
    r = (h >> np.uint64(40)).astype(np.int64) - (1 << 23)
    v = r.astype(np.float32) * np.float32(2.0**scale_log2)  # exact: |r| < 2^24
    if add is None:
        return v + np.float32(0.0)
    assert add.dtype == np.float32
    return (add + v).astype(np.float32)


def synth_i64(n: int, seed: int, stream: int, modulus: int, add: np.ndarray | None = None,
              start: int = 0) -> np.ndarray:
    h = _hashes(n, seed, stream, start)
    v = (h % np.uint64(modulus)).astype(np.int64)
    if add is None:
        return v
    with np.errstate(over="ignore"):
        return (add.astype(np.int64) + v).astype(np.int64)


# Payload recipe used by the fixtures, the GPU tests and bench.py (SURVEY.md
# §8(d) C2): baseline b ~ +-0.0625 uniform grid (2^-27 steps), client
# x_i = b + noise (+-2^-7, 2^-30 steps); counters b in [0, 10^4], x_i = b + U{0..8}.
BASE_SCALE = -27
CLIENT_SCALE = -30
I64_BASE_MOD = 10001
I64_CLIENT_MOD = 9


def baseline_arena(n_f32: int, n_i64: int, seed: int):
    bf = synth_f32(n_f32, seed, 0, BASE_SCALE)
    bi = synth_i64(n_i64, seed, 0, I64_BASE_MOD)
    return bf, bi


def client_arena(bf: np.ndarray, bi: np.ndarray, seed: int, client: int):
    """Client ``client`` (0-based) of seed ``seed``: stream id = client + 1."""
    xf = synth_f32(bf.size, seed, client + 1, CLIENT_SCALE, add=bf)
    xi = synth_i64(bi.size, seed, client + 1, I64_CLIENT_MOD, add=bi)
    return xf, xi


def num_samples(k: int, seed: int, equal: bool = False) -> list[int]:
    """int(1000 * U(0.1, 2.0)) per client, from the same counter generator."""
    if equal:
        return [1000] * k
    h = _hashes(k, seed, 0xFFFF, 0)
    u = (h >> np.uint64(11)).astype(np.float64) * (2.0**-53)
    return [int(1000 * (0.1 + 1.9 * x)) for x in u]

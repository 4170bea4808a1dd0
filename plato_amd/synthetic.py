"""Device-side synthetic client payloads (bench.py, GPU tests, smoke).

BASELINE.json's configurations aggregate K client updates of a named model;
there is no network for real client payloads, so the engine generates them in
HBM with the counter-based generator of ``plato_agg_fill_synth_*`` (recipe in
include/plato_agg.h; SURVEY.md §8(d) C2 distributions):

* baseline fp32 entries: uniform grid in [-2^-4, 2^-4) (2^-27 steps),
* client i fp32 entries: baseline + uniform noise in [-2^-7, 2^-7) (2^-30 steps),
* int64 counters: baseline in [0, 10^4], client = baseline + U{0..8}.

The same recipe is restated in numpy by ``oracle/synth.py`` (test-side only),
which is how the golden fixtures pin these inputs.
"""

from __future__ import annotations

import torch

from . import _lib
from .engine import ClientSlab, DeviceArena

BASE_SCALE = -27
CLIENT_SCALE = -30
I64_BASE_MOD = 10001
I64_CLIENT_MOD = 9


def _splitmix64(z: int) -> int:
    mask = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & mask
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & mask
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & mask
    return z ^ (z >> 31)


def num_samples(k: int, seed: int, equal: bool = False) -> list[int]:
    """Synthetic ``report.num_samples`` per client: int(1000 * U(0.1, 2.0)).

    A Dirichlet-partition analogue (plato/samplers/dirichlet.py:47-60); same
    counter generator (stream 0xFFFF) as the payloads.
    """
    if equal:
        return [1000] * k
    mask = (1 << 64) - 1
    key = _splitmix64((seed ^ ((0xFFFF * 0xD1B54A32D192ED03) & mask)) & mask)
    out = []
    for c in range(k):
        u = (_splitmix64((key + c) & mask) >> 11) * (2.0**-53)
        out.append(int(1000 * (0.1 + 1.9 * u)))
    return out


def staleness(k: int, seed: int, bound: int = 10) -> list[int]:
    """Synthetic staleness in U{0..bound} per client (C4 async workloads)."""
    mask = (1 << 64) - 1
    key = _splitmix64((seed ^ ((0xFFFE * 0xD1B54A32D192ED03) & mask)) & mask)
    return [_splitmix64((key + c) & mask) % (bound + 1) for c in range(k)]


def _h(stream) -> int:
    return stream.cuda_stream


def fill_baseline(arena: DeviceArena, seed: int, stream=None) -> None:
    stream = stream or torch.cuda.current_stream(arena.f32.device)
    lay = arena.layout
    _lib.call("plato_agg_fill_synth_f32", arena.f32.data_ptr(), None, lay.n_f32, seed, 0,
              BASE_SCALE, _h(stream))
    if lay.n_i64:
        _lib.call("plato_agg_fill_synth_i64", arena.i64.data_ptr(), None, lay.n_i64, seed, 0,
                  I64_BASE_MOD, _h(stream))


def fill_clients(slab: ClientSlab, base: DeviceArena, seed: int, k: int, stream=None,
                 first_client: int = 0) -> None:
    """Rows 0..k-1 of ``slab`` = clients first_client..first_client+k-1 of ``seed``."""
    stream = stream or torch.cuda.current_stream(base.f32.device)
    lay = base.layout
    for r in range(k):
        c = first_client + r
        _lib.call("plato_agg_fill_synth_f32", slab.f32[r].data_ptr(), base.f32.data_ptr(), lay.n_f32,
                  seed, c + 1, CLIENT_SCALE, _h(stream))
        if lay.n_i64:
            _lib.call("plato_agg_fill_synth_i64", slab.i64[r].data_ptr(), base.i64.data_ptr(),
                      lay.n_i64, seed, c + 1, I64_CLIENT_MOD, _h(stream))


def fill_slices(base: DeviceArena, slab: ClientSlab | None, slices, n_i64: int, seed: int, k: int,
                stream=None) -> None:
    """Arenas holding SLICES of the one global model and client set of ``seed``.

    ``slices``: [(local offset, global first element, n)] of the fp32 region; the local
    ``base.f32[off:off+n]`` gets baseline elements ``first..first+n-1`` and client row r's
    the matching elements of client r (``plato_agg_fill_synth_*_at``), so the slices of
    several arenas — a bucket-sharded rank's pieces, a window of a parity check — are
    bit-identical to the same elements of :func:`fill_baseline` / :func:`fill_clients`
    on the whole model.  The first ``n_i64`` int64 entries are filled whole (they are
    never cut).
    """
    stream = stream or torch.cuda.current_stream(base.f32.device)
    h = _h(stream)
    b0, bi0 = base.f32.data_ptr(), base.i64.data_ptr()
    for off, first, n in slices:
        _lib.call("plato_agg_fill_synth_f32_at", b0 + off * 4, None, n, seed, 0, first, BASE_SCALE, h)
    if n_i64:
        _lib.call("plato_agg_fill_synth_i64_at", bi0, None, n_i64, seed, 0, 0, I64_BASE_MOD, h)
    if slab is None:
        return
    for r in range(k):
        rf, ri = slab.f32[r].data_ptr(), slab.i64[r].data_ptr()
        for off, first, n in slices:
            _lib.call("plato_agg_fill_synth_f32_at", rf + off * 4, b0 + off * 4, n, seed, r + 1, first,
                      CLIENT_SCALE, h)
        if n_i64:
            _lib.call("plato_agg_fill_synth_i64_at", ri, bi0, n_i64, seed, r + 1, 0, I64_CLIENT_MOD, h)

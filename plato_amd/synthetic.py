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

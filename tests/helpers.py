"""Shared test helpers: synthetic arenas on host (oracle side) and on device."""

from __future__ import annotations

import hashlib

import numpy as np

from oracle import synth


def host_inputs(n_f32: int, n_i64: int, seed: int, k: int):
    bf, bi = synth.baseline_arena(n_f32, n_i64, seed)
    xs_f, xs_i = [], []
    for c in range(k):
        xf, xi = synth.client_arena(bf, bi, seed, c)
        xs_f.append(xf)
        xs_i.append(xi)
    return bf, bi, xs_f, xs_i


def sha256(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.shape == b.shape and a.tobytes() == b.tobytes()


def first_mismatch(a: np.ndarray, b: np.ndarray):
    av = np.ascontiguousarray(a).view(np.uint32)
    bv = np.ascontiguousarray(b).view(np.uint32)
    idx = np.nonzero(av != bv)[0]
    if idx.size == 0:
        return None
    i = int(idx[0])
    return i, float(a[i]), float(b[i]), int(idx.size)

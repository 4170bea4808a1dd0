"""Per-client aggregation weights of Plato's FedAvg-family servers (host side).

Every FedAvg-family server in the reference multiplies client deltas by a
per-client Python number and sums them in ``self.updates`` order; only that
number differs between variants.  The engine takes the numbers as fp32
(``engine.fp32_weights``: torch rounds the Python double to the fp32 compute
type at the multiply), so reproducing each variant = computing the same
Python doubles as the reference, with the same expression order:

* FedAvg   ``n_i / N``                         plato/servers/fedavg.py:140,154
* FedBuff  ``1 / len(updates)``                examples/async/fedbuff/fedbuff_server.py:33,45
* Port     ``n_i/N * ((sim+1)/2*sw + f(s)*tw)`` normalised by the sum
                                               examples/async/port/port_server.py:57-103,135-144
* Pisces   ``(n_i/N)`` then ``* 1/(mean(s[-5:])+1)**a`` as a second fp32 multiply
                                               examples/client_selection/pisces/pisces_server.py:83-95,97-100
* FedAsync mixing ``m * staleness_fn(s)``      examples/async/fedasync/fedasync_server.py:67-118
"""

from __future__ import annotations

from typing import Sequence

import numpy as np


def fedavg(num_samples: Sequence[int]) -> list[float]:
    total = sum(num_samples)
    return [n / total for n in num_samples]


def fedbuff(k: int) -> list[float]:
    return [1 / k for _ in range(k)]


def port_staleness_factor(staleness: int, staleness_bound: float = 10) -> float:
    return staleness_bound / (staleness + staleness_bound)


class _F32:
    """A 0-dim fp32 torch tensor's scalar arithmetic, restated with numpy float32.

    Port's cosine similarity is a 0-dim fp32 tensor (F.cosine_similarity), so
    every weight expression it enters follows tensor semantics: Python numbers
    are cast to fp32 at each op, ``number / tensor`` is
    ``tensor.reciprocal() * number`` (torch/_tensor.py ``__rdiv__``).
    """

    __slots__ = ("v",)

    def __init__(self, v):
        self.v = np.float32(v)

    @staticmethod
    def _f(x):
        return x.v if isinstance(x, _F32) else np.float32(x)

    def __add__(self, o):
        return _F32(self.v + self._f(o))

    __radd__ = __add__

    def __mul__(self, o):
        return _F32(self.v * self._f(o))

    __rmul__ = __mul__

    def __truediv__(self, o):
        return _F32(self.v / self._f(o))

    def __rtruediv__(self, o):
        return _F32((np.float32(1) / self.v) * self._f(o))


def port(num_samples: Sequence[int], staleness: Sequence[int], similarities=None,
         similarity_weight: float = 1, staleness_weight: float = 1,
         staleness_bound: float = 10) -> list[float]:
    """Port's normalised weights, evaluated with the reference's expression order.

    ``similarities[i]`` is the Python float 1.0 when the reference skips the
    cosine similarity, else the fp32 value of F.cosine_similarity (pass a
    ``numpy.float32``): then that client's weight and every weight normalised by
    the (now tensor-valued) sum follow fp32 tensor arithmetic, as in the reference.
    """
    total = sum(num_samples)
    raw = []
    for i, n in enumerate(num_samples):
        sim = 1.0 if similarities is None else similarities[i]
        if isinstance(sim, np.floating) and sim.dtype == np.float32:
            sim = _F32(sim)
        factor = port_staleness_factor(staleness[i], staleness_bound)
        raw.append(n / total * ((sim + 1) / 2 * similarity_weight + factor * staleness_weight))
    denom = sum(raw)
    out = []
    for r in raw:
        w = r / denom
        out.append(float(w.v) if isinstance(w, _F32) else w)
    return out


def pisces_staleness_factor(history: Sequence[int], exponent: float) -> float:
    """``1.0 / pow(np.mean(history[-5:]) + 1, a)`` with numpy's mean (float64)."""
    return 1.0 / pow(np.mean(list(history)[-5:]) + 1, exponent)


def pisces(num_samples: Sequence[int], staleness_histories: Sequence[Sequence[int]],
           exponent: float) -> tuple[list[float], list[float]]:
    """(first scalars n_i/N, second scalars staleness factors) — two fp32 multiplies."""
    total = sum(num_samples)
    first = [n / total for n in num_samples]
    second = [float(pisces_staleness_factor(h, exponent)) for h in staleness_histories]
    return first, second


def fedasync_mixing(mixing: float, staleness: int, func: str = "constant", a: float = 1,
                    b: float = 0) -> float:
    """Adaptive FedAsync mixing: ``mixing * s(staleness)``."""
    func = func.lower()
    if func == "constant":
        factor = 1
    elif func == "polynomial":
        factor = (staleness + 1) ** -a
    elif func == "hinge":
        factor = 1 if staleness <= b else 1 / (a * (staleness - b) + 1)
    else:
        raise ValueError(f"unknown staleness weighting function {func!r}")
    return mixing * factor


# --------------------------------------------------------------------------
# Per-entry variants: the numbers depend on reductions over the deltas, which
# the device computes (plato_agg_entry_stats, fp64, fixed order); the host
# finishes them with the reference's own scalar expressions.
# --------------------------------------------------------------------------
def fedatt_attention(norms: np.ndarray) -> np.ndarray:
    """FedAtt attention ``[entry, client]`` from the fp32 norms ``[entry, client]``.

    examples/server_aggregation/fedatt/fedatt_algorithm.py:32-42:
    ``atts[name][i] = torch.linalg.norm(-delta)`` into an fp32 tensor, then
    ``F.softmax(atts[name], dim=0)`` per entry — the same torch op here, one
    softmax over the clients of each entry.
    """
    import torch

    t = torch.from_numpy(np.ascontiguousarray(norms, dtype=np.float32))
    return torch.softmax(t, dim=1).numpy()


def fedadp_angles_from_dots(inner: Sequence, g_sq, l_sq: Sequence) -> list:
    """fedadp_server.py:94-99 from the reference's own float32 reductions, computed on the device.

    ``inner[k] = np.inner(g, loc_k)``, ``g_sq = g.dot(g)``, ``l_sq[k] = loc_k.dot(loc_k)`` are the
    float32 values numpy's BLAS produces (``plato_agg_flat_dots``, bit-exact);
    ``np.linalg.norm`` is ``sqrt`` of such a dot in float32, and the rest is
    the reference's numpy scalar code on those float32 values.
    """
    g_norm = np.sqrt(np.float32(g_sq))
    angles = []
    for k in range(len(inner)):
        norms = g_norm * np.sqrt(np.float32(l_sq[k]))
        angles.append(np.arccos(np.clip(np.float32(inner[k]) / norms, -1.0, 1.0)))
    return angles


def fedadp_contributions(angles, selected_clients, local_angles: dict, current_round: int,
                         alpha: float = 5) -> list:
    """fedadp_server.py:101-120: smoothed angles (updated in ``local_angles``) -> contributions."""
    import math

    contribs = [None] * len(angles)
    for i, angle in enumerate(angles):
        client_id = selected_clients[i]
        if client_id not in local_angles:
            local_angles[client_id] = angle
        local_angles[client_id] = ((current_round - 1) / current_round) * local_angles[client_id] + (
            1 / current_round) * angle
        contribs[i] = alpha * (1 - math.exp(-math.exp(-alpha * (local_angles[client_id] - 1))))
    return contribs


def fedadp_weighting(contribs, num_samples) -> list:
    """fedadp_server.py:70-84: ``n_i * exp(c_i) / sum_j n_j * exp(c_j)``."""
    import math

    total_weight = 0.0
    for i, contrib in enumerate(contribs):
        total_weight += num_samples[i] * math.exp(contrib)
    return [(num_samples[i] * math.exp(contrib)) / total_weight for i, contrib in enumerate(contribs)]


def polaris_delta_norms(dd: np.ndarray, names: Sequence[str]) -> list:
    """Per client ``sqrt(sum over 'conv' layers of np.sum(np.square(delta)))``.

    examples/client_selection/polaris/polaris_server.py:76-89: each layer's
    ``np.sum`` is a float32 scalar (``dd[k, e]``, from the device in numpy's
    order) and they are added in float32 (``0 + np.float32``), then
    ``np.sqrt`` in float32.
    """
    conv = [e for e, name in enumerate(names) if "conv" in name]
    out = []
    for k in range(dd.shape[0]):
        squared = 0
        for e in conv:
            squared += np.float32(dd[k, e])
        out.append(np.sqrt(squared))
    return out

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

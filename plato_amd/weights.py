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


def port(num_samples: Sequence[int], staleness: Sequence[int], similarities=None,
         similarity_weight: float = 1, staleness_weight: float = 1,
         staleness_bound: float = 10) -> list[float]:
    """Port's normalised weights; ``similarities`` default to 1.0 (no stale model on disk)."""
    total = sum(num_samples)
    raw = []
    for i, n in enumerate(num_samples):
        sim = 1.0 if similarities is None else similarities[i]
        factor = port_staleness_factor(staleness[i], staleness_bound)
        raw.append(n / total * ((sim + 1) / 2 * similarity_weight + factor * staleness_weight))
    return [r / sum(raw) for r in raw]


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

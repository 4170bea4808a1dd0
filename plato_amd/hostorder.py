"""Run-time guard for the host reduction orders that FedAdp's and Port's parity rests on.

The reference forms two of its weights with float32 reductions whose order is
chosen by the libraries on the server host, not by Plato:

* FedAdp's ``np.inner`` / ``np.linalg.norm`` of the flattened gradients
  (examples/server_aggregation/fedadp/fedadp_server.py:95-99) are ``cblas_sdot``
  of numpy's bundled OpenBLAS; on AVX-512 hosts that is ``sdot_k_SKYLAKEX``,
  whose 64-chain order the device kernels restate (``csrc/fedadp.hip``).
* Port's ``F.cosine_similarity`` (examples/async/port/port_server.py:50) is
  ATen's ``vector_norm`` and a two-pass cascade sum over
  ``min(threads, ceil(n / 32768))`` OpenMP chunks, which the device restates for
  a given thread count (``csrc/port.hip``, ``csrc/flat.hip``).

On a host whose BLAS kernel or ATen vector width differs, the reference itself
computes other float32 bits, and the device result would differ in the last
bits from that host's reference.  So before the first FedAdp / Port round on a
device a small probe model is aggregated through the SAME engine calls the
rounds make (``AggregationRound.fedadp_dots`` -> ``plato_agg_fedadp_dots``;
``AggregationRound.model_similarities`` -> ``plato_agg_port_norms`` +
``plato_agg_scale_by_norm`` + ``plato_agg_torch_cosine_sum_scaled``) and compared
bit for bit with the reference's numpy / torch calls on this host.  The probe's
arena is out of name order, carries an int64 counter and takes a non-unit lr,
so the segment map, the division and the int64 path are all exercised.

A mismatch is logged once as a warning naming the host's BLAS kernel, ATen CPU
capability and thread count (the aggregation goes on: only the last bits of the
weights can differ); ``strict=True`` raises :class:`HostOrderError` instead.
This is a check of the host, not a CPU path: the aggregation always runs on the
GPU.
"""

from __future__ import annotations

import logging
import threading
from collections import OrderedDict

import numpy as np
import torch

PROBE_N = (1 << 20) + 77  # ragged sdot tails (n mod 64 = 13, n mod 32 = 13)
PROBE_SEED = 20241017
GRAIN = 32768  # ATen's reduction grain: a reduction of n elements runs in min(threads, ceil(n / GRAIN)) chunks
PROBE_LR = 0.01


class HostOrderError(RuntimeError):
    """This host's numpy / torch reduction order is not the one the device reproduces."""


_lock = threading.Lock()
_checked: dict = {}  # key -> True (orders agree) / False (mismatch already reported)


def probe_size(threads: int = 1) -> int:
    """Probe length: at least PROBE_N, and long enough that ATen splits the sum over all ``threads``."""
    return max(PROBE_N, int(threads) * GRAIN + 77)


def probe_vectors(n: int = PROBE_N, seed: int = PROBE_SEED) -> tuple[np.ndarray, np.ndarray]:
    """Two float32 vectors with gradient-like spread (magnitudes over many binades)."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * np.exp2(rng.integers(-12, 4, n))).astype(np.float32)
    y = (rng.standard_normal(n) * np.exp2(rng.integers(-12, 4, n))).astype(np.float32)
    return x, y


def probe_models(n: int = PROBE_N, seed: int = PROBE_SEED) -> dict:
    """Baseline, client, global-gradient and previous models of a 3-entry probe (n values in all).

    State-dict order ``b.weight`` (fp32), ``b.num_batches_tracked`` (int64),
    ``a.weight`` (fp32): name order puts ``a.weight`` first, so the flattening
    reorders the arena, the counter sits between the fp32 entries and every
    entry after the first is divided by ``-lr`` (process_grad,
    fedadp_server.py:122-133).
    """
    n1 = n // 3 + 5
    n2 = n - n1 - 1
    x, y = probe_vectors(n, seed)
    rng = np.random.default_rng(seed + 1)
    b = (rng.standard_normal(n) * np.exp2(rng.integers(-10, 2, n))).astype(np.float32)
    prev = (b + y * np.float32(0.25)).astype(np.float32)

    def model(v, counter):
        return OrderedDict([("b.weight", torch.from_numpy(v[:n1].copy())),
                            ("b.num_batches_tracked", torch.tensor(counter, dtype=torch.int64)),
                            ("a.weight", torch.from_numpy(v[n1 + 1:].copy()).reshape(n2))])

    return {"baseline": model(b, 1_000_003), "client": model((b + x).astype(np.float32), 1_000_103),
            "previous": model(prev, 999_983),
            "grads": OrderedDict([("b.weight", torch.from_numpy(y[:n1].copy())),
                                  ("b.num_batches_tracked", torch.tensor(float(y[n1]), dtype=torch.float32)),
                                  ("a.weight", torch.from_numpy(y[n1 + 1:].copy()))])}


def host_description() -> str:
    """The host facts the orders depend on, for error messages and logs."""
    blas = "unknown"
    try:
        import threadpoolctl

        for info in threadpoolctl.threadpool_info():
            if info.get("user_api") == "blas":
                blas = f"{info.get('internal_api')} {info.get('version')} kernel {info.get('architecture')}"
                break
    except Exception:  # threadpoolctl absent or failing: the bit comparison still decides
        pass
    return (f"numpy BLAS: {blas}; ATen CPU capability: {torch.backends.cpu.get_cpu_capability()}; "
            f"torch threads: {torch.get_num_threads()}")


# ------------------------------------------------------------------ host halves
def _process_grad(grads: dict, lr: float) -> np.ndarray:
    """fedadp_server.py:122-133: entries by name.lower(), every one after the first as -g / lr, appended."""
    vals = list(dict(sorted(grads.items(), key=lambda kv: kv[0].lower())).values())
    flat = vals[0]
    for g in vals[1:]:
        flat = np.append(flat, -g / lr)
    return np.asarray(flat)


def host_fedadp_values(models: dict, lr: float) -> np.ndarray:
    """``np.inner(g, loc)``, ``loc.dot(loc)``, ``g.dot(g)`` as this host's numpy forms them (fedadp_server.py:91-99)."""
    base, client = models["baseline"], models["client"]
    g = _process_grad(models["grads"], lr)
    loc = _process_grad(OrderedDict((k, client[k] - base[k]) for k in base), lr)
    return np.asarray([np.inner(g, loc), loc.dot(loc), g.dot(g)], dtype=np.float32)


def host_port_value(models: dict, threads: int) -> np.float32:
    """``F.cosine_similarity(current - previous, deltas, dim=0)`` at ``threads`` threads (port_server.py:36-50)."""
    import torch.nn.functional as F

    base, prev, client = models["baseline"], models["previous"], models["client"]
    current = torch.cat([w.view(-1) for w in base.values()])
    previous = torch.cat([w.view(-1) for w in prev.values()])
    deltas = torch.cat([(client[k] - base[k]).view(-1) for k in base])
    saved = torch.get_num_threads()
    try:
        if threads != saved:
            torch.set_num_threads(threads)
        return np.float32(F.cosine_similarity(current - previous, deltas, dim=0).item())
    finally:
        if torch.get_num_threads() != saved:
            torch.set_num_threads(saved)


# ---------------------------------------------------------------- device halves
def _probe_round(device, models: dict, align: str | None = None, port_variant: int | None = None,
                 deltas: bool = False):
    """A one-client round of the probe model on a private engine (the server's engine keeps its layout).

    ``align`` / ``port_variant`` / ``deltas``: the server engine's arena alignment, Port kernel shape and
    delta arenas, so the probe takes the same descriptor / offset path and the same kernel as the rounds
    (FedAdp's servers run on aligned delta arenas: the dot kernel's no-baseline form)."""
    from .engine import FedAvgEngine

    eng = FedAvgEngine(device)
    eng.layout_align = align
    eng.port_variant = port_variant
    eng.delta_arenas = deltas
    rnd = eng.begin(models["baseline"], 1)
    rnd.put_baseline(models["baseline"])
    rnd.put_client(0, models["client"])
    return rnd


def device_fedadp_values(device, models: dict, lr: float, align: str | None = None,
                         deltas: bool = False) -> np.ndarray:
    """The same three dots through ``AggregationRound.fedadp_dots`` (the product's ``plato_agg_fedadp_dots``)."""
    from .arena import F32

    rnd = _probe_round(device, models, align, deltas=deltas)
    lay = rnd.layout
    gf = torch.zeros(lay.row_f32, dtype=torch.float32)
    gi = torch.zeros(max(1, lay.row_i64), dtype=torch.float32)
    for e in lay.entries:
        v = models["grads"][e.name].reshape(-1).to(torch.float32)
        (gf if e.region == F32 else gi)[e.offset:e.offset + e.numel] = v
    grads = (gf.to(rnd.engine.device), gi.to(rnd.engine.device))
    inner, g_sq, l_sq = rnd.fedadp_dots(grads, [0], lr)
    return np.asarray([inner[0], l_sq[0], g_sq], dtype=np.float32)


def device_port_value(device, models: dict, threads: int, align: str | None = None,
                      port_variant: int | None = None) -> np.float32:
    """The cosine through ``AggregationRound.model_similarities`` (port_norms + scale_by_norm + cosine sums)."""
    rnd = _probe_round(device, models, align, port_variant)
    return np.float32(rnd.model_similarities(models["previous"], [0], threads=threads)[0])


# ------------------------------------------------------------------- the guards
def _report(key, ok: bool, msg: str, strict: bool) -> bool:
    if not ok:
        if strict:
            raise HostOrderError(msg)
        logging.warning("[plato_amd] %s Continuing (host_order_check='strict' would refuse).", msg)
    _checked[key] = ok
    return ok


def check_fedadp(device, lr: float = PROBE_LR, strict: bool = False, align: str | None = None,
                 deltas: bool = False) -> bool:
    """True if this host's numpy dots equal the device's bit for bit (checked once per device, lr, alignment
    and arena form).

    ``align`` / ``deltas``: the server engine's arena alignment and delta arenas (FedAdp servers use
    "fedadp" and deltas), so the probe runs the kernel the rounds run.  A mismatch is logged once
    (``strict``: raises :class:`HostOrderError`).
    """
    key = ("fedadp", str(device), float(lr), align, bool(deltas))
    with _lock:
        if key in _checked and (_checked[key] or not strict):
            return _checked[key]
        models = probe_models(PROBE_N)
        want = host_fedadp_values(models, lr)
        got = device_fedadp_values(device, models, lr, align, deltas)
        msg = ("FedAdp: this host's numpy float32 dot order differs from the one the device reproduces "
               f"(OpenBLAS sdot_k_SKYLAKEX); probe np.inner/dot = {want.tolist()}, device {got.tolist()}. "
               f"{host_description()}. The reference's FedAdp weights on this host would differ in the last bits.")
        return _report(key, want.tobytes() == got.tobytes(), msg, strict)


def check_port(device, threads: int, strict: bool = False, align: str | None = None,
               port_variant: int | None = None) -> bool:
    """True if F.cosine_similarity at ``threads`` equals the device's bit for bit (checked once per device and count).

    The probe is long enough (:func:`probe_size`) that ATen splits its sum over all
    ``threads`` chunks, as it does for a real model.  A mismatch is logged once
    (``strict``: raises :class:`HostOrderError`).
    """
    key = ("port", str(device), int(threads), align, port_variant)
    with _lock:
        if key in _checked and (_checked[key] or not strict):
            return _checked[key]
        models = probe_models(probe_size(threads))
        want = host_port_value(models, threads)
        got = device_port_value(device, models, threads, align, port_variant)
        msg = (f"Port: this host's F.cosine_similarity order at {threads} threads differs from the one the "
               f"device reproduces (ATen vector_norm + cascade sum); probe {float(want)!r}, device {float(got)!r}. "
               f"{host_description()}. The reference's Port similarities on this host would differ in the last bits.")
        return _report(key, want.tobytes() == got.tobytes(), msg, strict)


def mode(setting) -> str | None:
    """A server's ``host_order_check`` as "warn" / "strict" / None (off); True means "strict"."""
    if setting is None or setting is False or setting == "off":
        return None
    if setting is True or setting == "strict":
        return "strict"
    if setting == "warn":
        return "warn"
    raise ValueError(f"host_order_check must be 'warn', 'strict' or False, got {setting!r}")

"""Run-time guard for the host reduction orders that FedAdp's and Port's parity rests on.

The reference forms two of its weights with float32 reductions whose order is
chosen by the libraries on the server host, not by Plato:

* FedAdp's ``np.inner`` / ``np.linalg.norm`` of the flattened gradients
  (examples/server_aggregation/fedadp/fedadp_server.py:95-99) are ``cblas_sdot``
  of numpy's bundled OpenBLAS; on AVX-512 hosts that is ``sdot_k_SKYLAKEX``,
  whose 64-chain order the device kernels restate (``csrc/flat.hip``).
* Port's ``F.cosine_similarity`` (examples/async/port/port_server.py:50) is
  ATen's ``vector_norm`` and a two-pass cascade sum over
  ``torch.get_num_threads()`` OpenMP chunks, which the device restates for a
  given thread count.

On a host whose BLAS kernel or ATen vector width differs, the reference itself
computes other float32 bits, and the device result would silently differ from
that host's reference.  So before the first FedAdp / Port round on an engine the
device reductions are run on a fixed probe and compared bit for bit with the
same numpy / torch calls on this host; a mismatch raises :class:`HostOrderError`
naming the host's BLAS kernel, ATen CPU capability and thread count.  This is a
check of the host, not a CPU path: the aggregation itself always runs on the GPU.
"""

from __future__ import annotations

import threading

import numpy as np
import torch

from . import _lib

PROBE_N = (1 << 20) + 77  # > 16 OpenMP chunks of ATen's 32,768-element grain; ragged sdot tails
PROBE_SEED = 20241017


class HostOrderError(RuntimeError):
    """This host's numpy / torch reduction order is not the one the device reproduces."""


_lock = threading.Lock()
_checked: dict = {}


def probe_vectors(n: int = PROBE_N, seed: int = PROBE_SEED) -> tuple[np.ndarray, np.ndarray]:
    """Two float32 vectors with gradient-like spread (magnitudes over many binades)."""
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * np.exp2(rng.integers(-12, 4, n))).astype(np.float32)
    y = (rng.standard_normal(n) * np.exp2(rng.integers(-12, 4, n))).astype(np.float32)
    return x, y


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
def host_fedadp_values(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """``np.inner(x, y)``, ``y.dot(y)``, ``x.dot(x)`` as this host's numpy forms them (fedadp_server.py:95-99)."""
    return np.asarray([np.inner(x, y), y.dot(y), x.dot(x)], dtype=np.float32)


def host_port_value(a: np.ndarray, b: np.ndarray, threads: int) -> np.float32:
    """``F.cosine_similarity(a, b, dim=0)`` at ``threads`` OpenMP threads (port_server.py:50)."""
    import torch.nn.functional as F

    saved = torch.get_num_threads()
    try:
        if threads != saved:
            torch.set_num_threads(threads)
        return np.float32(F.cosine_similarity(torch.from_numpy(a), torch.from_numpy(b), dim=0).item())
    finally:
        if torch.get_num_threads() != saved:
            torch.set_num_threads(saved)


# ---------------------------------------------------------------- device halves
def _rows(device, *vectors) -> tuple[torch.Tensor, int]:
    n = vectors[0].size
    stride = -(-n // 64) * 64
    host = torch.zeros((len(vectors), stride), dtype=torch.float32)
    for r, v in enumerate(vectors):
        host[r, :n] = torch.from_numpy(v)
    return host.to(device), stride


def device_fedadp_values(device, x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """The same three dots by the device's sdot order (``plato_agg_sdot_shared``, x shared, x.x folded in)."""
    dev = torch.device(device)
    rows, stride = _rows(dev, x, y)
    ys = torch.tensor([rows.data_ptr() + stride * 4], dtype=torch.int64, device=dev)
    ws = torch.empty(_lib.lib().plato_agg_sdot_shared_workspace(1, 1) // 4, dtype=torch.float32, device=dev)
    xy = torch.empty(2, dtype=torch.float32, device=dev)
    yy = torch.empty(2, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    _lib.call("plato_agg_sdot_shared", rows.data_ptr(), ys.data_ptr(), 1, x.size, 1, ws.data_ptr(), xy.data_ptr(),
              yy.data_ptr(), stream.cuda_stream)
    xy_h, yy_h = xy.cpu().numpy(), yy.cpu().numpy()
    return np.asarray([xy_h[0], yy_h[0], xy_h[1]], dtype=np.float32)


def device_port_value(device, a: np.ndarray, b: np.ndarray, threads: int, eps: float = 1e-8) -> np.float32:
    """The cosine by the device's torch order (``plato_agg_entry_norms_f32`` + ``plato_agg_torch_cosine_sum``)."""
    dev = torch.device(device)
    rows, stride = _rows(dev, a, b)
    n = a.size
    tab = torch.tensor([rows.data_ptr(), rows.data_ptr() + stride * 4], dtype=torch.int64, device=dev)
    chunk = torch.from_numpy(np.asarray([[0, 0, n, 0]], dtype=np.uint32).view(np.int32)).to(dev)
    norms = torch.empty(2, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream
    _lib.call("plato_agg_entry_norms_f32", tab.data_ptr(), None, 2, None, None, chunk.data_ptr(), 1, None, 0, 1,
              stride, 0, norms.data_ptr(), h)
    lib = _lib.lib()
    ws = torch.empty(max(1, lib.plato_agg_torch_cosine_workspace(1, threads) // 4), dtype=torch.float32, device=dev)
    out = torch.empty(1, dtype=torch.float32, device=dev)
    _lib.call("plato_agg_torch_cosine_sum", rows.data_ptr(), tab.data_ptr() + 8, 1, n, norms.data_ptr(),
              norms.data_ptr() + 4, float(eps), threads, ws.data_ptr(), out.data_ptr(), h)
    return np.float32(out.cpu().numpy()[0])


# ------------------------------------------------------------------- the guards
def check_fedadp(device) -> None:
    """Raise :class:`HostOrderError` unless this host's numpy dots equal the device's, bit for bit."""
    key = ("fedadp", str(device))
    with _lock:
        if _checked.get(key):
            return
        x, y = probe_vectors()
        want = host_fedadp_values(x, y)
        got = device_fedadp_values(device, x, y)
        if want.tobytes() != got.tobytes():
            raise HostOrderError(
                "FedAdp: this host's numpy float32 dot order differs from the one the device reproduces "
                f"(OpenBLAS sdot_k_SKYLAKEX); probe np.inner/dot = {want.tolist()}, device {got.tolist()}. "
                f"{host_description()}. The reference's FedAdp weights on this host would differ in the last bits.")
        _checked[key] = True


def check_port(device, threads: int) -> None:
    """Raise :class:`HostOrderError` unless F.cosine_similarity at ``threads`` equals the device's, bit for bit."""
    key = ("port", str(device), int(threads))
    with _lock:
        if _checked.get(key):
            return
        a, b = probe_vectors()
        want = host_port_value(a, b, threads)
        got = device_port_value(device, a, b, threads)
        if want.tobytes() != got.tobytes():
            raise HostOrderError(
                f"Port: this host's F.cosine_similarity order at {threads} threads differs from the one the "
                f"device reproduces (ATen vector_norm + cascade sum); probe {float(want)!r}, device {float(got)!r}. "
                f"{host_description()}. The reference's Port similarities on this host would differ in the last bits.")
        _checked[key] = True

"""The reduction-order guard on the GPU box: the probe passes here through the product's own
kernels, and a host whose numpy / torch order differed is reported (warn) or refused (strict)."""

import logging

import numpy as np
import pytest

from plato_amd import _lib
from plato_amd import hostorder as H

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _record_calls(monkeypatch):
    seen = []
    real = _lib.call

    def rec(name, *args):
        seen.append(name)
        return real(name, *args)

    monkeypatch.setattr(_lib, "call", rec)
    return seen


@pytest.mark.parametrize("deltas", [False, True])
@pytest.mark.parametrize("align", [None, "fedadp"])
@pytest.mark.parametrize("lr", [0.01, 0.3])
def test_fedadp_probe_passes_through_the_product_kernel(monkeypatch, lr, align, deltas):
    """Also on the aligned delta arenas FedAdp's servers use (the probe takes the server engine's alignment and
    arena form, so it runs the dot kernel the rounds run: with deltas, its no-baseline form)."""
    H._checked.clear()
    seen = _record_calls(monkeypatch)
    assert H.check_fedadp(DEV, lr, strict=True, align=align, deltas=deltas)
    if deltas:
        assert "plato_agg_compute_deltas" in seen  # the probe's client row was staged as its delta
    # the round's own calls (engine.AggregationRound.fedadp_dots), not a stand-in kernel
    assert "plato_agg_fedadp_dots_ex" in seen and "plato_agg_sdot_shared" not in seen


@pytest.mark.parametrize("threads", [1, 8, 16, 64])
def test_port_probe_passes_through_the_product_kernels(monkeypatch, threads):
    H._checked.clear()
    seen = _record_calls(monkeypatch)
    assert H.check_port(DEV, threads, strict=True)
    for name in ("plato_agg_port_norms", "plato_agg_scale_by_norm", "plato_agg_torch_cosine_sum_scaled"):
        assert name in seen
    assert "plato_agg_entry_norms_f32" not in seen


def test_a_different_host_order_is_reported_or_refused(monkeypatch, caplog):
    H._checked.clear()

    def other_blas(models, lr):  # a host whose dot rounds differently in the last bit
        v = H._process_grad(models["grads"], lr)
        return np.nextafter(np.asarray([1.0, 2.0, v.dot(v)], dtype=np.float32), np.float32(np.inf))

    monkeypatch.setattr(H, "host_fedadp_values", other_blas)
    with caplog.at_level(logging.WARNING):
        assert H.check_fedadp(DEV) is False  # default: warn once, go on
    assert "numpy BLAS" in caplog.text
    with pytest.raises(H.HostOrderError, match="numpy BLAS"):
        H.check_fedadp(DEV, strict=True)
    monkeypatch.setattr(H, "host_port_value", lambda models, t: np.float32(0.5))
    with pytest.raises(H.HostOrderError, match="threads"):
        H.check_port(DEV, 4, strict=True)
    assert H.check_port(DEV, 2) is False
    H._checked.clear()

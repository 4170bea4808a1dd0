"""The reduction-order guard on the GPU box: the probe passes here, and a host whose
numpy / torch order differed would be refused, not silently diverge."""

import numpy as np
import pytest

from plato_amd import hostorder as H

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_fedadp_probe_passes_on_this_host():
    H._checked.clear()
    H.check_fedadp(DEV)


@pytest.mark.parametrize("threads", [1, 8, 16])
def test_port_probe_passes_on_this_host(threads):
    H._checked.clear()
    H.check_port(DEV, threads)


def test_a_different_host_order_is_refused(monkeypatch):
    H._checked.clear()

    def other_blas(x, y):  # a host whose dot rounds differently in the last bit
        v = np.asarray([np.inner(x, y), y.dot(y), x.dot(x)], dtype=np.float32)
        return np.nextafter(v, np.float32(np.inf))

    monkeypatch.setattr(H, "host_fedadp_values", other_blas)
    with pytest.raises(H.HostOrderError, match="numpy BLAS"):
        H.check_fedadp(DEV)
    monkeypatch.setattr(H, "host_port_value", lambda a, b, t: np.float32(0.5))
    with pytest.raises(H.HostOrderError, match="threads"):
        H.check_port(DEV, 4)
    H._checked.clear()

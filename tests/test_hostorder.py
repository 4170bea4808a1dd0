"""The host half of the reduction-order guard (plato_amd.hostorder), on the CPU.

The probe's numpy / torch values on this host must equal the C restatement of
the orders the device runs (oracle/reductions.c): that is what makes the guard's
GPU comparison (tests/test_hostorder_gpu.py) a statement about the host.
"""

import numpy as np
import pytest

from oracle import reductions as R
from plato_amd import hostorder as H


def _skx():
    try:
        import threadpoolctl

        return any(i.get("architecture") in ("SkylakeX", "Cooperlake", "SapphireRapids")
                   for i in threadpoolctl.threadpool_info() if i.get("user_api") == "blas")
    except Exception:
        return False


@pytest.mark.skipif(not _skx(), reason="numpy's OpenBLAS is not the SkylakeX kernel on this host")
def test_probe_dots_follow_the_restated_sdot_order():
    x, y = H.probe_vectors()
    got = H.host_fedadp_values(x, y)
    want = np.asarray([R.sdot(x, y), R.sdot(y, y), R.sdot(x, x)], dtype=np.float32)
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_probe_cosine_follows_the_restated_torch_order(threads):
    a, b = H.probe_vectors()
    assert H.host_port_value(a, b, threads).tobytes() == R.torch_cosine(a, b, threads).tobytes()


def test_probe_is_fixed_and_describes_the_host():
    x1, y1 = H.probe_vectors()
    x2, y2 = H.probe_vectors()
    assert x1.tobytes() == x2.tobytes() and y1.tobytes() == y2.tobytes()
    assert x1.size == H.PROBE_N and x1.dtype == np.float32
    desc = H.host_description()
    assert "ATen CPU capability" in desc and "torch threads" in desc

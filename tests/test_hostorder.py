"""The host half of the reduction-order guard (plato_amd.hostorder), on the CPU.

The probe's numpy / torch values on this host must equal the C restatement of
the orders the device runs (oracle/reductions.c): that is what makes the guard's
GPU comparison (tests/test_hostorder_gpu.py) a statement about the host.
"""

import math

import numpy as np
import pytest
import torch

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
    models = H.probe_models()
    lr = 0.05
    got = H.host_fedadp_values(models, lr)
    g = H._process_grad(models["grads"], lr)
    loc = H._process_grad({k: models["client"][k] - models["baseline"][k] for k in models["baseline"]}, lr)
    assert g.dtype == np.float32 and loc.dtype == np.float32 and loc.size == H.PROBE_N
    want = np.asarray([R.sdot(g, loc), R.sdot(loc, loc), R.sdot(g, g)], dtype=np.float32)
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("threads", [1, 4, 8])
def test_probe_cosine_follows_the_restated_torch_order(threads):
    models = H.probe_models(H.probe_size(threads))
    cat = lambda m: torch.cat([w.view(-1) for w in m.values()]).numpy()  # noqa: E731
    a = cat(models["baseline"]) - cat(models["previous"])
    b = torch.cat([(models["client"][k] - models["baseline"][k]).view(-1) for k in models["baseline"]]).numpy()
    assert H.host_port_value(models, threads).tobytes() == R.torch_cosine(a, b, threads).tobytes()


def test_probe_model_shape():
    m = H.probe_models()
    assert list(m["baseline"]) == ["b.weight", "b.num_batches_tracked", "a.weight"]
    assert sum(v.numel() for v in m["baseline"].values()) == H.PROBE_N
    assert m["baseline"]["b.num_batches_tracked"].dtype == torch.int64
    assert sorted(m["baseline"], key=str.lower)[0] == "a.weight"  # name order reorders the arena


@pytest.mark.parametrize("threads", [1, 16, 33, 64, 256])
def test_probe_splits_over_every_thread(threads):
    # ATen's two-pass sum runs min(threads, ceil(n / 32768)) chunks: the probe must reach `threads` of them
    assert math.ceil(H.probe_size(threads) / H.GRAIN) >= threads
    assert H.probe_size(threads) >= H.PROBE_N


def test_probe_is_fixed_and_describes_the_host():
    x1, y1 = H.probe_vectors()
    x2, y2 = H.probe_vectors()
    assert x1.tobytes() == x2.tobytes() and y1.tobytes() == y2.tobytes()
    assert x1.size == H.PROBE_N and x1.dtype == np.float32
    desc = H.host_description()
    assert "ATen CPU capability" in desc and "torch threads" in desc


def test_mode_setting():
    assert H.mode("warn") == "warn"
    assert H.mode("strict") == "strict" and H.mode(True) == "strict"
    assert H.mode(False) is None and H.mode(None) is None and H.mode("off") is None
    with pytest.raises(ValueError):
        H.mode("sometimes")

"""The FedAdp producers' exact division (fedadp.hip adp_div_lr_f64, tuning variants 60-62):
float32 (-d) / lr computed as float32(float64(-d) * (1 / float64(lr))) must give the float32
division's bits for every finite d, including subnormals and overflow to infinity."""

import numpy as np
import pytest


@pytest.mark.parametrize("lr", [0.01, 0.1, 1.0, 3e-5, 0.37, 7.3e-39, 1e30, -0.05])
def test_f64_reciprocal_product_rounds_like_f32_division(lr):
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2**32, size=2_000_000, dtype=np.uint64).astype(np.uint32)
    v = bits.view(np.float32)
    v = np.concatenate([v[np.isfinite(v)], np.array([0.0, -0.0, 1e-45, -1e-45, 3.4e38], np.float32)])
    lr32 = np.float32(lr)
    with np.errstate(all="ignore"):
        want = v / lr32
        got = (v.astype(np.float64) * (1.0 / np.float64(lr32))).astype(np.float32)
    assert np.array_equal(want.view(np.uint32), got.view(np.uint32))

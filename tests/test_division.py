"""Exact float32 division by a float64 reciprocal product: x / d computed as
float32(float64(x) * (1 / float64(d))) must give the float32 division's bits (the FedAdp producers'
division by -lr, fedadp.hip adp_div_lr_f64) for every x and d, including subnormals, zeros,
infinities and overflow to infinity."""

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


def test_f64_reciprocal_product_rounds_like_f32_division_random_divisors():
    """Random divisors over the whole float32 range (signs, subnormals, zero and infinity included),
    random dividends: the identity for any learning rate, not only the sampled ones above."""
    rng = np.random.default_rng(11)
    dbits = rng.integers(0, 2**32, size=400, dtype=np.uint64).astype(np.uint32)
    ds = dbits.view(np.float32)
    ds = np.concatenate([ds[np.isfinite(ds)], np.array([1e-45, 1.17549435e-38, 1.0, 3.4e38, 0.0, np.inf],
                                                       np.float32)])
    for d in ds:
        bits = rng.integers(0, 2**32, size=50_000, dtype=np.uint64).astype(np.uint32)
        v = bits.view(np.float32)
        v = np.concatenate([v[~np.isnan(v)], np.array([0.0, -0.0, 1e-45, -3.4e38, np.inf], np.float32)])
        with np.errstate(all="ignore"):
            want = v / np.float32(d)
            got = (v.astype(np.float64) * (1.0 / np.float64(d))).astype(np.float32)
        nan = np.isnan(want)
        assert np.array_equal(np.isnan(got), nan), d
        assert np.array_equal(want[~nan].view(np.uint32), got[~nan].view(np.uint32)), d

"""Host-side model of the depth sort's key transform (binning.hip: depth_keys_kernel,
key_of, the first digit scan's base / pass count), run in numpy on the CPU.

The sort runs on its own stream beside preprocess, so its first pass counts digits
before the key base is known: the base has its low byte cleared (the first digit is
the raw bits' low byte), and in three-pass mode keys beyond 2^24 saturate their top
16 bits but keep their low byte, so every pass sorts by digits of one and the same
key.  This model runs the same LSD passes (stable, 8-bit digits) and checks that the
candidates (z > 0.2) come out in (depth bits, index) order — the order
tests/test_gpu_parity.py checks on the GPU against the oracle."""
import numpy as np
import pytest


def key_of(k, base, passes):
    d = (k - base) & 0xFFFFFFFF
    if passes == 3:
        d = np.where(d > 0xFFFFFF, 0xFFFF00 | (d & 0xFF), d)
    return d


def depth_order(z):
    """The library's depth sort, pass by pass (values = indices)."""
    cand = z > np.float32(0.2)
    keys = np.where(cand, z.view(np.uint32), np.uint32(0x7F800000)).astype(np.int64)
    if cand.any():
        kmin, kmax = int(keys[cand].min()), int(keys[cand].max())
        base = kmin & ~0xFF
        passes = 4 if kmax - base > 0xFFFFFF else 3
    else:
        base, passes = 0, 3
    vals = np.arange(z.size)
    # pass 1 digit: the raw low byte (counted by depth_keys_kernel before the base exists)
    order = np.argsort(keys & 0xFF, kind="stable")
    k = key_of(keys[order], base, passes)
    assert np.array_equal(k & 0xFF, keys[order] & 0xFF)  # the digit pass 1 counted is the one it sorted by
    vals = vals[order]
    for p in range(1, passes):
        o = np.argsort((k >> (8 * p)) & 0xFF, kind="stable")
        k, vals = k[o], vals[o]
    return vals, cand, passes


@pytest.mark.parametrize("spread", ["narrow", "wide", "extreme", "saturate"])
def test_depth_sort_model_orders_candidates(spread):
    rng = np.random.default_rng({"narrow": 1, "wide": 2, "extreme": 3, "saturate": 4}[spread])
    n = 50_000
    if spread == "narrow":  # config C: depths in [4, 8] -> three passes
        z = rng.uniform(4.0, 8.0, n)
    elif spread == "wide":  # a real scene: near and far -> four passes
        z = np.exp(rng.uniform(np.log(0.3), np.log(200.0), n))
    elif spread == "extreme":  # ties, the near plane, culled, +inf / NaN depths
        z = rng.choice([0.1, 0.2, 0.25, 1.0, 1.0, 3.5, np.inf, np.nan, -2.0], n)
    else:  # three passes whose non-candidates saturate beside candidates at the top of the 2^24 range
        z = rng.choice([0.1, 0.25, 0.3, 0.3, -np.inf, np.nan], n)
    z = z.astype(np.float32)
    if spread == "saturate":
        b = np.float32(0.25).view(np.uint32) & ~np.uint32(0xFF)
        z[:4] = np.array([b + 0xFFFFFF, b + 0xFFFF80, b + 0xFFFF00, b + 0xFFFFFF], np.uint32).view(np.float32)
    if spread == "extreme":
        b = np.float32(0.25).view(np.uint32) & ~np.uint32(0xFF)
        z[:3] = np.array([b + 0xFFFFFF, b + 0xFFFF80, b + 0x1000000], np.uint32).view(np.float32)
    vals, cand, passes = depth_order(z)
    assert np.array_equal(np.sort(vals), np.arange(n))
    got = vals[cand[vals]]
    idx = np.nonzero(cand)[0]
    expect = idx[np.lexsort((idx, z.view(np.uint32)[cand]))]
    np.testing.assert_array_equal(got, expect)
    assert passes == {"narrow": 3, "wide": 4, "extreme": 4, "saturate": 3}[spread]

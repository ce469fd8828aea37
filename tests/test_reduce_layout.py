"""CPU simulation of render_bwd's wave reduce-scatter (3dgs_study_amd/csrc/render_bwd.hip:
reduce_emit).  It checks the lane layout the kernel's single 9-lane atomic per
Gaussian relies on: after the five ds_swizzle stages and the v_permlane32
self-swap, Gaussian a's nine sums sit in lanes LA (slots 0..8) and b's in lanes
LB of one register, and the select-free odd-register stages (swz_fold) leave
those lanes bit for bit equal to the zero-padded form (swz_stage(c, 0)).

The semantics being reduced are upstream BACKWARD::renderCUDA's per-Gaussian
sums over a tile's pixels; this test covers only the
exchange pattern, the GPU parity tests cover the values."""
import numpy as np

LANES = np.arange(64)
LA = [0, 8, 4, 12, 2, 10, 6, 14, 1]
LB = [16, 24, 20, 28, 18, 26, 22, 30, 17]


def swizzle(v, k):
    """ds_swizzle bit-mask mode (and 0x1F, xor k): lane l reads lane l ^ k of its 32-lane half."""
    return v[LANES ^ k]


def swz_stage(c, d, k):
    hi = (LANES & k) != 0
    keep = np.where(hi, d, c)
    send = np.where(hi, c, d)
    return (keep + swizzle(send, k)).astype(np.float32)


def swz_fold(c, k):
    return (c + swizzle(c, k)).astype(np.float32)


def reduce_scatter(pa, pb, fold):
    """pa, pb: [9, 64] per-pixel values of Gaussians a and b; returns the register after the swap."""
    h16 = (LANES & 16) != 0
    o = [np.where(h16, pb[j], pa[j]) + swizzle(np.where(h16, pa[j], pb[j]), 16) for j in range(9)]
    o = [x.astype(np.float32) for x in o]
    pad = (lambda c, k: swz_fold(c, k)) if fold else (lambda c, k: swz_stage(c, np.zeros(64, np.float32), k))
    t0, t1, t2, t3 = (swz_stage(o[2 * i], o[2 * i + 1], 8) for i in range(4))
    t4 = pad(o[8], 8)
    u0, u1, u2 = swz_stage(t0, t1, 4), swz_stage(t2, t3, 4), pad(t4, 4)
    w0, w1 = swz_stage(u0, u1, 2), pad(u2, 2)
    x0 = swz_stage(w0, w1, 1)
    return (x0 + x0[LANES ^ 32]).astype(np.float32)


def test_slot_lanes_hold_the_full_sums():
    rng = np.random.default_rng(7)
    pa = rng.integers(-8, 8, (9, 64)).astype(np.float32)  # small integers: sums are exact
    pb = rng.integers(-8, 8, (9, 64)).astype(np.float32)
    v = reduce_scatter(pa, pb, fold=True)
    for j in range(9):
        assert v[LA[j]] == pa[j].sum() and v[LA[j] + 32] == pa[j].sum()
        assert v[LB[j]] == pb[j].sum() and v[LB[j] + 32] == pb[j].sum()


def test_fold_matches_zero_padded_stages_bitwise():
    rng = np.random.default_rng(11)
    for _ in range(20):
        pa = rng.standard_normal((9, 64)).astype(np.float32)
        pb = rng.standard_normal((9, 64)).astype(np.float32)
        a = reduce_scatter(pa, pb, fold=False)
        b = reduce_scatter(pa, pb, fold=True)
        slots = LA + LB + [l + 32 for l in LA + LB]
        assert np.array_equal(a[slots].view(np.uint32), b[slots].view(np.uint32))

"""Split replay of long tile lists (include/gsr.h gsr_split_mode; gsr_common.hpp;
render_fwd.hip's checkpoints, render_bwd.hip's segment waves).

With GSR_FLAG_PREPARE_BACKWARD the forward stores each pixel's T and colour before
every SEG-th entry of a list longer than SEG, and the backward replays every SEG
entries of such a list in a wave of its own.  At every segment length the forward's
outputs are the unsplit ones bit for bit, the gradients meet the oracle parity bar
(rel-L2 <= GRAD_TOL) and agree with the unsplit replay to float rounding, also for
pixels whose compositing stops (T < 1e-4) inside a later segment."""
import numpy as np
import pytest

from helpers import case, random_dL, rel_l2, run_hip, run_oracle
from test_gpu_parity import check_backward, check_forward

pytestmark = pytest.mark.gpu

GRADS = ("dmeans2D", "dcolors", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot")
# split vs unsplit replay: the segment's start state is the forward's T and
# (C_final - C) / T instead of the replay's divided-down T and running sum
SPLIT_TOL = 1e-5


@pytest.fixture
def set_split():
    from diff_gaussian_rasterization import _C

    prev = _C.get_split()
    yield _C.set_split
    _C.set_split(prev)


CASES = {
    # a dense ball: lists of several hundred entries, most pixels stop (T < 1e-4) mid-list
    "dense": dict(P=30_000, W=160, H=128, deg=3, seed=11, radius=0.6, scale_range=(0.01, 0.06)),
    # config B (its centre tiles: ~740 entries)
    "B": dict(P=100_000, W=800, H=800, deg=3, seed=1),
}


def _case(name):
    c = CASES[name]
    cam, g = case(c["P"], c["W"], c["H"], c["deg"], seed=c["seed"], radius=c.get("radius", 2.0),
                  scale_range=c.get("scale_range", (0.003, 0.03)))
    return c, cam, g


@pytest.mark.parametrize("footprint", ["rect", "tight"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_split_replay_gradients(dev, oracle, set_split, name, footprint):
    c, cam, g = _case(name)
    dL = random_dL(c["H"], c["W"])
    r = run_oracle(oracle, cam, g)
    rb = oracle.backward(r, dL)
    lens = (r["ranges"][:, 1] - r["ranges"][:, 0]).astype(np.int64)
    assert lens.max() > 2 * 128, lens.max()  # several segments at SEG = 128
    out = {}
    for seg in (0, 128, 256, -1):
        set_split(seg)
        out[seg] = run_hip(cam, g, dev, dL=dL, footprint=footprint, prepare=True)
    base = out[0]
    if footprint == "rect":
        check_forward(base, r)
    check_backward(base, rb)
    for seg in (128, 256, -1):
        h = out[seg]
        for k in ("color", "final_T", "n_contrib", "point_list", "ranges"):
            np.testing.assert_array_equal(h[k], base[k], err_msg=f"seg {seg}: {k}")
        check_backward(h, rb)
        errs = {n: rel_l2(h["grads"][n], base["grads"][n]) for n in GRADS if base["grads"][n].size}
        assert max(errs.values()) <= SPLIT_TOL, (seg, errs)


def test_split_replay_stops_inside_later_segments(dev, oracle, set_split):
    """Pixels whose compositing stops inside a segment after the first: their replay
    starts from final_T in that segment and from the checkpoints in the earlier ones."""
    c, cam, g = _case("dense")
    dL = random_dL(c["H"], c["W"])
    set_split(128)
    h = run_hip(cam, g, dev, dL=dL, prepare=True)
    W, H = c["W"], c["H"]
    gx = (W + 15) // 16
    ys, xs = np.mgrid[0:H, 0:W]
    tile = (ys // 16) * gx + xs // 16
    n = (h["ranges"][:, 1] - h["ranges"][:, 0]).astype(np.int64)[tile]
    nc = h["n_contrib"].astype(np.int64)
    stopped_late = (nc > 128) & (nc < n) & (h["final_T"] < 1e-3)
    assert stopped_late.sum() > 100, stopped_late.sum()
    r = run_oracle(oracle, cam, g)
    check_backward(h, oracle.backward(r, dL))


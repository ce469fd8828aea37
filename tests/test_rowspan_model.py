"""Host-side model of the row-span binning (rowspan.hip; rank_gather_kernel's row
counts in binning.hip), run in numpy on the CPU with the kernels' own block
decomposition and offset arithmetic.

Pass A: blocks of RSA_GAUSS ranks count their spans per tile row, the counts are
scanned per row over the blocks, and each block scatters its spans (in rank
order, rows inside a Gaussian ascending) to row start + block offset + in-block
rank.  Pass B: blocks of RSB_SPANS spans of one row (the segment table from the
row totals), column counts per block from a difference array, one exclusive scan
per column over all blocks, and each block scatters its tiles' ids to
rows-before + columns-before-in-the-row + the row's earlier blocks + in-block
rank; the row's first block writes the ranges.  The model must reproduce the
oracle's (upstream's) point_list and ranges exactly for the rect footprint, and a
direct (tile, rank) sort for masked footprints — the GPU tests then hold the
kernels to the same lists (test_gpu_parity.py)."""
import math

import numpy as np
import pytest

from helpers import activated, case

RSA_GAUSS, RSB_SPANS = 256, 1024  # pass B: 1,024 spans per block, 256 up to a capacity of 2^20 (gsr_common.hpp)


def excl(v):
    return np.concatenate([[0], np.cumsum(v)[:-1]]).astype(np.int64)


def spans_of(x0, x1, y0, y1, mask):
    """Per Gaussian (rank order) its spans [(row, xa, xb)] (gsr_spans.hpp)."""
    out = []
    x0, x1, y0, y1 = (np.asarray(v).astype(np.int64).tolist() for v in (x0, x1, y0, y1))
    for i in range(len(x0)):
        w, s = x1[i] - x0[i], []
        for k in range(max(y1[i] - y0[i], 0) if w > 0 else 0):
            if mask[i] is None:
                s.append((y0[i] + k, x0[i], x1[i]))
                continue
            bits = (mask[i] >> (k * w)) & ((1 << w) - 1)
            if bits:
                lo = (bits & -bits).bit_length() - 1
                s.append((y0[i] + k, x0[i] + lo, x0[i] + bits.bit_length()))
        out.append(s)
    return out


def rowspan_model(ids, spans, gx, gy, spb=RSB_SPANS):
    """point_list, ranges from the kernels' arithmetic; ids / spans in rank order;
    spb: spans per pass-B block."""
    P = len(ids)
    nA = max(1, -(-P // RSA_GAUSS))
    # pass A counts (rank_gather_kernel) and their per-row scan (launch_count_scan)
    ahist = np.zeros((gy, nA), np.int64)
    for r, s in enumerate(spans):
        for (y, _, _) in s:
            ahist[y, r // RSA_GAUSS] += 1
    atot = ahist.sum(1)
    ahist = np.cumsum(ahist, 1) - ahist
    S = int(atot.sum())
    span_x, span_id, span_row = np.zeros(S, np.int64), np.zeros(S, np.int64), np.full(S, -1)
    row0 = excl(atot)
    for blk in range(nA):  # rowspan_a_kernel (one round: the same positions as several)
        items = [(y, ids[r], xa, xb) for r in range(blk * RSA_GAUSS, min(P, (blk + 1) * RSA_GAUSS))
                 for (y, xa, xb) in spans[r]]
        run = np.zeros(gy, np.int64)
        for (y, i, xa, xb) in items:  # stable: item order inside each row
            pos = row0[y] + ahist[y, blk] + run[y]
            run[y] += 1
            assert span_row[pos] == -1
            span_x[pos], span_id[pos], span_row[pos] = xa | (xb << 16), i, y
    assert (span_row >= 0).all()
    # the segment table (write_b_segments)
    nb = -(-atot // spb)
    fb, fs, nB = excl(nb), excl(atot), int(nb.sum())
    fb = np.append(fb, nB)
    fs = np.append(fs, S)
    bhist = np.zeros((gx, max(nB, 1)), np.int64)
    blocks = []
    for b in range(nB):  # rowspan_b_count_kernel: the difference array
        r = int(np.searchsorted(fb[:-1], b, "right") - 1)
        s0 = fs[r] + (b - fb[r]) * spb
        s1 = min(s0 + spb, fs[r + 1])
        h = np.zeros(gx + 1, np.int64)
        for s in range(s0, s1):
            assert span_row[s] == r
            h[span_x[s] & 0xFFFF] += 1
            h[span_x[s] >> 16] -= 1
        bhist[:, b] = np.cumsum(h)[:gx]
        blocks.append((b, r, s0, s1))
    btot = bhist.sum(1)
    bhist = np.cumsum(bhist, 1) - bhist  # launch_count_scan over the nB blocks
    I = int(btot.sum())
    point_list, ranges = np.full(I, -1, np.int64), np.zeros((gx * gy, 2), np.int64)
    for (b, r, s0, s1) in blocks:  # rowspan_b_kernel
        h0 = bhist[:, fb[r]]
        h1 = bhist[:, fb[r + 1]] if fb[r + 1] < nB else btot
        hb = bhist[:, b]
        n = h1 - h0
        cs = h0.sum() + excl(n)
        gbase = cs + (hb - h0)
        if b == fb[r]:
            ranges[r * gx:(r + 1) * gx] = np.where(n[:, None] > 0, np.stack([cs, cs + n], 1), 0)
        run = np.zeros(gx, np.int64)
        for s in range(s0, s1):
            for x in range(span_x[s] & 0xFFFF, span_x[s] >> 16):
                pos = gbase[x] + run[x]
                run[x] += 1
                assert point_list[pos] == -1
                point_list[pos] = span_id[s]
    assert (point_list >= 0).all()
    return point_list, ranges


def rank_order(depths, visible):
    idx = np.flatnonzero(visible)
    return idx[np.lexsort((idx, depths[idx].view(np.uint32)))]


@pytest.mark.parametrize("spb", [1024, 256])
@pytest.mark.parametrize("P,W,H,seed", [(3_000, 333, 201, 1), (2_500, 160, 120, 5), (1_200, 800, 256, 7)])
def test_rowspan_model_matches_oracle_rect(oracle, P, W, H, seed, spb):
    cam, g = case(P, W, H, 0, seed=seed, scale_range=(0.003, 0.08))
    a = activated(g)
    r = oracle.forward(a["means3D"].numpy(), a["opacities"].numpy(), cam.world_view_transform.numpy(),
                       cam.full_proj_transform.numpy(), cam.camera_center.numpy(), np.zeros(3, np.float32), H, W,
                       math.tan(cam.FoVx / 2), math.tan(cam.FoVy / 2), 1.0, 0, shs=a["shs"].numpy(),
                       scales=a["scales"].numpy(), rotations=a["rotations"].numpy())
    gx, gy = (W + 15) // 16, (H + 15) // 16
    order = rank_order(r["depths"], r["radii"] > 0)
    rc = r["rects"][order]
    spans = spans_of(rc[:, 0], rc[:, 2], rc[:, 1], rc[:, 3], [None] * len(order))
    assert len(order) > RSA_GAUSS and sum(map(len, spans)) > spb  # several blocks in both passes
    pl, ranges = rowspan_model(order, spans, gx, gy, spb)
    np.testing.assert_array_equal(pl, r["point_list"])
    np.testing.assert_array_equal(ranges, r["ranges"].astype(np.int64))


@pytest.mark.parametrize("spb", [1024, 256])
def test_rowspan_model_masked_footprints(spb):
    """Tight-footprint masks (per row one run of columns or nothing, rects of at most
    64 tiles), mixed with full rects: the lists are the (tile, rank) sort."""
    rng = np.random.default_rng(3)
    gx, gy, P = 37, 23, 4_000
    x0, y0 = rng.integers(0, gx, P), rng.integers(0, gy, P)
    x1 = np.minimum(x0 + rng.integers(1, 9, P), gx)
    y1 = np.minimum(y0 + rng.integers(1, 9, P), gy)
    masks = []
    for i in range(P):
        w, h = int(x1[i] - x0[i]), int(y1[i] - y0[i])
        if w * h > 64 or rng.random() < 0.3:
            masks.append(None)  # all ones: the whole rect
            continue
        m = 0
        for k in range(h):
            if rng.random() < 0.2:
                continue  # an empty row
            a = int(rng.integers(0, w))
            b = int(rng.integers(a + 1, w + 1))
            m |= ((1 << (b - a)) - 1) << (k * w + a)
        masks.append(m)
    ids = rng.permutation(P)  # rank r holds Gaussian ids[r]
    spans = spans_of(x0, x1, y0, y1, masks)
    pl, ranges = rowspan_model(ids, spans, gx, gy, spb)
    tiles = [(y * gx + x, r) for r, s in enumerate(spans) for (y, xa, xb) in s for x in range(xa, xb)]
    tiles.sort()
    np.testing.assert_array_equal(pl, ids[[r for (_, r) in tiles]])
    t = np.array([t for (t, _) in tiles])
    for tile in range(gx * gy):
        s0, s1 = np.searchsorted(t, tile, "left"), np.searchsorted(t, tile, "right")
        assert tuple(ranges[tile]) == ((s0, s1) if s1 > s0 else (0, 0))

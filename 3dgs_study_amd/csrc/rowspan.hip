// rowspan.hip — row-span tile binning: upstream's per-tile lists from two stable
// counting sorts over the tile grid's rows and columns.
//
// Replaces upstream duplicateWithKeys + cub::DeviceRadixSort::SortPairs +
// identifyTileRanges (rasterizer_impl.cu) for
// grids of at most 256 x 256 tiles (binning.hip keeps the LSD tile sort for
// larger ones).  Upstream lists, per tile, the Gaussians whose footprint covers
// it in (depth bits, id) order.  After the depth sort (binning.hip: order[rank]
// = id in that order; rank_gather_kernel: the footprints in rank order) the same
// lists follow from the footprint's structure: per tile row it is one contiguous
// span of columns (gsr_spans.hpp).  So:
//
//   A. every Gaussian's spans {id, x0 | x1 << 16} are sorted stably by tile row,
//      in rank order: per block of RSA_GAUSS ranks a row histogram
//      (rank_gather_kernel), a per-row scan over the blocks (launch_count_scan),
//      and rowspan_a_kernel, which expands its Gaussians into spans and
//      scatters them by row;
//   B. each row's spans (rank order) expand into their tiles, sorted stably by
//      column: per block of RSB_SPANS spans of one row a column histogram
//      (rowspan_b_count_kernel: a difference array, two LDS adds per span), a
//      per-column scan, and rowspan_b_kernel, which expands the spans and
//      scatters the Gaussian ids by column into point_list, and writes the tile
//      ranges from the column counts.
//
// Both sorts are stable, so each tile's list stays in rank order — upstream's
// (depth bits, id) — and the lists follow each other in tile-index order
// (row-major), upstream's point_list bit for bit.  A Gaussian has at most one
// span per row and a span at most one tile per column, so no ties arise inside a
// digit except between different sources, which the stable rank orders.
//
// Traffic at config C (rect footprint: 1M Gaussians, 2.72M spans, 8.02M
// instances): 8 B per span written by A and read by both B kernels, 4 B per
// instance written once — against 27 B per instance for an emission in rank
// order plus two LSD passes by tile index.  Inside a workgroup the items of a
// round (the block's expansion, up to RS_THREADS x ITEMS of them) are ranked like
// the radix downsweep's (binning.hip): each wave takes a contiguous quarter in
// rounds of 64, lanes with the same digit found by ballots (match_digit), a
// running per-wave count per digit; the block's digit runs are laid out in LDS
// and leave coalesced.
#pragma clang fp contract(off)

#include "gsr_kernels.hpp"
#include "gsr_radix.hpp"
#include "gsr_spans.hpp"
#include "gsr_wave.hpp"

#include <type_traits>

namespace gsr {

constexpr int RS_WAVES = RS_THREADS / 64;
constexpr int RS_COUNT_GRID = 2048;  // rowspan_b_count_kernel's grid at most (256 CUs x 8)
#ifndef GSR_RSB_WAVES
#define GSR_RSB_WAVES 4
#endif
#ifndef GSR_RSA_WAVES
#define GSR_RSA_WAVES 6
#endif
constexpr int RSA_ROUND = RS_THREADS * RSA_ITEMS, RSB_ROUND = RS_THREADS * RSB_ITEMS;
constexpr int RSA_PER = RSA_GAUSS / RS_THREADS;  // Gaussians per thread
static_assert(RSA_PER * RS_THREADS == RSA_GAUSS && RSB_SPANS % RS_THREADS == 0 && RSB_SPANS_SMALL % RS_THREADS == 0,
              "whole sources per thread");

struct RowSpanArgs {
    int P, gx, gy;
    SpecGuard g;
    // pass A
    const uint32_t *order;   // GSR_GEOM_DEPTH_ORDER: id of each rank
    const uint4 *rects;      // the footprints in rank order (rank_gather_kernel), or NULL: rwords
    const uint32_t *rwords;  // the rect footprint's words in rank order (carried by the depth sort)
    const uint32_t *ahist;   // [gy][nA] after the scan: spans of row y in the blocks before
    const uint32_t *atot;    // [RADIX] spans per row
    int nA;
    uint32_t *span_x;        // [S] x0 | x1 << 16, row-major, rank order inside a row
    uint32_t *span_id;       // [S] the Gaussian's id
    uint32_t *seg;           // [2][RADIX + 1] pass B's blocks per row: first block, first span; [RADIX] =
                             // blocks, [2 RADIX + 1] = spans (written by pass A's block 0)
    // pass B
    uint32_t *bhist;         // [RADIX][nBmax] column counts per block -> block offsets (the scan)
    const uint32_t *btot;    // [RADIX] instances per column
    int nBmax;
    int spb;                 // spans per pass-B block (rsb_spans of the capacity)
    uint4 *btab;             // [nBmax] pass B's block table (rowspan_b_count_kernel)
    uint32_t *point_list;
    uint2 *ranges;           // [T] (zeroed by preprocess; empty tiles stay (0, 0))
};

// One round of a stable counting scatter inside a workgroup.  The round's n items
// sit in LDS in item order (dig[i], pay[i]).  Each wave ranks its quarter (ITEMS
// per lane in rounds of 64: lanes of equal digit by match_digit, a running count
// per wave and digit), the round's per-digit runs are laid out digit by digit in
// LDS (pay and dig are reused as the stage once every wave holds its items) and
// leave in order: item i of the stage goes to gbase[d] + run[d] + (i - start of
// d's run), and run[d] advances by the round's count of d.
template <int ITEMS, int NB, typename T, typename Store>
__device__ __forceinline__ void scatter_round(uint32_t n, uint8_t *dig, T *pay, uint32_t (*cnt)[RADIX],
                                              const uint32_t *gbase, uint32_t *run, uint32_t *gsh, uint32_t *wsum,
                                              Store store) {
    constexpr int WAVE_N = ITEMS * 64;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < RS_WAVES; k++) cnt[k][threadIdx.x] = 0u;
    __syncthreads();
    uint32_t dd[ITEMS], rk[ITEMS];
    T pp[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const uint32_t i = (uint32_t)(w * WAVE_N + r * 64 + lane);
        const bool ok = i < n;
        dd[r] = ok ? (uint32_t)dig[i] : 0u;
        pp[r] = ok ? pay[i] : T{};
    }
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const bool ok = (uint32_t)(w * WAVE_N + r * 64 + lane) < n;
        const uint64_t live = __ballot(ok);
        if (!live) break;
        const uint64_t peers = match_digit<NB>(dd[r], live);
        const uint32_t below = count_below(peers);
        const uint32_t c = cnt[w][dd[r]];
        rk[r] = c + below;
        if (ok && below == 0) cnt[w][dd[r]] = c + (uint32_t)__popcll(peers);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    __syncthreads();
    {  // the round's runs: digit by digit, each wave's items after the waves before
        uint32_t c[RS_WAVES], sum = 0;
#pragma unroll
        for (int k = 0; k < RS_WAVES; k++) {
            c[k] = cnt[k][threadIdx.x];
            sum += c[k];
        }
        uint32_t tot;
        const uint32_t start = block_inclusive_scan<RS_THREADS>(sum, wsum, &tot) - sum;
        gsh[threadIdx.x] = gbase[threadIdx.x] + run[threadIdx.x] - start;
        run[threadIdx.x] += sum;
        uint32_t off = start;
#pragma unroll
        for (int k = 0; k < RS_WAVES; k++) {
            cnt[k][threadIdx.x] = off;
            off += c[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if ((uint32_t)(w * WAVE_N + r * 64 + lane) < n) {
            const uint32_t p = cnt[w][dd[r]] + rk[r];
            pay[p] = pp[r];
            dig[p] = (uint8_t)dd[r];
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += RS_THREADS) store(gsh[dig[i]] + i, pay[i]);
    __syncthreads();
}

// Pass B's blocks: ceil(spans / RSB_SPANS) per row, in row order.  Written by pass
// A's block 0 from the row totals, read by both pass-B kernels.
__device__ __forceinline__ void write_b_segments(const RowSpanArgs &a, uint32_t *wsum) {
    const uint32_t t = threadIdx.x;
    const uint32_t tot = (int)t < a.gy ? a.atot[t] : 0u;
    const uint32_t nb = (tot + (uint32_t)a.spb - 1u) / (uint32_t)a.spb;
    uint32_t tb, ts;
    const uint32_t ib = block_inclusive_scan<RS_THREADS>(nb, wsum, &tb);
    const uint32_t is = block_inclusive_scan<RS_THREADS>(tot, wsum, &ts);
    a.seg[t] = ib - nb;
    a.seg[RADIX + 1 + t] = is - tot;
    if (t == 0) {
        a.seg[RADIX] = tb;
        a.seg[2 * RADIX + 1] = ts;
    }
}

// Pass A: the spans of RSA_GAUSS consecutive ranks, scattered by tile row.
template <int NB>
__global__ void __launch_bounds__(RS_THREADS, GSR_RSA_WAVES) rowspan_a_kernel(RowSpanArgs a) {
    __shared__ uint8_t dig[RSA_ROUND];
    __shared__ uint2 pay[RSA_ROUND];
    __shared__ uint32_t cnt[RS_WAVES][RADIX];
    __shared__ uint32_t gbase[RADIX], run[RADIX], gsh[RADIX], wsum[RS_WAVES];
    if (!spec_ok(a.g)) return;
    const uint32_t blk = radix_block(a.nA);
    const uint32_t t = threadIdx.x;
    // every load first (no barrier between them): this thread's Gaussians, ranks
    // r0 + RSA_PER t + j, and row t's totals
    const int r0 = (int)blk * RSA_GAUSS + (int)t * RSA_PER;
    uint4 q[RSA_PER];
    uint32_t id[RSA_PER];
#pragma unroll
    for (int j = 0; j < RSA_PER; j++) {
        const int r = r0 + j;
        if (a.rwords)
            q[j].x = r < a.P ? a.rwords[r] : 0xffu;
        else
            q[j] = r < a.P ? a.rects[r] : make_uint4(0u, 0u, 0u, 0u);
        id[j] = r < a.P ? a.order[r] : 0u;
    }
    const uint32_t tot = (int)t < a.gy ? a.atot[t] : 0u;
    const uint32_t before = (int)t < a.gy ? a.ahist[(size_t)t * a.nA + blk] : 0u;
    if (blk == 0) write_b_segments(a, wsum);
    {  // where this block's spans of each row start: the rows before, the blocks before
        uint32_t all;
        gbase[t] = block_inclusive_scan<RS_THREADS>(tot, wsum, &all) - tot + before;
        run[t] = 0u;
    }
    Foot f[RSA_PER];
    uint32_t pre[RSA_PER], my = 0;
#pragma unroll
    for (int j = 0; j < RSA_PER; j++) {
        f[j] = a.rwords ? foot_of_word(q[j].x) : foot_of(q[j]);
        pre[j] = my;
        my += foot_spans(f[j]);
    }
    uint32_t total;
    const uint32_t mine = block_inclusive_scan<RS_THREADS>(my, wsum, &total) - my;
    auto store = [&](uint32_t pos, uint2 p) {
        a.span_id[pos] = p.x;
        a.span_x[pos] = p.y;
    };
    for (uint32_t o = 0; o < total; o += RSA_ROUND) {
        const uint32_t n = min((uint32_t)RSA_ROUND, total - o);
        // expansion: each Gaussian's spans of this round, in row order
#pragma unroll
        for (int j = 0; j < RSA_PER; j++) {
            uint32_t it = mine + pre[j];  // the Gaussian's first span in the block's sequence
            for (uint32_t y = f[j].y0; y < f[j].y1 && it < o + n; y++) {
                const uint32_t k = y - f[j].y0;
                if (!foot_row_kept(f[j], k)) continue;
                if (it >= o) {
                    dig[it - o] = (uint8_t)y;
                    pay[it - o] = make_uint2(id[j], foot_row_span(f[j], k));
                }
                it++;
            }
        }
        __syncthreads();
        scatter_round<RSA_ITEMS, NB>(n, dig, pay, cnt, gbase, run, gsh, wsum, store);
    }
}

// Pass B's block table entry: {first span, row | spans << 16, the row's first
// block, the next row's first block} (the count kernel writes it, from the segment
// table of pass A's block 0; rowspan_b_kernel reads it)
__device__ __forceinline__ uint32_t bt_row(uint4 e) { return e.y & 0xffffu; }
__device__ __forceinline__ uint32_t bt_end(uint4 e) { return e.x + (e.y >> 16); }

// Pass B's counts: per block, the instances of each column (difference array),
// and the block's table entry.  A grid-stride loop over the device's block count
// (the grid is sized by the capacity, which bounds it: most of a fixed-size grid
// sized that way would find no block).
__global__ void __launch_bounds__(RS_THREADS) rowspan_b_count_kernel(RowSpanArgs a) {
    __shared__ uint32_t sfb[RADIX + 1], sfs[RADIX + 1], h[RADIX + 1], wsum[RS_WAVES];
    if (!spec_ok(a.g)) return;
    const uint32_t nB = min(a.seg[RADIX], (uint32_t)a.nBmax);
    // XCD-contiguous: workgroup w of XCD x takes blocks x * per + w + k * grid
    const uint32_t per = gridDim.x >> 3, b0 = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (b0 >= nB) return;
    sfb[threadIdx.x] = a.seg[threadIdx.x];
    sfs[threadIdx.x] = a.seg[RADIX + 1 + threadIdx.x];
    if (threadIdx.x == 0) {
        sfb[RADIX] = nB;
        sfs[RADIX] = a.seg[2 * RADIX + 1];
    }
    for (uint32_t b = b0; b < nB; b += gridDim.x) {
        h[threadIdx.x] = 0u;
        if (threadIdx.x == 0) h[RADIX] = 0u;
        __syncthreads();
        uint32_t r = 0;  // the last row whose first block is <= b (sfb is non-decreasing, sfb[0] = 0)
#pragma unroll
        for (uint32_t step = RADIX / 2; step >= 1; step >>= 1)
            if (sfb[r + step] <= b) r += step;
        const uint32_t s0 = sfs[r] + (b - sfb[r]) * (uint32_t)a.spb, s1 = min(s0 + (uint32_t)a.spb, sfs[r + 1]);
        if (threadIdx.x == 0) a.btab[b] = make_uint4(s0, r | ((s1 - s0) << 16), sfb[r], sfb[r + 1]);
        for (uint32_t s = s0 + threadIdx.x; s < s1; s += RS_THREADS) {
            const uint32_t x = a.span_x[s];
            atomicAdd(&h[x & 0xffffu], 1u);
            atomicAdd(&h[x >> 16], ~0u);  // - 1
        }
        __syncthreads();
        uint32_t tot;
        const uint32_t c = block_inclusive_scan<RS_THREADS>(h[threadIdx.x], wsum, &tot);
        if ((int)threadIdx.x < a.gx) a.bhist[(size_t)threadIdx.x * a.nBmax + b] = c;
    }
}

// Pass B: the tiles of the block's spans, their ids scattered by column into
// point_list; the row's first block writes the row's tile ranges.  One block per
// workgroup (a grid-stride loop over the blocks measured 52 -> 58 us at config C:
// the dispatcher's fresh workgroups overlap each other's load chains better); the
// grid is sized by the capacity and the workgroups beyond the device's block count
// exit at once.
template <int NB, int SPB>
__global__ void __launch_bounds__(RS_THREADS, GSR_RSB_WAVES) rowspan_b_kernel(RowSpanArgs a) {
    constexpr int RSB_PER = SPB / RS_THREADS;  // spans per thread
    __shared__ uint8_t dig[RSB_ROUND];
    __shared__ uint32_t pay[RSB_ROUND];
    __shared__ uint32_t cnt[RS_WAVES][RADIX];
    __shared__ uint32_t gbase[RADIX], run[RADIX], gsh[RADIX], wsum[RS_WAVES];
    if (!spec_ok(a.g)) return;
    const uint32_t nB = min(a.seg[RADIX], (uint32_t)a.nBmax);
    uint32_t b;
    if (!radix_block_of(nB, &b)) return;
    const uint4 e = a.btab[b];
    const uint32_t row = bt_row(e), s0 = e.x, s1 = bt_end(e), first = e.z, next = e.w;
    const uint32_t t = threadIdx.x;
    // every load first: this thread's spans s0 + RSB_PER t + j, and column t's counts —
    // h0 = its instances in the blocks before the row, h1 = ... before the next row,
    // hb = ... before this block (the scanned counts)
    const uint32_t sb = s0 + t * RSB_PER;
    uint32_t x[RSB_PER], id[RSB_PER];
#pragma unroll
    for (int j = 0; j < RSB_PER; j++) {
        const uint32_t s = sb + j;
        x[j] = s < s1 ? a.span_x[s] : 0u;
        id[j] = s < s1 ? a.span_id[s] : 0u;
    }
    const bool col = (int)t < a.gx;
    const size_t rowc = (size_t)t * a.nBmax;
    const uint32_t h0 = col ? a.bhist[rowc + first] : 0u;
    const uint32_t h1 = col ? (next < nB ? a.bhist[rowc + next] : a.btot[t]) : 0u;
    const uint32_t hb = col ? a.bhist[rowc + b] : 0u;
    {
        uint32_t row0;
        block_inclusive_scan<RS_THREADS>(h0, wsum, &row0);  // instances of the rows before
        const uint32_t n = h1 - h0;
        uint32_t rowtot;
        const uint32_t cs = row0 + block_inclusive_scan<RS_THREADS>(n, wsum, &rowtot) - n;
        gbase[t] = cs + (hb - h0);
        run[t] = 0u;
        if (b == first && col) a.ranges[(size_t)row * a.gx + t] = n ? make_uint2(cs, cs + n) : make_uint2(0u, 0u);
    }
    uint32_t pre[RSB_PER], my = 0;
#pragma unroll
    for (int j = 0; j < RSB_PER; j++) {
        pre[j] = my;
        my += (x[j] >> 16) - (x[j] & 0xffffu);
    }
    uint32_t total;
    const uint32_t mine = block_inclusive_scan<RS_THREADS>(my, wsum, &total) - my;
    auto store = [&](uint32_t pos, uint32_t v) { a.point_list[pos] = v; };
    for (uint32_t o = 0; o < total; o += RSB_ROUND) {
        const uint32_t n = min((uint32_t)RSB_ROUND, total - o);
#pragma unroll
        for (int j = 0; j < RSB_PER; j++) {
            const uint32_t fi = mine + pre[j], xa = x[j] & 0xffffu, xb = x[j] >> 16;
            // the span's tiles inside [o, o + n) of the block's sequence
            const uint32_t lo = fi < o ? o - fi : 0u;
            const uint32_t hi = min(xb - xa, o + n > fi ? o + n - fi : 0u);
            for (uint32_t k = lo; k < hi; k++) {
                dig[fi + k - o] = (uint8_t)(xa + k);
                pay[fi + k - o] = id[j];
            }
        }
        __syncthreads();
        scatter_round<RSB_ITEMS, NB>(n, dig, pay, cnt, gbase, run, gsh, wsum, store);
    }
}

// the digit width as a compile-time constant: 6, 7 or 8 compared bits
static int nb_class(int digits) {
    const int bits = tile_bits(digits);
    return bits <= 6 ? 6 : bits == 7 ? 7 : 8;
}

static RowSpanArgs rowspan_args(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                                bool carry = false) {
    const GeomLayout L = geom_layout(P, W, H);
    const BinningLayout B = binning_layout(cap, W, H);
    const GridDims gd = grid_dims(W, H);
    RowSpanArgs a;
    a.P = P;
    a.gx = gd.gx;
    a.gy = gd.gy;
    a.g = g;
    a.order = at<const uint32_t>(geom, L.off[GSR_GEOM_DEPTH_ORDER]);
    a.rects = carry ? nullptr : at<const uint4>(geom, L.rects_ranked);
    a.rwords = carry ? at<const uint32_t>(geom, L.rs_words) + 2 * (size_t)P : nullptr;
    a.ahist = at<const uint32_t>(geom, L.rs_ahist);
    a.atot = at<const uint32_t>(geom, L.rs_atot);
    a.nA = rsa_blocks(P);
    a.span_x = at<uint32_t>(binning, B.keys_b);
    a.span_id = at<uint32_t>(binning, B.vals_b);
    a.seg = at<uint32_t>(binning, B.seg_table);
    a.bhist = at<uint32_t>(binning, B.hist);
    a.btot = at<const uint32_t>(binning, B.totals);
    a.nBmax = (int)B.hist_stride;
    a.spb = rsb_spans(cap > 0 ? cap : 1);
    a.btab = at<uint4>(binning, B.rs_btab);
    a.point_list = at<uint32_t>(binning, B.off[GSR_BIN_POINT_LIST]);
    a.ranges = at<uint2>(geom, L.off[GSR_GEOM_RANGES]);
    return a;
}

hipError_t launch_rowspan_a(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                            bool carry, hipStream_t s) {
    const RowSpanArgs a = rowspan_args(P, W, H, geom, binning, cap, g, carry);
    const dim3 grid(a.nA), block(RS_THREADS);
    switch (nb_class(a.gy)) {
        case 6: hipLaunchKernelGGL(rowspan_a_kernel<6>, grid, block, 0, s, a); break;
        case 7: hipLaunchKernelGGL(rowspan_a_kernel<7>, grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL(rowspan_a_kernel<8>, grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_rowspan_b(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                            hipStream_t s) {
    RowSpanArgs a = rowspan_args(P, W, H, geom, binning, cap, g);
    const dim3 block(RS_THREADS);
    // the count kernel loops: 8 workgroups per CU at most, a multiple of the 8 XCDs
    const int cgrid = (int)(min(a.nBmax, RS_COUNT_GRID) + 7) & ~7;
    hipLaunchKernelGGL(rowspan_b_count_kernel, dim3(cgrid), block, 0, s, a);
    if (hipError_t e = launch_count_scan(a.bhist, a.nBmax, a.seg + RADIX, const_cast<uint32_t *>(a.btot), a.gx, g, s))
        return e;
    const dim3 bgrid(a.nBmax);
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, bgrid, block, 0, s, a); };
    const bool small = a.spb == RSB_SPANS_SMALL;
    switch (nb_class(a.gx)) {
        case 6: small ? go(rowspan_b_kernel<6, RSB_SPANS_SMALL>) : go(rowspan_b_kernel<6, RSB_SPANS>); break;
        case 7: small ? go(rowspan_b_kernel<7, RSB_SPANS_SMALL>) : go(rowspan_b_kernel<7, RSB_SPANS>); break;
        default: small ? go(rowspan_b_kernel<8, RSB_SPANS_SMALL>) : go(rowspan_b_kernel<8, RSB_SPANS>); break;
    }
    return hipGetLastError();
}

}  // namespace gsr

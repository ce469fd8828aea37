// gsr_common.hpp — shared constants, scratch layouts and device helpers of the
// gfx950 Gaussian rasterizer.  Helpers that decide integer outputs (projection,
// ndc2Pix, getRect, covariance) follow the exact operation order of the CPU
// oracle (oracle/gsr_oracle.c), which restates upstream cuda_rasterizer/
// auxiliary.h + forward.cu.  Translation units that
// produce those integers compile with `#pragma clang fp contract(off)`.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gsr.h"

#ifndef GSR_ACCUM_STRIDE
#define GSR_ACCUM_STRIDE 16  // floats per Gaussian in the backward accumulator
#endif

namespace gsr {

constexpr int TILE_X = 16;  // BLOCK_X (upstream config.h)
constexpr int TILE_Y = 16;  // BLOCK_Y
constexpr int TILE_PIX = TILE_X * TILE_Y;
constexpr int WAVE = 64;

// Binning radix passes (binning.hip): 8-bit digits, 256-thread workgroups with
// ITEMS keys per thread (depth sort over P: 4, tile sort over I: 8).
constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int RX_THREADS = 256;
#ifndef GSR_DSORT_ITEMS
#define GSR_DSORT_ITEMS 4
#endif
#ifndef GSR_TSORT_ITEMS
#define GSR_TSORT_ITEMS 8
#endif
constexpr int DSORT_ITEMS = GSR_DSORT_ITEMS;
// The depth sort of many Gaussians (config E: 5M) likewise takes 8 items per
// thread: 285 -> 256 us at E; 1M (config C) is unchanged either way.
#ifndef GSR_DSORT_ITEMS_BIG
#define GSR_DSORT_ITEMS_BIG 8
#endif
constexpr int DSORT_ITEMS_BIG = GSR_DSORT_ITEMS_BIG;
constexpr int DSORT_BIG_N = 2 << 20;
__host__ __device__ inline int dsort_items(int P) { return P > DSORT_BIG_N ? DSORT_ITEMS_BIG : DSORT_ITEMS; }
constexpr int TSORT_ITEMS = GSR_TSORT_ITEMS;
// Long instance lists (config E: 60M) sort in bigger radix blocks: longer
// contiguous per-digit output runs and half the blocks for the digit scan
// (tile sort 875 -> 730 us at E); short ones (config C: 4.9M) keep more
// workgroups in flight (8 items: 85 us vs 91 us with 16).
#ifndef GSR_TSORT_ITEMS_BIG
#define GSR_TSORT_ITEMS_BIG 16
#endif
constexpr int TSORT_ITEMS_BIG = GSR_TSORT_ITEMS_BIG;
constexpr int64_t TSORT_BIG_N = 16 << 20;
__host__ __device__ inline int tsort_items(int64_t n) { return n > TSORT_BIG_N ? TSORT_ITEMS_BIG : TSORT_ITEMS; }
#ifndef GSR_EMIT_BLOCK
#define GSR_EMIT_BLOCK 256
#endif
constexpr int EMIT_BLOCK = GSR_EMIT_BLOCK;  // Gaussians per rank-order emit workgroup (a power of two, 64..1024)
static_assert(EMIT_BLOCK >= 64 && EMIT_BLOCK <= 1024 && (EMIT_BLOCK & (EMIT_BLOCK - 1)) == 0, "EMIT_BLOCK");
// rank_gather_kernel (binning.hip): 1024 threads x 4 ranks = RG_SUPER emit blocks
constexpr int RG_THREADS = 1024, RG_RANKS = 4, RG_SUPER = RG_THREADS * RG_RANKS / EMIT_BLOCK;
constexpr int PRE_THREADS = 256;          // preprocess block (scan granule)

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct GridDims {
    int gx, gy, tiles;
};
__host__ __device__ inline GridDims grid_dims(int W, int H) {
    GridDims g;
    g.gx = (W + TILE_X - 1) / TILE_X;
    g.gy = (H + TILE_Y - 1) / TILE_Y;
    g.tiles = g.gx * g.gy;
    return g;
}

__host__ __device__ inline int radix_blocks(int64_t n, int items) {
    const int64_t tile = (int64_t)RX_THREADS * items;
    const int64_t nb = (n + tile - 1) / tile;
    return nb < 1 ? 1 : (int)nb;
}
__host__ __device__ inline int emit_blocks(int P) { return (P + EMIT_BLOCK - 1) / EMIT_BLOCK; }
__host__ __device__ inline int rg_blocks(int P) { return (P + RG_THREADS * RG_RANKS - 1) / (RG_THREADS * RG_RANKS); }
// LSD passes of the tile sort: enough 8-bit digits to cover tile indices [0, T)
__host__ __device__ inline int tile_bits(int T) {
    int bits = 0;
    while (bits < 32 && ((uint32_t)(T - 1) >> bits) != 0u) bits++;
    return bits;
}
__host__ __device__ inline int tile_sort_passes(int T) { return (tile_bits(T) + RADIX_BITS - 1) / RADIX_BITS; }
// The two-pass tile sort (9-16 tile bits: 1080p, 4K) packs its first pass's
// output as (high tile digit << id bits) | Gaussian id, one word per instance,
// when the ids fit beside the digit (P <= 2^(32 - high bits): 16.7M Gaussians
// at 4K); the second pass then moves one word in and one out, and the tile
// ranges come from its digit counts (binning.hip).
__host__ __device__ inline bool tile_sort_packed(int T, int P) {
    if (tile_sort_passes(T) != 2) return false;
    const int bits = tile_bits(T), hi = bits - bits / 2;
    return (uint64_t)P <= (1ull << (32 - hi));
}
// Depth passes 2-4 without a digit-scan launch (binning.hip, "grouped" passes):
// the upsweep adds its digit counts into its group of DSORT_SB blocks as well, and
// each downsweep block sums the groups before its own and the blocks before it in
// its group.  For up to DSORT_GROUPED_NB blocks (1.5M Gaussians); beyond that the
// per-block reads outgrow the scan launch they replace.
constexpr int DSORT_SB_LOG2 = 5, DSORT_SB = 1 << DSORT_SB_LOG2;
#ifndef GSR_DSORT_GROUPED_NB
#define GSR_DSORT_GROUPED_NB 1536
#endif
__host__ __device__ inline bool dsort_grouped(int P) { return radix_blocks(P, dsort_items(P)) <= GSR_DSORT_GROUPED_NB; }
// the first pass grouped too (its counts from depth_keys_kernel, num_rendered published
// by that launch's extra workgroup, the key base reduced in every downsweep block):
// no digit-scan launch in the whole depth sort
#ifndef GSR_DSORT_GROUP1
#define GSR_DSORT_GROUP1 1
#endif
__host__ __device__ inline bool dsort_grouped1(int P) { return GSR_DSORT_GROUP1 && dsort_grouped(P); }
__host__ __device__ inline int dsort_nsup(int P) {
    return dsort_grouped(P) ? (radix_blocks(P, dsort_items(P)) + DSORT_SB - 1) / DSORT_SB : 1;
}
__host__ __device__ inline int pre_blocks(int P) { return (P + PRE_THREADS - 1) / PRE_THREADS; }

// Row-span binning (rowspan.hip), the default for grids of at most RADIX x RADIX
// tiles (a tile row and a tile column are each one 8-bit digit): pass A sorts the
// footprints' row spans by tile row in blocks of RSA_GAUSS ranks, pass B their
// tiles by column in blocks of RSB_SPANS spans of one row.  Each workgroup expands
// and scatters its items in rounds of RS_THREADS * ITEMS.
// pass A: 256 ranks per block, 4 spans per thread per round (8 waves per SIMD):
// duplicate 20.5 -> 18 us at C, 135 -> 133 us at E against 512 / 8 (A/B, two rounds)
#ifndef GSR_RSA_GAUSS
#define GSR_RSA_GAUSS 256
#endif
#ifndef GSR_RSA_ITEMS
#define GSR_RSA_ITEMS 4
#endif
#ifndef GSR_RSB_SPANS
#define GSR_RSB_SPANS 1024
#endif
#ifndef GSR_RSB_ITEMS
#define GSR_RSB_ITEMS 16
#endif
constexpr int RS_THREADS = 256;
constexpr int RSA_GAUSS = GSR_RSA_GAUSS, RSA_ITEMS = GSR_RSA_ITEMS;
constexpr int RSB_SPANS = GSR_RSB_SPANS, RSB_ITEMS = GSR_RSB_ITEMS;
static_assert(RS_THREADS == RADIX, "one thread per digit in the per-block digit loops");
static_assert(RG_THREADS % RSA_GAUSS == 0, "rank_gather_kernel counts whole A blocks");
__host__ __device__ inline bool rowspan_grid(int W, int H) {
    const GridDims g = grid_dims(W, H);
    return g.gx <= RADIX && g.gy <= RADIX;
}
__host__ __device__ inline int rsa_blocks(int P) { return P > 0 ? (P + RSA_GAUSS - 1) / RSA_GAUSS : 1; }
// Pass B's block size: RSB_SPANS spans, or RSB_SPANS_SMALL for capacities up to
// RSB_SMALL_CAP (config B: ~100 blocks of 1,024 spans left most CUs idle)
constexpr int RSB_SPANS_SMALL = 256;
constexpr int64_t RSB_SMALL_CAP = 1 << 20;
__host__ __device__ inline int rsb_spans(int64_t cap) { return cap <= RSB_SMALL_CAP ? RSB_SPANS_SMALL : RSB_SPANS; }
// pass B's blocks: ceil(spans of row r / rsb_spans(cap)) per row, spans <= instances <= cap
__host__ __device__ inline int rsb_blocks_max(int64_t cap, int gy) { return (int)(cap / rsb_spans(cap)) + gy + 1; }

// ---- control words (uint32 [16]) inside the geom buffer (a device copy of what
// preprocess publishes to the host: num_rendered, the prefiltered error) ----
enum CtrlWord {
    CTRL_NUM_RENDERED_LO = 0,
    CTRL_NUM_RENDERED_HI = 1,
    CTRL_PREFILTER_ERR = 2,
    CTRL_DSORT_PASSES = 3,  // host copy only: the depth sort's pass count (its first digit scan publishes it)
    CTRL_SHJAC = 4,         // device only: 1 when this forward's preprocess stored the SH direction Jacobian
    CTRL_WORDS = 16
};
// the depth sort's own control words (GeomLayout::dsort_ctrl, a line of their own)
enum DsortCtrlWord {
    DCTRL_KEY_BASE = 0,  // smallest depth key (bits) of a candidate Gaussian, low byte cleared
    DCTRL_PASSES = 1,    // 3 when every candidate key lies within 2^24 of the base, else 4
};

// Speculative binning (gsr_forward): emit and the tile sort are queued before the
// host has read num_rendered, into a binning buffer of `cap` instances.  Each of
// their kernels reads the count the depth sort's first digit scan published into
// the geom control words and does nothing at all unless it fits (and, when the
// host queued only three depth passes, unless three sufficed: a four-pass sort's
// rank order is not ready yet).  The host then re-runs what it must (gsr_forward).
// ctrl == NULL: not speculative, the host-side count is exact.
// Streaming stores for outputs no kernel of the step reads again (the leaf
// gradients preprocess_bwd writes last; read by the optimizer or the next step's
// exchange, long after): non-temporal, so they leave the Infinity Cache instead of
// sitting there dirty until the next step's preprocess evicts them while it streams
// the parameters in (its reads then wait behind the write-backs: preprocess 84 →
// 68 µs at config C with the dsh rows streamed).  GSR_NT_GRAD: 0 plain stores, 1
// (default) the dsh rest rows only — whole 128-B lines from the LDS-staged float4
// stores; 2 also the 4-16 B per-Gaussian leaf rows (written by scalar stores that
// cover a line only together: streamed, they cost preprocess_bwd 7 us for 2 us of
// preprocess at config C).
#ifndef GSR_NT_GRAD
#define GSR_NT_GRAD 1
#endif
#ifndef GSR_NT_JAC
#define GSR_NT_JAC 1  // the forward's SH Jacobian planes streamed too (read back by preprocess_bwd only)
#endif
typedef float gsr_v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_jac(float *p, float v) {
    if constexpr (GSR_NT_JAC)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <int LEVEL>
__device__ __forceinline__ void store_stream(float *p, float v) {
    if constexpr (GSR_NT_GRAD >= LEVEL)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <int LEVEL>
__device__ __forceinline__ void store_stream(float4 *p, float4 v) {
    if constexpr (GSR_NT_GRAD >= LEVEL) {
        const gsr_v4f w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<gsr_v4f *>(p));
    } else {
        *p = v;
    }
}

// The colour half of preprocess as riders on the depth sort (gsr_colour.hpp,
// gsr_colour_mode 2): colour blocks [b0, b0 + nb) of PRE_THREADS Gaussians run as
// extra workgroups of a depth-pass downsweep.  The degree-3 register path only (48
// floats per SH row: one cat row 16-B aligned, or the two leaves); nb == 0 = none.
struct ColourRide {
    const float *sh, *sh_rest, *means3D, *campos;
    const int32_t *radii;
    float *shjac;      // [9][P], or NULL
    float4 *splats;    // [P][3]: the colour words are written
    uint8_t *clamped;
    int P, D;
    int b0, nb;
};

struct SpecGuard {
    const uint32_t *ctrl;   // geom control words (CTRL_NUM_RENDERED_LO / HI)
    const uint32_t *dctrl;  // the depth sort's control words (DCTRL_PASSES)
    uint32_t cap;
    int need3;              // only three depth passes were queued
};
__device__ __forceinline__ bool spec_ok(const SpecGuard &g) {
    if (!g.ctrl) return true;
    return g.ctrl[CTRL_NUM_RENDERED_HI] == 0u && g.ctrl[CTRL_NUM_RENDERED_LO] <= g.cap &&
           (!g.need3 || g.dctrl[DCTRL_PASSES] == 3u);
}
// the instance count a binning kernel works on: the host's, or the published one
// (0 when the speculation failed: every block is then empty)
__device__ __forceinline__ uint32_t spec_count(const SpecGuard &g, uint32_t host_n) {
    if (!g.ctrl) return host_n;
    return spec_ok(g) ? g.ctrl[CTRL_NUM_RENDERED_LO] : 0u;
}

struct GeomLayout {
    size_t off[GSR_GEOM_NFIELDS];
    size_t block_sums;    // uint4 [pre_blocks(P)] per preprocess workgroup: instances | error << 31
    size_t rects;         // uint4 [P] tile rect {x0 | x1 << 16, y0 | y1 << 16} + 64-bit tile mask; 0 when not visible
    size_t rects_ranked;  // uint4 [P] the same in depth order (written by the last depth pass)
    size_t dsort_keys_a;  // uint32 [P] depth-sort ping-pong (the order lands in GSR_GEOM_DEPTH_ORDER)
    size_t dsort_keys_b;
    size_t dsort_vals_b;
    size_t dsort_vals_c;
    size_t dsort_hist;    // uint32 [RADIX][radix_blocks(P, dsort_items(P))]
    size_t dsort_totals;  // uint32 [RADIX]
    size_t dsort_minmax;  // uint2 [radix_blocks(P, dsort_items(P))] candidate key range per first-pass block
    size_t dsort_ctrl;    // uint32 [16] DsortCtrlWord
    size_t dsort_sup;     // uint32 [3][dsort_nsup(P)][RADIX] passes 2-4: digit counts per group of DSORT_SB blocks
    size_t dsort_sup0;    // uint32 [dsort_nsup(P)][RADIX] the same for pass 1 (depth_keys_kernel; zeroed by preprocess)
    size_t emit_sums;     // uint32 [emit_blocks(P)] instances before each emit block within its rank-gather block
    size_t emit_super;    // uint32 [rg_blocks(P)] instances per rank-gather block (RG_SUPER emit blocks)
    size_t rs_ahist;      // uint32 [gy][rsa_blocks(P)] row-span pass A: spans per (tile row, block) -> block offsets
    size_t rs_atot;       // uint32 [RADIX] spans per tile row
    size_t rs_words;      // uint32 [4][P] the depth sort's carried rect words (two ping-pong arrays, the
                          // rank-ordered result, preprocess's output); aliases rects_ranked (16 P bytes),
                          // which that form does not use
    size_t order_cnt;    // uint32 [8][32] backward wave-order bucket counts + the ORDER_FLAGS words (zeroed by preprocess)
    size_t accum;         // float [P][ACCUM_STRIDE] the backward's gradient accumulator (gsr.h GSR_FLAG_PREPARE_BACKWARD)
    size_t shjac;         // float [9][P] d colour / d view direction (GSR_FLAG_PREPARE_BACKWARD with SH colours)
    size_t bytes;
};
__host__ __device__ inline GeomLayout geom_layout(int P, int W, int H) {
    GeomLayout L;
    GridDims g = grid_dims(W, H);
    size_t o = 0;
    auto take = [&](size_t n) { size_t r = o; o = align_up(o + n, 256); return r; };
    L.off[GSR_GEOM_DEPTHS] = take((size_t)P * 4);
    L.off[GSR_GEOM_MEANS2D] = take((size_t)P * 8);
    L.off[GSR_GEOM_SPLATS] = take((size_t)P * 48);
    L.off[GSR_GEOM_CLAMPED] = take((size_t)P);
    L.off[GSR_GEOM_TILES_TOUCHED] = take((size_t)P * 4);
    L.off[GSR_GEOM_RANGES] = take((size_t)g.tiles * 8);
    L.off[GSR_GEOM_CTRL] = take(CTRL_WORDS * 4);
    L.off[GSR_GEOM_DEPTH_ORDER] = take((size_t)P * 4);
    L.block_sums = take((size_t)pre_blocks(P) * 16);
    L.rects = take((size_t)P * 16);
    L.rects_ranked = take((size_t)P * 16);
    L.dsort_keys_a = take((size_t)P * 4);
    L.dsort_keys_b = take((size_t)P * 4);
    L.dsort_vals_b = take((size_t)P * 4);
    L.dsort_vals_c = take((size_t)P * 4);
    L.dsort_hist = take((size_t)RADIX * radix_blocks(P, dsort_items(P)) * 4);
    L.dsort_totals = take((size_t)RADIX * 4);
    L.dsort_minmax = take((size_t)radix_blocks(P, dsort_items(P)) * 8);
    L.dsort_ctrl = take(CTRL_WORDS * 4);
    L.dsort_sup = take((size_t)3 * dsort_nsup(P) * RADIX * 4);
    L.dsort_sup0 = take((size_t)dsort_nsup(P) * RADIX * 4);
    L.off[GSR_GEOM_DSORT_CTRL] = L.dsort_ctrl;
    L.emit_sums = take((size_t)emit_blocks(P) * 4 + 4);
    L.emit_super = take((size_t)rg_blocks(P) * 4 + 4);
    L.rs_ahist = take(rowspan_grid(W, H) ? (size_t)g.gy * rsa_blocks(P) * 4 : 4);
    L.rs_atot = take((size_t)RADIX * 4);
    L.rs_words = L.rects_ranked;
    L.order_cnt = take((8 * 32 + 2) * 4);
    L.accum = take((size_t)(P > 0 ? P : 1) * GSR_ACCUM_STRIDE * 4);
    L.shjac = take((size_t)9 * (P > 0 ? P : 1) * 4);
    L.bytes = o;
    return L;
}

// The binning buffer of an instance capacity `cap` (>= num_rendered: gsr_forward
// sizes it before the count is known).  point_list comes first, at offset 0 for
// every capacity, so the blend kernels and the backward find it from the pointer
// alone; the other fields are the forward's own scratch, laid out by the capacity
// the forward was given.
struct BinningLayout {
    size_t off[GSR_BIN_NFIELDS];
    size_t keys_b;  // uint32 [cap] tile-sort ping-pong; row-span binning: the spans' columns x0 | x1 << 16
    size_t vals_b;  // uint32 [cap]; row-span binning: the spans' Gaussian ids (spans <= instances)
    size_t hist;    // uint32 [RADIX][radix_blocks(cap, tsort_items(cap)) + RADIX] (+ RADIX: segment-aligned blocks);
                    // row-span pass B: [RADIX][rsb_blocks_max(cap, gy)] column counts per block
    size_t hist_stride;  // row-span pass B's block stride in hist (rsb_blocks_max)
    size_t rs_btab;      // uint4 [rsb_blocks_max] row-span pass B's blocks: {first span, row | spans << 16,
                         // the row's first block, the next row's first block} (the count kernel writes it)
    size_t totals;  // uint32 [RADIX]
    size_t totals1; // uint32 [RADIX] the first tile pass's digit totals (the second pass's segments)
    size_t seg_table; // uint32 [2][RADIX + 1] the second pass's segment table: first block, first item
                      // (row-span pass B: per tile row; [RADIX] = blocks, [2 RADIX + 1] = spans)
    size_t qmask;   // uint64 [4][qmask_stride] per quadrant, per 64-entry chunk of its tile's list: the
                    // entries that reach the quadrant (render_fwd's cull), for render_bwd (qmask_index)
    size_t qmask_stride;
    // split replay (render_bwd.hip): per checkpoint slot (split_slot), per quadrant and
    // pixel, the forward's {T, C} before the slot's list position; per split tile (the
    // slot of its first checkpoint) the final {C, T}; the tile of each slot
    size_t ckpt;    // float4 [split_slots][4][64]
    size_t cfin;    // float4 [split_slots][4][64]
    size_t ctab;    // uint32 [split_slots]
    size_t bytes;
};

// ---- split replay: the backward of a long tile list in segments (render_bwd.hip)
// A wave replays its quadrant's list serially, so a tile far longer than the
// average load per wave slot sets the kernel's time on its own (config B: 743
// entries against a mean of 125).  The forward stores each pixel's T and colour
// at every SEG-th list position of a list longer than SEG; the backward then
// replays segment k ([k SEG, (k + 1) SEG)) of such a list in a wave of its own,
// starting from that state.  SEG balances the longest segment against the average
// wave-slot load 4 I / SPLIT_SLOTS (256 CUs x 4 SIMDs x 6 waves); lists are never
// split when that exceeds SPLIT_MAX (the longest lists then hold a small share of a
// wave slot's load: config C, E).
#ifndef GSR_SPLIT_SLOTS
#define GSR_SPLIT_SLOTS 6144
#endif
constexpr int SPLIT_MIN = 128, SPLIT_MAX = 1024;
constexpr int SPLIT_SLOT_CAP = 4096;  // checkpoint slots at most (8 KB each)
// checkpoint slots of a binning buffer of capacity cap (every SEG the buffer allows)
__host__ __device__ inline int64_t split_slots(int64_t cap) {
    const int64_t s = cap / SPLIT_MIN;
    return (s < SPLIT_SLOT_CAP ? s : SPLIT_SLOT_CAP) + 2;
}
__host__ __device__ inline int64_t pow2_at_least(int64_t v) {
    int64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}
// the smallest SEG the buffer's slots allow (a power of two: render_fwd tests chunk
// positions against it with a mask)
__host__ __device__ inline int split_seg_min(int64_t cap) {
    const int64_t q = (cap + SPLIT_SLOT_CAP - 1) / SPLIT_SLOT_CAP;
    return (int)pow2_at_least(q > SPLIT_MIN ? q : SPLIT_MIN);
}
// SEG for a forward into capacity cap: mode < 0 automatic, 0 off, > 0 that length
// (raised to a power of two >= 64 the buffer allows); 0 = no split
__host__ inline int split_seg(int64_t cap, int mode) {
    if (mode == 0 || cap <= 0) return 0;
    int64_t s = pow2_at_least(mode > 0 ? (int64_t)mode : 4 * cap / GSR_SPLIT_SLOTS);
    if (s < split_seg_min(cap)) s = split_seg_min(cap);
    if (mode < 0 && s > SPLIT_MAX) return 0;
    return (int)s;
}
// the slot of list position p (= r.x + k SEG, k >= 1, p < r.y) of a sorted list:
// distinct for every (tile, k) — a later tile's first checkpoint lies more than
// SEG past an earlier tile's last — and at most cap / SEG
__host__ __device__ inline uint32_t split_slot(uint32_t p, uint32_t seg) { return p / seg; }
// The chunk-mask slot of quadrant w's chunk j of tile t (list range r): (r.x >> 6) + t + j
// is distinct for every (tile, chunk) of a sorted list whose tile ranges follow each
// other (tile t + 1 starts at r.y: (r.y >> 6) + 1 >= (r.x >> 6) + ceil((r.y - r.x) / 64)),
// and below cap / 64 + tiles + 1.
__host__ __device__ inline size_t qmask_index(uint32_t rx, int tile, int j) {
    return (size_t)(rx >> 6) + (size_t)tile + (size_t)j;
}
__host__ __device__ inline BinningLayout binning_layout(int64_t cap, int W, int H) {
    BinningLayout L;
    size_t n = (size_t)(cap > 0 ? cap : 1);
    size_t o = 0;
    auto take = [&](size_t b) { size_t r = o; o = align_up(o + b, 256); return r; };
    L.off[GSR_BIN_POINT_LIST] = take(n * 4);
    L.off[GSR_BIN_KEYS] = take(n * 4);
    L.keys_b = take(n * 4);
    L.vals_b = take(n * 4);
    const GridDims gd = grid_dims(W, H);
    const size_t lsd = (size_t)radix_blocks((int64_t)n, tsort_items((int64_t)n)) + RADIX;
    L.hist_stride = (size_t)rsb_blocks_max((int64_t)n, gd.gy);
    L.hist = take((size_t)RADIX * (lsd > L.hist_stride ? lsd : L.hist_stride) * 4);
    L.totals = take((size_t)RADIX * 4);
    L.totals1 = take((size_t)RADIX * 4);
    L.seg_table = take((size_t)2 * (RADIX + 1) * 4);
    L.off[GSR_BIN_ROWSPAN] = L.seg_table;
    L.rs_btab = take(L.hist_stride * 16);
    L.qmask_stride = n / 64 + (size_t)grid_dims(W, H).tiles + 2;
    L.qmask = take(4 * L.qmask_stride * 8);
    const size_t ns = (size_t)split_slots((int64_t)n);
    L.ckpt = take(ns * 4 * 64 * 16);
    L.cfin = take(ns * 4 * 64 * 16);
    L.ctab = take((ns + 2) * 4);  // (+ 2: render_bwd reads the word of every slot workgroup, an even count)
    L.bytes = o;
    return L;
}

struct ImgLayout {
    size_t off[GSR_IMG_NFIELDS];
    size_t qlist;   // uint32 [8][32][maxc] quadrants filed by XCD and forward work (gsr_blend.hpp)
    size_t qbucket; // uint8 [4 * tiles] each quadrant's forward work bucket (render_fwd.hip)
    size_t l1_part; // float [L1_BLOCKS][2] the L1 loss's partial sums (gsr_forward_render_l1, gsr_l1.hpp)
    size_t l1_ticket; // uint32 [L1_TICKETS] the partial-sum blocks' finish tickets (zeroed by render_fwd_kernel)
    size_t l1_sign; // int8 [3][H][W] sign(image - gt), written beside the partial sums for the L1-seeded backward
    size_t bytes;
};
__host__ __device__ inline ImgLayout img_layout(int W, int H) {
    ImgLayout L;
    const GridDims g = grid_dims(W, H);
    size_t o = 0;
    auto take = [&](size_t b) { size_t r = o; o = align_up(o + b, 256); return r; };
    L.off[GSR_IMG_FINAL_T] = take((size_t)W * H * 4);
    L.off[GSR_IMG_N_CONTRIB] = take((size_t)W * H * 4);
    // per (XCD, bucket) room for every quadrant of the XCD (the longest list <= T / 2 + 16)
    L.qlist = take((size_t)8 * 32 * ((size_t)g.tiles / 2 + 16) * 4);
    L.qbucket = take((size_t)g.tiles * 4);
    L.l1_part = take((size_t)1024 * 2 * 4);
    L.l1_ticket = take(9 * 128);  // gsr_l1.hpp: L1_TICKETS words, 128 B apart
    L.l1_sign = take((size_t)3 * W * H);
    L.bytes = o;
    return L;
}

constexpr int ACCUM_STRIDE = GSR_ACCUM_STRIDE;  // floats per Gaussian in the backward accumulator (64 B row)
// flag words after the 8 x 32 wave-order counts in GeomLayout::order_cnt
enum OrderFlag {
    ORDER_FILED = 8 * 32,  // the quadrants are filed in img.qlist (by the forward's prepare or a backward)
    ORDER_FRESH,           // geom's accumulator is zeroed and unused (the forward's prepare; render_bwd clears it)
};
enum AccumSlot {
    ACC_MEAN2D_X = 0,
    ACC_MEAN2D_Y,
    ACC_CONIC_X,
    ACC_CONIC_Y,
    ACC_CONIC_W,
    ACC_OPACITY,
    ACC_COLOR_R,
    ACC_COLOR_G,
    ACC_COLOR_B,
    ACC_NVALS
};

template <typename T>
__host__ __device__ inline T *at(void *base, size_t off) {
    return reinterpret_cast<T *>(reinterpret_cast<char *>(base) + off);
}
template <typename T>
__host__ __device__ inline const T *at(const void *base, size_t off) {
    return reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + off);
}

// ---------------------------------------------------------------- device math
__device__ constexpr float SH_C0 = 0.28209479177387814f;
__device__ constexpr float SH_C1 = 0.4886025119029199f;
__device__ constexpr float SH_C2_0 = 1.0925484305920792f;
__device__ constexpr float SH_C2_1 = -1.0925484305920792f;
__device__ constexpr float SH_C2_2 = 0.31539156525252005f;
__device__ constexpr float SH_C2_3 = -1.0925484305920792f;
__device__ constexpr float SH_C2_4 = 0.5462742152960396f;
__device__ constexpr float SH_C3_0 = -0.5900435899266435f;
__device__ constexpr float SH_C3_1 = 2.890611442640554f;
__device__ constexpr float SH_C3_2 = -0.4570457994644658f;
__device__ constexpr float SH_C3_3 = 0.3731763325901154f;
__device__ constexpr float SH_C3_4 = -0.4570457994644658f;
__device__ constexpr float SH_C3_5 = 1.445305721320277f;
__device__ constexpr float SH_C3_6 = -0.5900435899266435f;

// The SH basis at the unit direction (x, y, z) for degree <= 3 (coefficients
// past (deg+1)^2 are left alone): dL/dsh[k][c] = b[k] * dL/dRGB[c] is the SH
// part of backward.cu computeColorFromSH.  Shared by preprocess_bwd (one view)
// and sh_exchange (the sum over views), so both form bit-identical products.
__device__ __forceinline__ void sh_basis(int deg, float x, float y, float z, float b[16]) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    b[0] = SH_C0;
    if (deg > 0) {
        b[1] = -SH_C1 * y;
        b[2] = SH_C1 * z;
        b[3] = -SH_C1 * x;
        if (deg > 1) {
            b[4] = SH_C2_0 * xy;
            b[5] = SH_C2_1 * yz;
            b[6] = SH_C2_2 * (2.f * zz - xx - yy);
            b[7] = SH_C2_3 * xz;
            b[8] = SH_C2_4 * (xx - yy);
            if (deg > 2) {
                b[9] = SH_C3_0 * y * (3.f * xx - yy);
                b[10] = SH_C3_1 * xy * z;
                b[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
                b[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                b[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
                b[14] = SH_C3_5 * z * (xx - yy);
                b[15] = SH_C3_6 * x * (xx - 3.f * yy);
            }
        }
    }
}

// backward.cu computeColorFromSH (backward): the derivatives of the SH colour with
// respect to the normalised view direction, dRGB/dx, dRGB/dy, dRGB/dz per
// channel, J[3 axis + c].  The forward (preprocess, when a backward will follow)
// and the backward (otherwise) evaluate them with this one function, so the
// stored values are the backward's own bit for bit.  `sh` = the Gaussian's row.
__device__ __forceinline__ void sh_dir_jacobian(const float *sh, int deg, float x, float y, float z, float J[9]) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
#pragma unroll
    for (int c = 0; c < 3; c++) {
#define SH(k) sh[3 * (k) + c]
        float dx = 0.f, dy = 0.f, dz = 0.f;
        if (deg > 0) {
            dx = -SH_C1 * SH(3);
            dy = -SH_C1 * SH(1);
            dz = SH_C1 * SH(2);
            if (deg > 1) {
                dx += SH_C2_0 * y * SH(4) + SH_C2_2 * 2.f * -x * SH(6) + SH_C2_3 * z * SH(7) + SH_C2_4 * 2.f * x * SH(8);
                dy += SH_C2_0 * x * SH(4) + SH_C2_1 * z * SH(5) + SH_C2_2 * 2.f * -y * SH(6) + SH_C2_4 * 2.f * -y * SH(8);
                dz += SH_C2_1 * y * SH(5) + SH_C2_2 * 2.f * 2.f * z * SH(6) + SH_C2_3 * x * SH(7);
                if (deg > 2) {
                    dx += (SH_C3_0 * SH(9) * 3.f * 2.f * xy + SH_C3_1 * SH(10) * yz + SH_C3_2 * SH(11) * -2.f * xy +
                           SH_C3_3 * SH(12) * -3.f * 2.f * xz + SH_C3_4 * SH(13) * (-3.f * xx + 4.f * zz - yy) +
                           SH_C3_5 * SH(14) * 2.f * xz + SH_C3_6 * SH(15) * 3.f * (xx - yy));
                    dy += (SH_C3_0 * SH(9) * 3.f * (xx - yy) + SH_C3_1 * SH(10) * xz +
                           SH_C3_2 * SH(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3_3 * SH(12) * -3.f * 2.f * yz +
                           SH_C3_4 * SH(13) * -2.f * xy + SH_C3_5 * SH(14) * -2.f * yz +
                           SH_C3_6 * SH(15) * -3.f * 2.f * xy);
                    dz += (SH_C3_1 * SH(10) * xy + SH_C3_2 * SH(11) * 4.f * 2.f * yz +
                           SH_C3_3 * SH(12) * 3.f * (2.f * zz - xx - yy) + SH_C3_4 * SH(13) * 4.f * 2.f * xz +
                           SH_C3_5 * SH(14) * (xx - yy));
                }
            }
        }
#undef SH
        J[c] = dx;
        J[3 + c] = dy;
        J[6 + c] = dz;
    }
}

// 4x4 matrices arrive as 16 floats (row-major storage of the transposed
// matrix); like upstream they are read column-major.
struct Mat4 {
    float m[16];
};
__device__ inline Mat4 load_mat4(const float *p) {
    Mat4 r;
#pragma unroll
    for (int i = 0; i < 16; i++) r.m[i] = p[i];
    return r;
}

struct M3 {
    float m[3][3];  // glm layout m[col][row]
};

}  // namespace gsr

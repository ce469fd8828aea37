// binning.hip — depth-ordered tile binning.
//
// Replaces upstream duplicateWithKeys + cub::DeviceRadixSort::SortPairs +
// identifyTileRanges (rasterizer_impl.cu).
// Upstream emits one (tile << 32 | depth_bits, id) pair per touched tile, in
// Gaussian-index order, and stably radix-sorts all I pairs over 32 + log2(T)
// bits (~6 passes over 12-B pairs).  The resulting order inside a tile is
// (depth_bits, id).  Here the same order comes from two much cheaper sorts:
//
//  1. depth sort  — stable LSD radix sort of the P depth bit patterns with the
//                   index as value (3 passes over P when the keys span < 2^24,
//                   else 4; not over I): order[rank] = id in (depth_bits, id)
//                   order.  It needs only the view depths (depth_keys_kernel
//                   computes the keys and the first pass's digit counts itself);
//                   it runs right after preprocess, and its first digit scan also
//                   publishes num_rendered (gsr_publish.hpp).  Gaussians that
//                   preprocess culls sort anywhere: they emit nothing.
//  2. rank scan   — the tile rects gathered in rank order (rank_gather_kernel),
//                   instances per emit block, an exclusive scan of those.
//  3. emit        — each Gaussian, in rank order, writes (tile, id) for every
//                   tile of its rect (row-major, as upstream) at its offset.
//  4. tile sort   — stable LSD radix sort of the I instances by tile index
//                   (ceil(log2 T / 8) passes: 2 at 1080p and 4K).  Stability
//                   keeps rank order inside a tile, i.e. (depth_bits, id).  In
//                   the two-pass case emit already writes each instance as
//                   one byte (its low tile digit) and one word, (high tile
//                   digit << id bits) | id; the first pass sorts the words by
//                   the byte, the second sorts them by the high digit in blocks
//                   that never straddle a low digit, writing only the ids:
//                   22 B per instance over emit and both passes, instead of
//                   28 + 8 (a word each for tile and id from emit).
//  5. ranges      — from the second pass's per-block digit counts (two-pass
//                   case), else identifyTileRanges on the sorted tile keys.
//
// Steps 1-2 run in gsr_forward_preprocess, 3-5 in gsr_forward_render once the
// caller has sized the binning buffer.
//
// One radix pass = upsweep (per-block digit histogram), digit scan (one
// workgroup per digit over the blocks), downsweep (stable scatter).  Inside a
// workgroup each wave owns a contiguous quarter of the block's items and walks
// it in rounds of 64; lanes holding the same digit are found with 8 ballots
// (wave "match"), ranked with mbcnt, and a per-wave LDS counter per digit
// carries the running count from round to round — no atomics anywhere.
#pragma clang fp contract(off)

#include "gsr_colour.hpp"
#include "gsr_kernels.hpp"
#include "gsr_math.hpp"
#include "gsr_publish.hpp"
#include "gsr_radix.hpp"
#include "gsr_spans.hpp"
#include "gsr_wave.hpp"

#include <type_traits>

namespace gsr {

constexpr int RX_WAVES = RX_THREADS / 64;
static_assert(RX_THREADS == RADIX, "one thread per digit in the per-block digit loops");

struct RadixPass {
    const uint32_t *kin;   // keys (the digit source)
    const uint32_t *vin;   // values; nullptr = the item index
    uint32_t *kout;        // nullptr = keys not needed after this pass
    uint32_t *vout;
    uint32_t n;
    int shift;
    int nbits;             // significant bits of this pass's digit (<= RADIX_BITS)
    uint32_t dmask;        // (1 << nbits) - 1
    uint32_t *hist;        // [RADIX][NB] block counts -> block offsets within each digit
    uint32_t *totals;      // [RADIX]
    int NB;
    // depth sort only (nullptr / 0 otherwise): the geom control words and this
    // pass's role when the key range allows three passes instead of four
    const uint32_t *ctrl;  // GeomLayout::dsort_ctrl
    uint2 *minmax;         // first depth pass: the candidate key range per block (its digit scan reduces it)
    uint32_t *ctrl_out;    // ... into these control words
    uint32_t *host_ctrl;   // ... and the pass count into the caller's pinned words (CTRL_DSORT_PASSES), or NULL
    int role;              // RX_PLAIN, RX_DEPTH_FIRST, RX_DEPTH_THIRD, RX_DEPTH_FOURTH
    uint32_t *vout_final;  // RX_DEPTH_THIRD in three-pass mode: the order lands here
    // packed two-pass tile sort (tile_sort_packed): the first pass (RXM_PACK)
    // takes byte keys (kin as uint8: the low tile digit) and moves the packed
    // words (high tile digit << id_bits | id) emit wrote as values; the second
    // (RXM_UNPACK) reads those words (digit = word >> shift, value = the id bits)
    // in blocks aligned to the first pass's digit runs (seg_totals: 2^seg_bits
    // segments, one low tile digit each) and fills the T tile ranges
    const uint32_t *seg_totals;
    uint32_t *seg_table;   // [2][RADIX + 1]: RXM_PACK's block 0 writes it, RXM_UNPACK reads it
    int seg_bits;
    int id_bits;
    uint2 *ranges;
    int T;
    // grouped depth passes (dsort_grouped, passes 2-4): hist holds block rows
    // [NB][RADIX], sup the digit counts per group of DSORT_SB blocks [nsup][RADIX]
    // (zeroed by depth_keys_kernel); no digit-scan launch.  NULL otherwise.
    uint32_t *sup;
    int nsup;
    // first depth pass after preprocess: one more digit-scan workgroup publishes
    // num_rendered (gsr_publish.hpp) from preprocess's block sums; NULL otherwise
    const uint4 *pub_sums;
    int pub_n;
    uint32_t *pub_ctrl, *pub_host;
    // tile sort queued before the host knows num_rendered (gsr_forward): n is the
    // buffer's capacity and every kernel works on the published count instead
    SpecGuard g;
    // digit scan over a block count the device computed (row-span pass B): NB is
    // then the hist stride and *nb_dev (<= NB) the blocks to scan; the scan does
    // nothing unless the speculative guard holds
    const uint32_t *nb_dev;
    // depth sort with the rect footprint's words carried beside the ids (the
    // row-span binning, gsr_spans.hpp rect_word): the first pass packs them from
    // the rects (rin), the later ones move them (win -> wout; the last pass into
    // wout_final, in rank order).  NULL otherwise (a downsweep without carry).
    const uint4 *rin;
    const uint32_t *win;
    uint32_t *wout, *wout_final;
    // grouped first pass whose key base depth_keys_kernel's publishing workgroup
    // already wrote (from preprocess's per-workgroup key ranges): no block reduces it
    int base_published;
    // the colour half of preprocess riding this downsweep (gsr_colour.hpp): its
    // ride.nb workgroups follow the NB sorting ones in the grid; nb == 0 = none
    ColourRide ride;
};
enum RadixRole { RX_PLAIN = 0, RX_DEPTH_FIRST, RX_DEPTH_THIRD, RX_DEPTH_FOURTH };
enum RadixMode { RXM_KV = 0, RXM_PACK, RXM_UNPACK };

// First depth pass: key = depth bits - base (base = the smallest candidate key
// with its low byte cleared, so the key's low byte — this pass's digit, which
// depth_keys_kernel counted before the base was known — is the raw bits' own);
// in three-pass mode keys beyond 2^24 (only non-candidates, +inf keys, reach it)
// saturate their top 16 bits and keep that low byte: every pass then sorts by the
// digits of one and the same key.
__device__ __forceinline__ uint32_t key_rel(uint32_t k, uint32_t base, uint32_t passes);
__device__ __forceinline__ uint32_t key_of(const RadixPass &a, uint32_t k) {
    if (a.role != RX_DEPTH_FIRST) return k;
    return key_rel(k, a.ctrl[DCTRL_KEY_BASE], a.ctrl[DCTRL_PASSES]);
}
__device__ __forceinline__ uint32_t load_key(const RadixPass &a, uint32_t idx) { return key_of(a, a.kin[idx]); }
__device__ __forceinline__ bool pass_skipped(const RadixPass &a) {
    return a.role == RX_DEPTH_FOURTH && a.ctrl[DCTRL_PASSES] == 3;
}

// (dsort_base_passes: gsr_publish.hpp)
__device__ __forceinline__ uint32_t key_rel(uint32_t k, uint32_t base, uint32_t passes) {
    const uint32_t d = k - base;
    return passes == 3 && d > 0xffffffu ? (0xffff00u | (d & 0xffu)) : d;
}

// The second pass's segment table from the first pass's digit totals: segment
// (low tile digit) s starts at block sfb[s] and item sst[s]; [RADIX] = the totals.
// Written once, by the first pass's block 0 (its downsweep reads the totals
// anyway), so the second pass's blocks load it instead of each scanning the totals.
template <int TILE_N>
__device__ __forceinline__ void write_seg_table(const RadixPass &a, uint32_t *wsum) {
    const uint32_t c = (int)threadIdx.x < (1 << a.nbits) ? a.totals[threadIdx.x] : 0u;
    const uint32_t nb = (c + (uint32_t)TILE_N - 1u) / (uint32_t)TILE_N;
    uint32_t totb, totc;
    const uint32_t ib = block_inclusive_scan<RX_THREADS>(nb, wsum, &totb);
    const uint32_t ic = block_inclusive_scan<RX_THREADS>(c, wsum, &totc);
    a.seg_table[threadIdx.x] = ib - nb;
    a.seg_table[RADIX + 1 + threadIdx.x] = ic - c;
    if (threadIdx.x == 0) {
        a.seg_table[RADIX] = totb;
        a.seg_table[2 * RADIX + 1] = totc;
    }
}

// Items [x, y) of radix block blk.  Plain: TILE_N items per block.  RXM_UNPACK:
// each segment (one digit run of the previous pass) starts a new block, so a
// block's instances share their low tile digit and the digit counts per block
// give the tile ranges; sfb / sst [RADIX + 1] (LDS) receive each segment's first
// block and first item (the table write_seg_table left).  The grid has
// radix_blocks(n) + 2^seg_bits blocks, the unused tail ones are empty.
template <int TILE_N, int MODE>
__device__ __forceinline__ uint2 block_span(const RadixPass &a, uint32_t blk, uint32_t *sfb, uint32_t *sst,
                                            uint32_t *wsum) {
    if constexpr (MODE != RXM_UNPACK) {
        const uint32_t n = spec_count(a.g, a.n), b0 = blk * (uint32_t)TILE_N;
        return b0 < n ? make_uint2(b0, min(b0 + (uint32_t)TILE_N, n)) : make_uint2(0u, 0u);
    } else {
        (void)wsum;
        sfb[threadIdx.x] = a.seg_table[threadIdx.x];
        sst[threadIdx.x] = a.seg_table[RADIX + 1 + threadIdx.x];
        if (threadIdx.x == 0) {
            sfb[RADIX] = a.seg_table[RADIX];
            sst[RADIX] = a.seg_table[2 * RADIX + 1];
        }
        __syncthreads();
        int sg = 0;  // the last segment whose first block is <= blk (sfb is non-decreasing, sfb[0] = 0)
#pragma unroll
        for (int step = RADIX / 2; step >= 1; step >>= 1)
            if (sfb[sg + step] <= blk) sg += step;
        const uint32_t b0 = sst[sg] + (blk - sfb[sg]) * (uint32_t)TILE_N, send = sst[sg + 1];
        return b0 < send ? make_uint2(b0, min(b0 + (uint32_t)TILE_N, send)) : make_uint2(0u, 0u);
    }
}

// ITEMS per thread: fewer for short inputs (more workgroups, shorter serial
// rank chains), more for long ones (fewer blocks in the digit scan).
template <int ITEMS, int MODE>
__global__ void __launch_bounds__(RX_THREADS) radix_upsweep_kernel(RadixPass a) {
    constexpr int TILE_N = RX_THREADS * ITEMS;
    constexpr int SEG = MODE == RXM_UNPACK ? RADIX + 1 : 1;
    __shared__ uint32_t h[RX_WAVES][RADIX];
    __shared__ uint32_t sfb[SEG], sst[SEG], wsum[RX_WAVES];
    if (pass_skipped(a)) return;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < RX_WAVES; k++) h[k][threadIdx.x] = 0;
    const uint32_t blk = radix_block(a.NB);
    const uint2 span = block_span<TILE_N, MODE>(a, blk, sfb, sst, wsum);
    __syncthreads();
    if constexpr (MODE == RXM_PACK) {
        // byte keys: 16 per 16-B load over the block's 16-B aligned body, single
        // bytes for its ragged tail (blocks start at multiples of TILE_N)
        const uint8_t *k8 = reinterpret_cast<const uint8_t *>(a.kin);
        const uint32_t v1 = span.y & ~15u;
        const uint4 *k4 = reinterpret_cast<const uint4 *>(k8);
        auto count4 = [&](uint32_t word) {
#pragma unroll
            for (int b = 0; b < 4; b++) atomicAdd(&h[w][(word >> (8 * b)) & a.dmask], 1u);
        };
        for (uint32_t qi = (span.x >> 4) + threadIdx.x; qi < (v1 >> 4); qi += RX_THREADS) {
            const uint4 q = k4[qi];
            count4(q.x);
            count4(q.y);
            count4(q.z);
            count4(q.w);
        }
        if (threadIdx.x < span.y - v1) atomicAdd(&h[w][k8[v1 + threadIdx.x] & a.dmask], 1u);
        __syncthreads();
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < RX_WAVES; k++) c += h[k][threadIdx.x];
        a.hist[(size_t)threadIdx.x * a.NB + blk] = c;
        return;
    }
    // order-free count: 16-B loads over the block's 16-B aligned body (ITEMS / 4
    // per thread), single keys for its ragged head and tail (< 4 each)
    static_assert(ITEMS % 4 == 0, "quads");
    const uint32_t v0 = min((span.x + 3u) & ~3u, span.y), v1 = max(span.y & ~3u, v0);
    const uint4 *k4 = reinterpret_cast<const uint4 *>(a.kin);
    uint4 q[ITEMS / 4];
#pragma unroll
    for (int r = 0; r < ITEMS / 4; r++) {
        const uint32_t qi = (v0 >> 2) + threadIdx.x + (uint32_t)(r * RX_THREADS);
        q[r] = qi < (v1 >> 2) ? k4[qi] : make_uint4(0u, 0u, 0u, 0u);
    }
    auto count = [&](uint32_t k) { atomicAdd(&h[w][(key_of(a, k) >> a.shift) & a.dmask], 1u); };
#pragma unroll
    for (int r = 0; r < ITEMS / 4; r++) {
        if ((v0 >> 2) + threadIdx.x + (uint32_t)(r * RX_THREADS) < (v1 >> 2)) {
            count(q[r].x);
            count(q[r].y);
            count(q[r].z);
            count(q[r].w);
        }
    }
    if (threadIdx.x < v0 - span.x) count(a.kin[span.x + threadIdx.x]);
    if (threadIdx.x < span.y - v1) count(a.kin[v1 + threadIdx.x]);
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < RX_WAVES; k++) c += h[k][threadIdx.x];
    if (a.sup) {  // grouped: the block's row, and its group's running counts
        a.hist[(size_t)blk * RADIX + threadIdx.x] = c;
        if (c) atomicAdd(&a.sup[(size_t)(blk >> DSORT_SB_LOG2) * RADIX + threadIdx.x], c);
    } else {
        a.hist[(size_t)threadIdx.x * a.NB + blk] = c;
    }
}

// One workgroup per digit: exclusive scan of that digit's block counts.
// One workgroup per digit, 1024 threads x 16 entries per round (coalesced,
// wave-chained: block_exclusive_scan_inplace).  The config-E tile sort's scans of
// 14.8k block counts: 27.7 us each as one block scan per 256 entries, 8.2 us like
// this (256 x 16: 9.9, 512 x 8: 9.0, 1024 x 4: 8.8).
constexpr int DSCAN_THREADS = 1024, DSCAN_PER = 16;
static_assert(DSCAN_THREADS == TOTAL_THREADS, "the publish workgroup runs in the digit scan's launch");
__global__ void __launch_bounds__(DSCAN_THREADS) radix_digit_scan_kernel(RadixPass a) {
    __shared__ uint32_t wsum[DSCAN_THREADS / 64];
    if (blockIdx.x == RADIX + 1) {  // (grid RADIX + 2 only with pub_sums)
        publish_total(a.pub_sums, a.pub_n, a.pub_ctrl, a.pub_host);
        return;
    }
    if (blockIdx.x == RADIX) {  // first depth pass: one more workgroup reduces the candidate key range
        __shared__ uint32_t wmin[DSCAN_THREADS / 64], wmax[DSCAN_THREADS / 64];
        uint32_t kmin = 0xffffffffu, kmax = 0u;
        for (int i = threadIdx.x; i < a.NB; i += DSCAN_THREADS) {
            const uint2 m = a.minmax[i];
            kmin = min(kmin, m.x);
            kmax = max(kmax, m.y);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
            kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        }
        if ((threadIdx.x & 63) == 0) {
            wmin[threadIdx.x >> 6] = kmin;
            wmax[threadIdx.x >> 6] = kmax;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < DSCAN_THREADS / 64; k++) {
                kmin = min(kmin, wmin[k]);
                kmax = max(kmax, wmax[k]);
            }
            const uint2 bp = dsort_base_passes(kmin, kmax);
            const uint32_t base = bp.x, passes = bp.y;
            a.ctrl_out[DCTRL_KEY_BASE] = base;
            a.ctrl_out[DCTRL_PASSES] = passes;
            if (a.host_ctrl) {  // the host launches the fourth pass only when it is needed
                __hip_atomic_store(&a.host_ctrl[CTRL_DSORT_PASSES], passes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
            }
        }
        return;
    }
    if (pass_skipped(a)) return;
    if (a.nb_dev && !spec_ok(a.g)) return;
    const int n = a.nb_dev ? (int)min(*a.nb_dev, (uint32_t)a.NB) : a.NB;
    const uint32_t tot =
        block_exclusive_scan_inplace<DSCAN_THREADS, DSCAN_PER>(a.hist + (size_t)blockIdx.x * a.NB, n, wsum);
    if (threadIdx.x == 0) a.totals[blockIdx.x] = tot;
}

// Exclusive scan of each of `digits` count rows hist[d][0, n) in place (stride
// NB; n = *nb_dev when given), totals[d] = the row's sum: the digit scan of the
// row-span passes (rowspan.hip).
hipError_t launch_count_scan(uint32_t *hist, int NB, const uint32_t *nb_dev, uint32_t *totals, int digits,
                             const SpecGuard &g, hipStream_t s) {
    RadixPass a = {};
    a.hist = hist;
    a.NB = NB;
    a.nb_dev = nb_dev;
    a.totals = totals;
    a.role = RX_PLAIN;
    a.g = g;
    hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(digits), dim3(DSCAN_THREADS), 0, s, a);
    return hipGetLastError();
}

template <int ITEMS, int MODE, bool CARRY = false, bool RIDE = false>
__global__ void __launch_bounds__(RX_THREADS) radix_downsweep_kernel(RadixPass a) {
    if constexpr (RIDE) {
        // colour riders: the workgroups past the sorting ones.  The sort is bound by
        // its launch and dependency latency and leaves most of the chip idle; the
        // colour half streams the SH rows meanwhile, in the same launch (no second
        // queue).  Whole workgroups return here, before any barrier.
        if ((int)blockIdx.x >= a.NB) {
            const int cb = a.ride.b0 + (int)blockIdx.x - a.NB;
            if (a.ride.sh_rest)
                colour_rows48<true>(a.ride, cb);
            else
                colour_rows48<false>(a.ride, cb);
            return;
        }
    }
    constexpr int TILE_N = RX_THREADS * ITEMS, WAVE_N = TILE_N / RX_WAVES;
    constexpr int SEG = MODE == RXM_UNPACK ? RADIX + 1 : 1;
    __shared__ uint32_t cnt[RX_WAVES][RADIX];
    // global start of this block's run of each digit, minus the run's start in
    // the block (so an item's output position is gshift[digit] + its block slot)
    __shared__ uint32_t gshift[RADIX];
    __shared__ uint32_t dstart[SEG];     // RXM_UNPACK: global start of each digit
    __shared__ uint32_t wsum[RX_WAVES];
    __shared__ uint32_t sfb[SEG], sst[SEG];
    // RXM_UNPACK stages the packed words alone (the value is in the word)
    __shared__ uint32_t stage_k[TILE_N], stage_v[MODE == RXM_UNPACK ? 1 : TILE_N], stage_w[CARRY ? TILE_N : 1];
    if (pass_skipped(a)) return;
    // A grouped first depth pass has no digit scan to reduce the candidate key
    // range: every block reduces the per-block ranges itself (the same operations,
    // so the same base and pass count everywhere), and block 0 publishes them
    uint2 bp = make_uint2(0u, 0u);
    const bool local_base = MODE == RXM_KV && a.role == RX_DEPTH_FIRST && a.sup != nullptr && !a.base_published;
    if (local_base) {
        uint32_t kmin = 0xffffffffu, kmax = 0u;
        for (int i = threadIdx.x; i < a.NB; i += RX_THREADS) {
            const uint2 m = a.minmax[i];
            kmin = min(kmin, m.x);
            kmax = max(kmax, m.y);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
            kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        }
        if ((threadIdx.x & 63) == 0) {
            stage_k[threadIdx.x >> 6] = kmin;
            stage_k[RX_WAVES + (threadIdx.x >> 6)] = kmax;
        }
        __syncthreads();
        for (int k = 0; k < RX_WAVES; k++) {
            kmin = min(kmin, stage_k[k]);
            kmax = max(kmax, stage_k[RX_WAVES + k]);
        }
        bp = dsort_base_passes(kmin, kmax);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            a.ctrl_out[DCTRL_KEY_BASE] = bp.x;
            a.ctrl_out[DCTRL_PASSES] = bp.y;
            if (a.host_ctrl) {  // the host launches the fourth pass only when it is needed
                __hip_atomic_store(&a.host_ctrl[CTRL_DSORT_PASSES], bp.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
            }
        }
        __syncthreads();  // (stage_k is reused below)
    }
    // three-pass depth sort: the third pass is the last one
    const bool final3 = a.role == RX_DEPTH_THIRD && a.ctrl[DCTRL_PASSES] == 3;
    uint32_t *const kout = final3 ? nullptr : a.kout;
    uint32_t *const vout = final3 ? a.vout_final : a.vout;
    uint32_t *const wout = final3 ? a.wout_final : a.wout;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t blk = radix_block(a.NB);
    const uint2 span = block_span<TILE_N, MODE>(a, blk, sfb, sst, wsum);
    const uint32_t b0 = span.x;
    const uint32_t base = b0 + w * (uint32_t)WAVE_N + lane;
    // where this block's items of digit d go: all smaller digits + earlier blocks.
    // The grouped prefix is summed before the item loads (its 16-B row loads and
    // the items would otherwise be live together: 112 instead of 57 VGPRs).
    uint32_t t, before;
    bool grouped = false;
    if constexpr (MODE == RXM_KV) grouped = a.sup != nullptr;
    if (grouped) {
        // grouped: the groups before this block's, then its group's blocks before
        // it.  Wave w sums the rows w, w + 4, ... (a lane: 4 digits, one 16-B
        // load per row, every load of the wave in flight at once); the four
        // partial sums meet in LDS (the stages, not yet in use).
        const uint32_t g = blk >> DSORT_SB_LOG2, g0 = g << DSORT_SB_LOG2;
        auto add4 = [](uint4 &s, uint4 v, bool on) {
            s.x += on ? v.x : 0u;
            s.y += on ? v.y : 0u;
            s.z += on ? v.z : 0u;
            s.w += on ? v.w : 0u;
        };
        uint4 t4 = make_uint4(0u, 0u, 0u, 0u), b4 = t4;
        const uint4 *sup4 = reinterpret_cast<const uint4 *>(a.sup), *hist4 = reinterpret_cast<const uint4 *>(a.hist);
        for (int q0 = 0; q0 < a.nsup; q0 += 4 * RX_WAVES) {
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = sup4[(size_t)min(q0 + 4 * k + w, a.nsup - 1) * (RADIX / 4) + lane];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int q = q0 + 4 * k + w;
                add4(t4, v[k], q < a.nsup);
                add4(b4, v[k], (uint32_t)q < g);
            }
        }
        {
            constexpr int PER = DSORT_SB / RX_WAVES;  // rows of the group per wave, 4 loads at a time
#pragma unroll
            for (int k0 = 0; k0 < PER; k0 += 4) {
                uint4 v[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t j = g0 + (uint32_t)(RX_WAVES * (k0 + k) + w);
                    v[k] = hist4[(size_t)(j < blk ? j : 0u) * (RADIX / 4) + lane];
                }
#pragma unroll
                for (int k = 0; k < 4; k++) add4(b4, v[k], g0 + (uint32_t)(RX_WAVES * (k0 + k) + w) < blk);
            }
        }
        static_assert(TILE_N >= RX_WAVES * RADIX, "the stages hold the partial sums");
        reinterpret_cast<uint4 *>(stage_k)[w * 64 + lane] = t4;
        reinterpret_cast<uint4 *>(stage_v)[w * 64 + lane] = b4;
        __syncthreads();
        t = 0u;
        before = 0u;
#pragma unroll
        for (int k = 0; k < RX_WAVES; k++) {
            t += stage_k[k * RADIX + threadIdx.x];
            before += stage_v[k * RADIX + threadIdx.x];
        }
        __syncthreads();
    }
    uint32_t kk[ITEMS], vv[MODE == RXM_UNPACK ? 1 : ITEMS], rk[ITEMS], ww[CARRY ? ITEMS : 1];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const uint32_t idx = base + 64u * r;
        const bool ok = idx < span.y;
        if constexpr (MODE == RXM_PACK)
            kk[r] = ok ? (uint32_t)reinterpret_cast<const uint8_t *>(a.kin)[idx] : 0u;
        else
            kk[r] = ok ? (local_base ? key_rel(a.kin[idx], bp.x, bp.y) : load_key(a, idx)) : 0u;
        if constexpr (MODE != RXM_UNPACK) vv[r] = a.vin ? (ok ? a.vin[idx] : 0u) : idx;
        if constexpr (CARRY) ww[r] = ok ? (a.win ? a.win[idx] : rect_word(a.rin[idx])) : 0u;
    }
    {
        if (!grouped) {
            t = a.totals[threadIdx.x];
            before = a.hist[(size_t)threadIdx.x * a.NB + blk];
        }
        uint32_t tot;
        const uint32_t inc = block_inclusive_scan<RX_THREADS>(t, wsum, &tot);
        gshift[threadIdx.x] = inc - t + before;
        if constexpr (MODE == RXM_UNPACK) dstart[threadIdx.x] = inc - t;
    }
    if constexpr (MODE == RXM_PACK)
        if (blk == 0) write_seg_table<TILE_N>(a, wsum);
#pragma unroll
    for (int k = 0; k < RX_WAVES; k++) cnt[k][threadIdx.x] = 0;
    __syncthreads();
    // stable ranks inside each wave's quarter (the bit count as a compile-time
    // constant: 6 / 7 / 8-bit passes, anything else compares 8)
    auto rank_items = [&](auto nbits) {
        constexpr int NB = decltype(nbits)::value;
#pragma unroll
        for (int r = 0; r < ITEMS; r++) {
            const bool ok = base + 64u * r < span.y;
            const uint64_t live = __ballot(ok);
            if (!live) break;
            const uint32_t d = (kk[r] >> a.shift) & a.dmask;
            const uint64_t peers = match_digit<NB>(d, live);
            const uint32_t below = count_below(peers);
            const uint32_t c = cnt[w][d];
            rk[r] = c + below;
            if (ok && below == 0) cnt[w][d] = c + (uint32_t)__popcll(peers);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
    };
    if (a.nbits == 6)
        rank_items(std::integral_constant<int, 6>{});
    else if (a.nbits == 7)
        rank_items(std::integral_constant<int, 7>{});
    else
        rank_items(std::integral_constant<int, RADIX_BITS>{});
    __syncthreads();
    {  // block-local digit runs, and each wave's start inside its digit's run
        uint32_t c[RX_WAVES], sum = 0;
#pragma unroll
        for (int k = 0; k < RX_WAVES; k++) {
            c[k] = cnt[k][threadIdx.x];
            sum += c[k];
        }
        uint32_t tot;
        const uint32_t start = block_inclusive_scan<RX_THREADS>(sum, wsum, &tot) - sum;
        gshift[threadIdx.x] -= start;  // this thread's own digit
        uint32_t off = start;
#pragma unroll
        for (int k = 0; k < RX_WAVES; k++) {
            cnt[k][threadIdx.x] = off;
            off += c[k];
        }
    }
    __syncthreads();
    // block-sorted image in LDS ...
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        if (base + 64u * r < span.y) {
            const uint32_t d = (kk[r] >> a.shift) & a.dmask;
            const uint32_t p = cnt[w][d] + rk[r];
            stage_k[p] = kk[r];
            if constexpr (MODE != RXM_UNPACK) stage_v[p] = vv[r];
            if constexpr (CARRY) stage_w[p] = ww[r];
        }
    }
    __syncthreads();
    // ... written out in order: each digit's run is contiguous in the output too
    const uint32_t nb = span.y - b0;
    for (uint32_t i = threadIdx.x; i < nb; i += RX_THREADS) {
        const uint32_t k = stage_k[i];
        const uint32_t d = (k >> a.shift) & a.dmask;
        const uint32_t pos = gshift[d] + i;
        if constexpr (MODE == RXM_UNPACK) {
            vout[pos] = k & ((1u << a.id_bits) - 1u);
        } else if constexpr (MODE == RXM_PACK) {
            vout[pos] = stage_v[i];
        } else {
            const uint32_t v = stage_v[i];
            if (kout) kout[pos] = k;
            vout[pos] = v;
            if constexpr (CARRY) wout[pos] = stage_w[i];
        }
    }
    if constexpr (MODE == RXM_UNPACK) {
        // identifyTileRanges from the counts: tile (d, s) = digit d's items of
        // segment s, which start at segment s's first block.  After the digit scan
        // hist[d][b] = digit d's items before block b, so tile (d, s) covers
        // dstart[d] + [hist[d][sfb[s]], hist[d][sfb[s + 1]]) (totals[d] past the
        // last block).  One digit per workgroup; empty tiles get (0, 0).
        const int nseg = 1 << a.seg_bits;
        for (uint32_t d = blockIdx.x; d < (1u << a.nbits); d += gridDim.x) {
            if ((int)threadIdx.x < nseg) {
                const uint32_t sg = threadIdx.x, fb = sfb[sg], fe = sfb[sg + 1];
                const uint32_t *row = a.hist + (size_t)d * a.NB;
                const uint32_t x = fb < (uint32_t)a.NB ? row[fb] : a.totals[d];
                const uint32_t y = fe < (uint32_t)a.NB ? row[fe] : a.totals[d];
                const uint32_t tile = (d << a.seg_bits) | sg;
                if (tile < (uint32_t)a.T) a.ranges[tile] = y > x ? make_uint2(dstart[d] + x, dstart[d] + y) : make_uint2(0u, 0u);
            }
        }
    }
}

template <int ITEMS, int MODE = RXM_KV>
static hipError_t radix_pass(const RadixPass &a, hipStream_t s, bool counted = false) {
    if (a.n == 0) return hipSuccess;
    // counted: the digit counts are already in a.hist (depth_keys_kernel)
    if (!counted) hipLaunchKernelGGL((radix_upsweep_kernel<ITEMS, MODE>), dim3(a.NB), dim3(RX_THREADS), 0, s, a);
    if (!a.sup)  // grouped depth passes: each downsweep block sums its own prefix
        hipLaunchKernelGGL(radix_digit_scan_kernel, dim3(a.pub_sums ? RADIX + 2 : a.minmax ? RADIX + 1 : RADIX),
                           dim3(DSCAN_THREADS), 0, s, a);
    const bool carry = MODE == RXM_KV && (a.wout || a.wout_final);
    if (MODE == RXM_KV && a.ride.nb > 0) {
        const dim3 grid(a.NB + a.ride.nb);
        if (carry)
            hipLaunchKernelGGL((radix_downsweep_kernel<ITEMS, RXM_KV, true, true>), grid, dim3(RX_THREADS), 0, s, a);
        else
            hipLaunchKernelGGL((radix_downsweep_kernel<ITEMS, RXM_KV, false, true>), grid, dim3(RX_THREADS), 0, s, a);
    } else if (carry) {
        hipLaunchKernelGGL((radix_downsweep_kernel<ITEMS, RXM_KV, true>), dim3(a.NB), dim3(RX_THREADS), 0, s, a);
    } else {
        hipLaunchKernelGGL((radix_downsweep_kernel<ITEMS, MODE>), dim3(a.NB), dim3(RX_THREADS), 0, s, a);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------ rank-order scan

__device__ __forceinline__ uint32_t rect_area(uint4 q) {
    return ((q.x >> 16) - (q.x & 0xffffu)) * ((q.y >> 16) - (q.y & 0xffffu));
}
// instances of a Gaussian: the whole rect when its tile mask (preprocess.hip) is
// all ones (the upstream footprint, and every rect of more than 64 tiles), else
// the set bits of the mask (a tight rect of at most 64 tiles: never all ones
// below 64 tiles, and equal to the area at 64)
__device__ __forceinline__ uint32_t rect_count(uint4 q) {
    return (q.z & q.w) == ~0u ? rect_area(q) : (uint32_t)(__builtin_popcount(q.z) + __builtin_popcount(q.w));
}
// index of the k-th set bit (k < popcount) of the 64-bit mask {lo, hi}
__device__ __forceinline__ uint32_t kth_set_bit(uint32_t lo, uint32_t hi, uint32_t k) {
    uint32_t c = __builtin_popcount(lo), x = lo, base = 0;
    if (k >= c) {
        k -= c;
        x = hi;
        base = 32;
    }
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        c = __builtin_popcount(x & ((1u << w) - 1u));
        if (k >= c) {
            k -= c;
            x >>= w;
            base += w;
        }
    }
    return base;
}

// The tile rects in rank (depth) order, and where each emit block's instances
// start: one random 16-B gather per Gaussian (the depth sort's order meets
// preprocess's rects here, after both streams), the rest coalesced.  A workgroup
// covers RG_SUPER emit blocks (4,096 ranks, RG_RANKS per thread with every load
// issued first) and writes each one's instances before it within the workgroup,
// and its total; emit_kernel adds the totals of the workgroups before its own —
// so no scan launch sits between this kernel and the emission.
// Row-span binning (rs_gy > 0, rowspan.hip) instead: the spans of each pass-A
// block (RSA_GAUSS ranks) per tile row, rs_ahist[row][block] (one LDS add per span).
// With the words carried through the depth sort (rwords: the rect footprint in rank
// order, gsr_spans.hpp rect_word) the row counts read those, coalesced, and nothing
// is gathered or written beside them.
__global__ void __launch_bounds__(RG_THREADS)
    rank_gather_kernel(const uint32_t *order, const uint4 *rects, int P, uint4 *rects_ranked, uint32_t *local,
                       uint32_t *super, const uint32_t *dsort_ctrl, uint32_t *rs_ahist, int rs_nA, int rs_gy,
                       const uint32_t *rwords) {
    constexpr int AB = RG_THREADS * RG_RANKS / RSA_GAUSS;  // pass-A blocks per workgroup
    __shared__ uint32_t wsum[RG_RANKS][RG_THREADS / 64];
    __shared__ uint32_t rows[AB][RADIX];
    // queued before the host knows the pass count: a four-pass sort is not done yet
    // (the host launches its fourth pass and this kernel again)
    if (dsort_ctrl && dsort_ctrl[DCTRL_PASSES] != 3u) return;
    const int r0 = blockIdx.x * RG_THREADS * RG_RANKS + threadIdx.x;
    if (rs_gy)
        for (int i = threadIdx.x; i < AB * RADIX; i += RG_THREADS) (&rows[0][0])[i] = 0u;
    uint32_t id[RG_RANKS];
    uint4 q[RG_RANKS];
    if (rwords) {
#pragma unroll
        for (int k = 0; k < RG_RANKS; k++) {
            const int r = r0 + k * RG_THREADS;
            id[k] = r < P ? rwords[r] : 0xffu;  // (the word, not the id)
        }
    } else {
#pragma unroll
        for (int k = 0; k < RG_RANKS; k++) {
            const int r = r0 + k * RG_THREADS;
            id[k] = r < P ? order[r] : 0u;
        }
#pragma unroll
        for (int k = 0; k < RG_RANKS; k++) q[k] = r0 + k * RG_THREADS < P ? rects[id[k]] : make_uint4(0u, 0u, 0u, 0u);
    }
    if (rs_gy) {
        __syncthreads();  // the row counts are zeroed
#pragma unroll
        for (int k = 0; k < RG_RANKS; k++) {
            const int r = r0 + k * RG_THREADS;
            if (!rwords && r < P) rects_ranked[r] = q[k];
            const Foot f = rwords ? foot_of_word(id[k]) : foot_of(q[k]);
            uint32_t *h = rows[(k * RG_THREADS + threadIdx.x) / RSA_GAUSS];
            for (uint32_t y = f.y0; y < f.y1; y++)
                if (foot_row_kept(f, y - f.y0)) atomicAdd(&h[y], 1u);
        }
        __syncthreads();
        // rows[j][y] -> rs_ahist[y][block]: eight consecutive threads write one row's
        // 32-B run of this workgroup's eight blocks
        for (int i = threadIdx.x; i < AB * rs_gy; i += RG_THREADS) {
            const int y = i / AB, j = i % AB, blk = blockIdx.x * AB + j;
            if (blk < rs_nA) rs_ahist[(size_t)y * rs_nA + blk] = rows[j][y];
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < RG_RANKS; k++) {
        const int r = r0 + k * RG_THREADS;
        if (r < P) rects_ranked[r] = q[k];
        uint32_t c = rect_count(q[k]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
        if ((threadIdx.x & 63) == 0) wsum[k][threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // emit block j of the workgroup: round j / 4, threads 256 (j % 4) ...
        constexpr int WPE = EMIT_BLOCK / 64;                 // waves per emit block
        constexpr int EPR = RG_THREADS / EMIT_BLOCK;          // emit blocks per round
        const int j = threadIdx.x;
        uint32_t v = 0;
        if (j < RG_SUPER)
#pragma unroll
            for (int w = 0; w < WPE; w++) v += wsum[j / EPR][(j % EPR) * WPE + w];
        const uint32_t inc = wave_inclusive_scan(v);
        const int e = blockIdx.x * RG_SUPER + j;
        if (j < RG_SUPER && e < emit_blocks(P)) local[e] = inc - v;
        if (j == RG_SUPER - 1) super[blockIdx.x] = inc;
    }
}

// duplicateWithKeys in rank order: (tile, id) for every tile of the rect.
// The workgroup's 256 Gaussians own one contiguous run of instances.  Each thread
// takes EMIT_IPT consecutive instances: one binary search over the LDS offsets
// finds the Gaussian of the first, then the thread walks on, moving to the next
// Gaussian at each offset it passes and to the next tile incrementally (the next
// column of the rect, or the next set bit of its tile mask); the round's
// instances leave through LDS, coalesced.  Config E: 189 -> 175 us (one search
// per instance: 8 dependent LDS reads and a k-th-set-bit search each); 16
// instances per thread left too few threads busy per workgroup at config C
// (28 -> 50 us), and stores straight from the walk were uncoalesced (58 us).
#ifndef GSR_EMIT_IPT
#define GSR_EMIT_IPT 4
#endif
constexpr int EMIT_IPT = GSR_EMIT_IPT;
constexpr int EMIT_LOG2 = __builtin_ctz(EMIT_BLOCK);
struct EmitArgs {
    int P, gx;
    // packed two-pass tile sort: tile_keys receives one byte per instance (the
    // low lo_bits of its tile) and ids the word (tile >> lo_bits) << id_bits | id
    int packed, lo_bits, id_bits;
    const uint32_t *order;
    const uint4 *rects;
    const uint32_t *block_local;  // instances before the block within its rank-gather workgroup
    const uint32_t *super;        // instances per rank-gather workgroup
    uint32_t *tile_keys;
    uint32_t *ids;
    SpecGuard g;  // speculative (gsr_forward): nothing at all unless the published count fits
};
__device__ __forceinline__ uint32_t div_small(uint32_t pos, uint32_t w) {  // pos / w for pos < 2^24
    uint32_t y = (uint32_t)((float)pos * __builtin_amdgcn_rcpf((float)w));
    if (y * w > pos) y--;
    if ((y + 1) * w <= pos) y++;
    return y;
}
__global__ void __launch_bounds__(EMIT_BLOCK) emit_kernel(EmitArgs a) {
    if (!spec_ok(a.g)) return;
    __shared__ uint32_t wsum[2 * (EMIT_BLOCK / 64)];
    __shared__ uint32_t loff[EMIT_BLOCK + 1];
    __shared__ uint4 rect[EMIT_BLOCK];  // x0, width, y0, id
    __shared__ uint2 mask[EMIT_BLOCK];  // tile mask; {~0, ~0} = every tile of the rect
    const int r = blockIdx.x * EMIT_BLOCK + threadIdx.x;
    // the block's first instance: the rank-gather workgroups before its own, summed
    // here (<= 2 loads per thread up to 2M Gaussians), + its offset within its own
    uint32_t pre = 0;
    const int ns = blockIdx.x / RG_SUPER;
    for (int i = threadIdx.x; i < ns; i += EMIT_BLOCK) pre += a.super[i];
    const uint32_t loc = a.block_local[blockIdx.x];
    const uint32_t id = r < a.P ? a.order[r] : 0u;
    const uint4 q = r < a.P ? a.rects[r] : make_uint4(0u, 0u, 0u, 0u);  // rects in depth order
    const uint32_t v = rect_count(q);
    uint32_t tot;
    const uint32_t inc = block_inclusive_scan<EMIT_BLOCK>(v, wsum, &tot);
    loff[threadIdx.x] = inc - v;
    if (threadIdx.x == EMIT_BLOCK - 1) loff[EMIT_BLOCK] = tot;
    if (v) {
        rect[threadIdx.x] = make_uint4(q.x & 0xffffu, (q.x >> 16) - (q.x & 0xffffu), q.y & 0xffffu, id);
        mask[threadIdx.x] = make_uint2(q.z, q.w);
    }
    const uint32_t base = block_sum<EMIT_BLOCK>(pre, wsum + EMIT_BLOCK / 64) + loc;  // (its own barriers)
    // a round's EMIT_BLOCK x EMIT_IPT instances go through LDS (thread t's run at
    // stride EMIT_IPT + 1 words: conflict-free) and leave coalesced
    constexpr int RS = EMIT_IPT + 1;
    __shared__ uint32_t kbuf[EMIT_BLOCK * RS], ibuf[EMIT_BLOCK * RS];
    for (uint32_t r0 = 0; r0 < tot; r0 += EMIT_BLOCK * EMIT_IPT) {
        const uint32_t j0 = r0 + threadIdx.x * EMIT_IPT;
        if (j0 < tot) {
            int g = 0, hi = EMIT_BLOCK;  // largest g with loff[g] <= j0 (it has v > 0)
#pragma unroll
            for (int step = 0; step < EMIT_LOG2; step++) {
                const int mid = (g + hi) >> 1;
                if (loff[mid] <= j0) g = mid; else hi = mid;
            }
            uint32_t end_g = loff[g + 1];
            uint4 rc = rect[g];
            uint2 mk = mask[g];
            bool full = (mk.x & mk.y) == ~0u;
            // current tile: row y, column x of the rect; for a mask, rem = its set
            // bits above the current one
            uint32_t pos = full ? j0 - loff[g] : kth_set_bit(mk.x, mk.y, j0 - loff[g]);
            uint64_t rem = full ? 0ull : ((((uint64_t)mk.y << 32) | mk.x) & ~((2ull << pos) - 1ull));
            uint32_t y = div_small(pos, rc.y), x = pos - y * rc.y;
            const uint32_t n = min((uint32_t)EMIT_IPT, tot - j0);
            for (uint32_t t = 0; t < n; t++) {
                const uint32_t j = j0 + t;
                if (j >= end_g) {  // the next Gaussian with instances
                    do {
                        g++;
                        end_g = loff[g + 1];
                    } while (j >= end_g);
                    rc = rect[g];
                    mk = mask[g];
                    full = (mk.x & mk.y) == ~0u;
                    const uint64_t m = ((uint64_t)mk.y << 32) | mk.x;
                    pos = full ? 0u : (uint32_t)__builtin_ctzll(m);
                    rem = full ? 0ull : m & (m - 1ull);
                    y = full ? 0u : div_small(pos, rc.y);
                    x = pos - y * rc.y;
                }
                kbuf[threadIdx.x * RS + t] = (rc.z + y) * (uint32_t)a.gx + rc.x + x;
                ibuf[threadIdx.x * RS + t] = rc.w;
                if (full) {
                    if (++x == rc.y) {
                        x = 0;
                        y++;
                    }
                } else if (rem) {
                    pos = (uint32_t)__builtin_ctzll(rem);
                    rem &= rem - 1ull;
                    y = div_small(pos, rc.y);
                    x = pos - y * rc.y;
                }
            }
        }
        __syncthreads();
        const uint32_t nr = min((uint32_t)(EMIT_BLOCK * EMIT_IPT), tot - r0);
        for (uint32_t i = threadIdx.x; i < nr; i += EMIT_BLOCK) {
            const uint32_t li = (i / EMIT_IPT) * RS + i % EMIT_IPT;
            if (a.packed) {
                const uint32_t tile = kbuf[li];
                reinterpret_cast<uint8_t *>(a.tile_keys)[base + r0 + i] = (uint8_t)(tile & ((1u << a.lo_bits) - 1u));
                a.ids[base + r0 + i] = ((tile >> a.lo_bits) << a.id_bits) | ibuf[li];
            } else {
                a.tile_keys[base + r0 + i] = kbuf[li];
                a.ids[base + r0 + i] = ibuf[li];
            }
        }
        __syncthreads();
    }
}

// identifyTileRanges: ranges were zeroed (preprocess.hip); empty tiles stay (0, 0).
// Four keys per thread (one 16-B load); the thread holding position i (> 0) of a
// tile change closes the previous tile and opens the next.
constexpr int RANGE_THREADS = 256;
__global__ void __launch_bounds__(RANGE_THREADS) identify_ranges_kernel(const uint32_t *tile_keys, uint32_t n,
                                                                         uint2 *ranges, SpecGuard g) {
    n = spec_count(g, n);
    const uint32_t i0 = (blockIdx.x * RANGE_THREADS + threadIdx.x) * 4u;
    if (i0 >= n) return;
    uint32_t v[4];
    if (i0 + 4 <= n) {
        const uint4 q = *reinterpret_cast<const uint4 *>(tile_keys + i0);
        v[0] = q.x;
        v[1] = q.y;
        v[2] = q.z;
        v[3] = q.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = tile_keys[min(i0 + j, n - 1)];
    }
    uint32_t prev = i0 ? tile_keys[i0 - 1] : v[0];
    if (i0 == 0) ranges[v[0]].x = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = i0 + j;
        if (i < n && v[j] != prev) {
            ranges[prev].y = i;
            ranges[v[j]].x = i;
        }
        prev = i < n ? v[j] : prev;
    }
    if (i0 + 4 >= n) ranges[prev].y = n;
}

// upstream's sorted 64-bit keys (binningState.point_list_keys of
// rasterizer_impl.cu): (tile << 32) | depth bits of the entry's Gaussian, one
// workgroup per tile over its range (the packed tile sort keeps no sorted tile
// array)
__global__ void point_list_keys_kernel(const uint2 *ranges, const uint32_t *point_list, const uint32_t *depths,
                                       uint32_t n, uint64_t *keys) {
    const uint2 r = ranges[blockIdx.x];
    for (uint32_t i = r.x + threadIdx.x; i < min(r.y, n); i += blockDim.x)
        keys[i] = ((uint64_t)blockIdx.x << 32) | depths[point_list[i]];
}

hipError_t launch_point_list_keys(int P, int W, int H, const void *geom, const void *binning, int64_t I,
                                  uint64_t *keys, hipStream_t s) {
    if (I <= 0) return hipSuccess;
    const GeomLayout L = geom_layout(P, W, H);
    const BinningLayout B = binning_layout(I, W, H);  // (point_list: offset 0 for every capacity)
    hipLaunchKernelGGL(point_list_keys_kernel, dim3((unsigned)grid_dims(W, H).tiles), dim3(256), 0, s,
                       at<const uint2>(geom, L.off[GSR_GEOM_RANGES]),
                       at<const uint32_t>(binning, B.off[GSR_BIN_POINT_LIST]),
                       at<const uint32_t>(geom, L.off[GSR_GEOM_DEPTHS]), (uint32_t)I, keys);
    return hipGetLastError();
}

// The depth sort's keys and its first pass's digit counts in one launch (the
// first pass needs no upsweep of its own): per Gaussian the view-space depth as
// preprocess computes it (xform_point4x3, the same operations, no contraction),
// key = its bits for a candidate (z > 0.2: not culled by the near plane), +inf
// bits otherwise; per radix block the histogram of the keys' low byte (the first
// digit needs no base: key_of keeps it) and the candidates' key range, which the
// first digit scan reduces into the base and the pass count.
struct DepthKeyArgs {
    const float *means3D;
    const float *viewmatrix;
    uint32_t n;
    int NB;
    uint32_t *keys;
    uint32_t *hist;   // [RADIX][NB]
    uint2 *minmax;    // [NB]
    uint32_t *zero;   // the grouped passes' group counts, cleared here (every block a slice), or NULL
    int zero_n;
    // grouped first pass (dsort_grouped): the block's digit-count row (hist
    // block-major) and its group's running counts (zeroed by preprocess), and
    // workgroup NB publishes num_rendered (the digit scan it replaces did); NULL otherwise
    uint32_t *sup0;
    const uint4 *pub_sums;
    int pub_n;
    uint32_t *pub_ctrl, *pub_host;
    uint32_t *pub_dctrl;  // ... and the depth sort's key base and pass count (GeomLayout::dsort_ctrl), or NULL
};
template <int ITEMS>
__global__ void __launch_bounds__(RX_THREADS) depth_keys_kernel(DepthKeyArgs a) {
    constexpr int TILE_N = RX_THREADS * ITEMS;
    __shared__ uint32_t h[RX_WAVES][RADIX];
    __shared__ uint32_t wmin[RX_WAVES], wmax[RX_WAVES];
    if (a.zero)  // (every workgroup of the grid its slice, the publishing one included)
        for (int i = blockIdx.x * RX_THREADS + threadIdx.x; i < a.zero_n; i += gridDim.x * RX_THREADS) a.zero[i] = 0u;
    if (a.sup0 && (int)blockIdx.x == a.NB) {  // the grouped form's extra workgroup
        publish_total<RX_THREADS>(a.pub_sums, a.pub_n, a.pub_ctrl, a.pub_host, a.pub_dctrl);
        return;
    }
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < RX_WAVES; k++) h[k][threadIdx.x] = 0;
    const uint32_t blk = radix_block(a.NB);
    const Mat4 V = load_mat4(a.viewmatrix);
    float z[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {  // every load first
        const uint32_t idx = blk * (uint32_t)TILE_N + (uint32_t)(r * RX_THREADS) + threadIdx.x;
        const uint32_t li = idx < a.n ? idx : a.n - 1;
        const f3 p = {a.means3D[3 * (size_t)li], a.means3D[3 * (size_t)li + 1], a.means3D[3 * (size_t)li + 2]};
        z[r] = xform_point4x3(p, V).z;
    }
    __syncthreads();
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < ITEMS; r++) {
        const uint32_t idx = blk * (uint32_t)TILE_N + (uint32_t)(r * RX_THREADS) + threadIdx.x;
        if (idx < a.n) {
            const bool cand = z[r] > 0.2f;  // preprocess culls z <= 0.2 (and a NaN depth sorts last)
            const uint32_t key = cand ? __float_as_uint(z[r]) : 0x7f800000u;
            a.keys[idx] = key;
            atomicAdd(&h[w][key & (RADIX - 1)], 1u);
            if (cand) {
                kmin = min(kmin, key);
                kmax = max(kmax, key);
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    if ((threadIdx.x & 63) == 0) {
        wmin[w] = kmin;
        wmax[w] = kmax;
    }
    __syncthreads();
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < RX_WAVES; k++) c += h[k][threadIdx.x];
    if (a.sup0) {  // grouped (as radix_upsweep_kernel's grouped form)
        a.hist[(size_t)blk * RADIX + threadIdx.x] = c;
        if (c) atomicAdd(&a.sup0[(size_t)(blk >> DSORT_SB_LOG2) * RADIX + threadIdx.x], c);
    } else {
        a.hist[(size_t)threadIdx.x * a.NB + blk] = c;
    }
    if (threadIdx.x == 0) {
        for (int k = 1; k < RX_WAVES; k++) {
            kmin = min(kmin, wmin[k]);
            kmax = max(kmax, wmax[k]);
        }
        a.minmax[blk] = make_uint2(kmin, kmax);
    }
}

// ------------------------------------------------------------ launchers
// The depth sort: depth_keys_kernel, then passes 1-3; the fourth pass is launched
// by the host after its sync when the published pass count needs it, or queued up
// front (the last forward needed four) as a kernel that returns at once unless the
// key range needs it.  The order lands in GSR_GEOM_DEPTH_ORDER either way.
// carry: the rect footprint's words travel with the ids (rank_gather_kernel and the
// row-span pass A then read them in rank order: no random gather of the rects)
#ifndef GSR_PUBLISH_BASE
#define GSR_PUBLISH_BASE 1
#endif
// the colour riders spread over the first RIDE_PASSES depth passes (always launched)
#ifndef GSR_RIDE_PASSES
#define GSR_RIDE_PASSES 3
#endif
constexpr int RIDE_PASSES = GSR_RIDE_PASSES;
static_assert(RIDE_PASSES >= 1 && RIDE_PASSES <= 3, "passes 1-3 always run");
static RadixPass depth_pass(int P, int W, int H, void *geom, int p, bool carry) {
    const GeomLayout L = geom_layout(P, W, H);
    RadixPass a = {};
    a.n = (uint32_t)P;
    a.NB = radix_blocks(P, dsort_items(P));
    a.hist = at<uint32_t>(geom, L.dsort_hist);
    a.totals = at<uint32_t>(geom, L.dsort_totals);
    uint32_t *ka = at<uint32_t>(geom, L.dsort_keys_a), *kb = at<uint32_t>(geom, L.dsort_keys_b);
    uint32_t *va = at<uint32_t>(geom, L.off[GSR_GEOM_DEPTH_ORDER]), *vb = at<uint32_t>(geom, L.dsort_vals_b);
    uint32_t *vc = at<uint32_t>(geom, L.dsort_vals_c);
    // keys: a (depth_keys_kernel) -> b -> a -> b -> -; values: index -> b -> c -> b -> order
    const uint32_t *kin[4] = {ka, kb, ka, kb};
    const uint32_t *vin[4] = {nullptr, vb, vc, vb};
    uint32_t *kout[4] = {kb, ka, kb, nullptr};
    uint32_t *vout[4] = {vb, vc, vb, va};
    const int role[4] = {RX_DEPTH_FIRST, RX_PLAIN, RX_DEPTH_THIRD, RX_DEPTH_FOURTH};
    a.ctrl = at<const uint32_t>(geom, L.dsort_ctrl);
    if (p == 0) {
        a.minmax = at<uint2>(geom, L.dsort_minmax);
        a.ctrl_out = at<uint32_t>(geom, L.dsort_ctrl);
    }
    a.vout_final = va;
    a.kin = kin[p];
    a.vin = vin[p];
    a.kout = kout[p];
    a.vout = vout[p];
    a.role = role[p];
    if (carry) {  // words: preprocess's (the fourth array) -> b -> c -> b -> final, like the values
        uint32_t *wb = at<uint32_t>(geom, L.rs_words), *wc = wb + P, *wf = wb + 2 * (size_t)P, *wp = wb + 3 * (size_t)P;
        const uint32_t *win[4] = {wp, wb, wc, wb};
        uint32_t *wout[4] = {wb, wc, wb, wf};
        a.win = win[p];
        a.wout = wout[p];
        a.wout_final = wf;
    }
    a.shift = 8 * p;
    a.nbits = RADIX_BITS;
    a.dmask = RADIX - 1;
    if (p > 0 ? dsort_grouped(P) : dsort_grouped1(P)) {  // passes 2-4, and the first (counts from depth_keys_kernel)
        a.nsup = dsort_nsup(P);
        a.sup = p > 0 ? at<uint32_t>(geom, L.dsort_sup) + (size_t)(p - 1) * a.nsup * RADIX
                      : at<uint32_t>(geom, L.dsort_sup0);
    }
    return a;
}

template <int ITEMS>
static hipError_t depth_sort_items(int P, int W, int H, const float *means3D, const float *viewmatrix, void *geom,
                                   int passes, uint32_t *host_ctrl, bool carry, const ColourRide *ride,
                                   hipStream_t s) {
    const GeomLayout L = geom_layout(P, W, H);
    DepthKeyArgs k;
    k.means3D = means3D;
    k.viewmatrix = viewmatrix;
    k.n = (uint32_t)P;
    k.NB = radix_blocks(P, ITEMS);
    k.keys = at<uint32_t>(geom, L.dsort_keys_a);
    k.hist = at<uint32_t>(geom, L.dsort_hist);
    k.minmax = at<uint2>(geom, L.dsort_minmax);
    k.zero = dsort_grouped(P) ? at<uint32_t>(geom, L.dsort_sup) : nullptr;
    k.zero_n = dsort_grouped(P) ? 3 * dsort_nsup(P) * RADIX : 0;
    // grouped: the first pass needs no digit scan either; num_rendered's publish
    // (that scan's extra workgroup) moves to this launch's extra workgroup
    const bool g1 = dsort_grouped1(P);
    k.sup0 = g1 ? at<uint32_t>(geom, L.dsort_sup0) : nullptr;
    k.pub_sums = at<const uint4>(geom, L.block_sums);
    k.pub_n = pre_blocks(P);
    k.pub_ctrl = at<uint32_t>(geom, L.off[GSR_GEOM_CTRL]);
    k.pub_host = host_ctrl;
    // the key base from preprocess's per-workgroup candidate ranges (GSR_PUBLISH_BASE)
    const bool pb = g1 && GSR_PUBLISH_BASE;
    k.pub_dctrl = pb ? at<uint32_t>(geom, L.dsort_ctrl) : nullptr;
    hipLaunchKernelGGL(depth_keys_kernel<ITEMS>, dim3(k.NB + (g1 ? 1 : 0)), dim3(RX_THREADS), 0, s, k);
    // passes 3: the host reads the published pass count after its sync and launches
    // the fourth (launch_depth_sort_fourth) when the keys need it — three
    // early-returning launches (~14 us at config C) saved in the common case;
    // passes 4: queued up front (the last forward needed it), returning at once
    // when three suffice
    for (int p = 0; p < passes; p++) {
        RadixPass a = depth_pass(P, W, H, geom, p, carry);
        if (ride && ride->nb > 0 && p < RIDE_PASSES) {  // this pass's share of the colour blocks
            a.ride = *ride;
            a.ride.b0 = ride->b0 + (int)((int64_t)ride->nb * p / RIDE_PASSES);
            a.ride.nb = ride->b0 + (int)((int64_t)ride->nb * (p + 1) / RIDE_PASSES) - a.ride.b0;
        }
        if (p == 0) {  // the first digit scan (or, grouped, the first downsweep) publishes the pass count ...
            a.host_ctrl = host_ctrl;
            a.base_published = pb ? 1 : 0;
            if (!g1) {  // ... and num_rendered (grouped: depth_keys_kernel's extra workgroup)
                a.pub_sums = at<const uint4>(geom, L.block_sums);
                a.pub_n = pre_blocks(P);
                a.pub_ctrl = at<uint32_t>(geom, L.off[GSR_GEOM_CTRL]);
                a.pub_host = host_ctrl;
            }
        }
        hipError_t e = radix_pass<ITEMS>(a, s, p == 0);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_depth_sort(int P, int W, int H, const float *means3D, const float *viewmatrix, void *geom,
                             int passes, uint32_t *host_ctrl, bool carry, hipStream_t s, const ColourRide *ride) {
    if (P <= 0) return hipSuccess;
    return dsort_items(P) == DSORT_ITEMS_BIG
               ? depth_sort_items<DSORT_ITEMS_BIG>(P, W, H, means3D, viewmatrix, geom, passes, host_ctrl, carry, ride, s)
               : depth_sort_items<DSORT_ITEMS>(P, W, H, means3D, viewmatrix, geom, passes, host_ctrl, carry, ride, s);
}

hipError_t launch_depth_sort_fourth(int P, int W, int H, void *geom, bool carry, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    return dsort_items(P) == DSORT_ITEMS_BIG ? radix_pass<DSORT_ITEMS_BIG>(depth_pass(P, W, H, geom, 3, carry), s)
                                             : radix_pass<DSORT_ITEMS>(depth_pass(P, W, H, geom, 3, carry), s);
}

// After the depth sort: the rects in rank order and the rank-order instance offsets
// of the emit blocks.
// rowspan: the row-span binning follows (rowspan.hip): the pass-A row counts
// instead of the emission offsets, and their per-row scan
hipError_t launch_rank_gather(int P, int W, int H, void *geom, bool require3, bool rowspan, bool carry,
                              hipStream_t s) {
    if (P <= 0) return hipSuccess;
    const GeomLayout L = geom_layout(P, W, H);
    const int gy = rowspan ? grid_dims(W, H).gy : 0, nA = rsa_blocks(P);
    uint32_t *ahist = at<uint32_t>(geom, L.rs_ahist);
    hipLaunchKernelGGL(rank_gather_kernel, dim3(rg_blocks(P)), dim3(RG_THREADS), 0, s,
                       at<const uint32_t>(geom, L.off[GSR_GEOM_DEPTH_ORDER]), at<const uint4>(geom, L.rects), P,
                       at<uint4>(geom, L.rects_ranked), at<uint32_t>(geom, L.emit_sums),
                       at<uint32_t>(geom, L.emit_super), require3 ? at<const uint32_t>(geom, L.dsort_ctrl) : nullptr,
                       ahist, nA, gy, rowspan && carry ? at<const uint32_t>(geom, L.rs_words) + 2 * (size_t)P : nullptr);
    if (!rowspan) return hipGetLastError();
    return launch_count_scan(ahist, nA, nullptr, at<uint32_t>(geom, L.rs_atot), gy, SpecGuard{}, s);
}

hipError_t launch_emit(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &guard,
                       hipStream_t s) {
    const GeomLayout L = geom_layout(P, W, H);
    const BinningLayout B = binning_layout(cap, W, H);
    const GridDims g = grid_dims(W, H);
    EmitArgs a;
    a.P = P;
    a.gx = g.gx;
    a.order = at<const uint32_t>(geom, L.off[GSR_GEOM_DEPTH_ORDER]);
    a.rects = at<const uint4>(geom, L.rects_ranked);
    a.block_local = at<const uint32_t>(geom, L.emit_sums);
    a.super = at<const uint32_t>(geom, L.emit_super);
    // emit into the buffer pair that the tile passes will end in KEYS/POINT_LIST
    // (the packed form: emit -> b, first pass -> KEYS, second -> POINT_LIST)
    const bool packed = tile_sort_packed(g.tiles, P);
    const bool odd = packed || (tile_sort_passes(g.tiles) & 1);
    const int bits = tile_bits(g.tiles);
    a.packed = packed ? 1 : 0;
    a.lo_bits = bits / 2;
    a.id_bits = 32 - (bits - bits / 2);
    a.tile_keys = at<uint32_t>(binning, odd ? B.keys_b : B.off[GSR_BIN_KEYS]);
    a.ids = at<uint32_t>(binning, odd ? B.vals_b : B.off[GSR_BIN_POINT_LIST]);
    a.g = guard;
    hipLaunchKernelGGL(emit_kernel, dim3(emit_blocks(P)), dim3(EMIT_BLOCK), 0, s, a);
    return hipGetLastError();
}

// n: the instances to sort (the capacity, when g is speculative); cap: the binning
// buffer's capacity, which fixes its layout and the radix block size
hipError_t launch_tile_sort(int P, int W, int H, void *geom, void *binning, int64_t n, int64_t cap,
                            const SpecGuard &guard, hipStream_t s) {
    const int64_t I = n;
    const GeomLayout L = geom_layout(P, W, H);
    const BinningLayout B = binning_layout(cap, W, H);
    const GridDims g = grid_dims(W, H);
    const int npass = tile_sort_passes(g.tiles);
    uint32_t *keys[2] = {at<uint32_t>(binning, B.off[GSR_BIN_KEYS]), at<uint32_t>(binning, B.keys_b)};
    uint32_t *vals[2] = {at<uint32_t>(binning, B.off[GSR_BIN_POINT_LIST]), at<uint32_t>(binning, B.vals_b)};
    const int bits = tile_bits(g.tiles);
    int cur = npass & 1;
    RadixPass a = {};
    a.n = (uint32_t)I;
    a.g = guard;
    const int items = tsort_items(cap);
    a.NB = radix_blocks(I, items);
    a.role = RX_PLAIN;
    a.hist = at<uint32_t>(binning, B.hist);
    a.totals = at<uint32_t>(binning, B.totals);
    uint2 *ranges = at<uint2>(geom, L.off[GSR_GEOM_RANGES]);
    if (tile_sort_packed(g.tiles, P)) {
        // pass 1: the low tile digit (emit's bytes in b) moves the packed words
        // (emit's words in b) to KEYS
        const int lo = bits / 2, hi = bits - lo;
        a.kin = keys[1];
        a.vin = vals[1];
        a.kout = nullptr;
        a.vout = keys[0];
        a.shift = 0;
        a.nbits = lo;
        a.dmask = (1u << lo) - 1u;
        a.id_bits = 32 - hi;
        a.totals = at<uint32_t>(binning, B.totals1);
        a.seg_table = at<uint32_t>(binning, B.seg_table);
        hipError_t e = items == TSORT_ITEMS_BIG ? radix_pass<TSORT_ITEMS_BIG, RXM_PACK>(a, s)
                                                : radix_pass<TSORT_ITEMS, RXM_PACK>(a, s);
        if (e != hipSuccess) return e;
        // pass 2: the high tile bits of the packed words, segment-aligned blocks;
        // ids -> POINT_LIST, ranges from the digit counts
        a.kin = keys[0];
        a.vin = nullptr;
        a.vout = vals[0];
        a.shift = 32 - hi;
        a.nbits = hi;
        a.dmask = (1u << hi) - 1u;
        a.totals = at<uint32_t>(binning, B.totals);
        a.seg_totals = at<const uint32_t>(binning, B.totals1);
        a.seg_bits = lo;
        a.NB = radix_blocks(I, items) + (1 << lo);
        a.ranges = ranges;
        a.T = g.tiles;
        return items == TSORT_ITEMS_BIG ? radix_pass<TSORT_ITEMS_BIG, RXM_UNPACK>(a, s)
                                        : radix_pass<TSORT_ITEMS, RXM_UNPACK>(a, s);
    }
    for (int p = 0; p < npass; p++) {
        a.kin = keys[cur];
        a.vin = vals[cur];
        a.kout = keys[cur ^ 1];
        a.vout = vals[cur ^ 1];
        // split the tile bits evenly over the passes (13 -> 7 + 6 at 1080p): fewer
        // digits in the low pass = longer contiguous output runs per block
        const int lo_bits = (bits * p) / npass, hi_bits = (bits * (p + 1)) / npass;
        a.shift = lo_bits;
        a.nbits = hi_bits - lo_bits;
        a.dmask = (1u << a.nbits) - 1u;
        hipError_t e = items == TSORT_ITEMS_BIG ? radix_pass<TSORT_ITEMS_BIG>(a, s) : radix_pass<TSORT_ITEMS>(a, s);
        if (e != hipSuccess) return e;
        cur ^= 1;
    }
    const int64_t per_block = 4 * RANGE_THREADS;
    hipLaunchKernelGGL(identify_ranges_kernel, dim3((unsigned)((I + per_block - 1) / per_block)), dim3(RANGE_THREADS),
                       0, s, (const uint32_t *)keys[0], (uint32_t)I, ranges, guard);
    return hipGetLastError();
}

}  // namespace gsr

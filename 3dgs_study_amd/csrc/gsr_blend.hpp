// gsr_blend.hpp — pieces shared by the forward and backward blend kernels.
//
// Work unit: one wave64 = one 8x8 pixel quadrant of a 16x16 tile (lane l ->
// pixel (l & 7, l >> 3)).  A wave streams the tile's depth-sorted list in
// chunks of 64 entries, one entry per lane: the lane gathers the entry's 48-B
// splat record, tests in parallel whether the Gaussian can reach ANY pixel of
// the quadrant, and a ballot turns the chunk into a bit mask.  The wave then
// walks only the set bits; each Gaussian's parameters are broadcast from the
// owning lane with v_readlane into SGPRs, so the per-pixel math reads scalar
// operands and no LDS or workgroup barrier is involved.
#pragma once

#include "gsr_common.hpp"
#include "gsr_wave.hpp"

namespace gsr {

// Waves per workgroup: 4 = the 4 quadrants of one tile; 1 = one quadrant per
// workgroup (a finished quadrant frees its slot at once instead of waiting for
// the tile's slowest quadrant).
#ifndef GSR_BLEND_WAVES
#define GSR_BLEND_WAVES 1
#endif
constexpr int BLEND_WAVES = GSR_BLEND_WAVES;
constexpr int BLEND_THREADS = 64 * BLEND_WAVES;
static_assert(BLEND_WAVES == 4 || BLEND_WAVES == 1, "GSR_BLEND_WAVES must be 4 or 1");

// Exact cull: min over the quadrant's pixel centres [x0, x0+7] x [y0, y0+7] of
// q(d) = ca dx^2 + 2 cb dx dy + cc dy^2 (d = pixel - mean) against qmax.  The
// forward/backward reject a pixel when o*exp(-q/2) < 1/255, i.e. q > 2 ln(255 o);
// qmax is that bound widened in preprocess, so a skipped Gaussian is one that
// every pixel of the quadrant would have skipped.  A NaN bound keeps the entry.
// box_hit is the same test over [x0, x0+ext] x [y0, y0+ext] (preprocess.hip uses
// it per 16x16 tile, ext = 15, to drop the bounding-rect tiles a Gaussian cannot
// reach).
__device__ __forceinline__ bool box_hit(float mx, float my, float ca, float cb, float cc, float qmax, float x0,
                                        float y0, float ext) {
    // ca, cb, cc, qmax come from the splat record, i.e. times -1/2: the form is
    // concave, so "min over the box of q <= qmax" reads "max of q' >= qmax'"
    const float dx0 = x0 - mx, dx1 = x0 + ext - mx;
    const float dy0 = y0 - my, dy1 = y0 + ext - my;
    if (dx0 <= 0.f && dx1 >= 0.f && dy0 <= 0.f && dy1 >= 0.f) return true;  // mean inside: q_min = 0
    // with the extremum outside the box, the box extremum lies on an edge (the
    // edge optimiser -cb dx / cc is scale-invariant).  Approximate reciprocals
    // only move it by an ulp: q changes at second order, far inside the margin
    const float icc = __builtin_amdgcn_rcpf(cc), ica = __builtin_amdgcn_rcpf(ca);
    float q = -INFINITY;
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const float dx = e ? dx1 : dx0;
        const float dy = fminf(fmaxf(-cb * dx * icc, dy0), dy1);
        q = fmaxf(q, ca * dx * dx + 2.0f * cb * dx * dy + cc * dy * dy);
        const float ey = e ? dy1 : dy0;
        const float ex = fminf(fmaxf(-cb * ey * ica, dx0), dx1);
        q = fmaxf(q, ca * ex * ex + 2.0f * cb * ex * ey + cc * ey * ey);
    }
    return !(q < qmax);
}
__device__ __forceinline__ bool quad_hit(float mx, float my, float ca, float cb, float cc, float qmax, float x0,
                                         float y0) {
    return box_hit(mx, my, ca, cb, cc, qmax, x0, y0, 7.0f);
}

// power and G = exp(power) of one (pixel, Gaussian), for upstream's
// `power > 0` skip and alpha = min(0.99, opacity * expf(power)) with its
// `alpha < 1/255` skip.  The blend loops evaluate power as d^T conic' d
// (conic' = -conic/2, contracted) and exp in hardware (v_exp_f32 of
// power * log2 e): both within a few ulp of upstream's float expression and
// the correctly rounded expf.  Where that could move a skip decision — alpha
// within 2^-12 relative of 1/255 (the combined error is below 2^-16), or a
// positive power (the conic is positive definite, so only rounding makes one)
// — the pair is redone exactly as the CPU restatement does it (blend_fix):
// upstream's expression in upstream's operation order without contraction,
// and exp in double rounded once (the correctly rounded expf).  So every skip
// decision, and with it n_contrib, matches the oracle's.  The loops test the
// flags of both Gaussians of an iteration with ONE wave-uniform branch
// (ballot), taken for ~1e-4 of the pairs: a per-lane branch around each
// Gaussian cost render_fwd 20 % and render_bwd 7 % (exec-mask juggling that
// broke the two Gaussians' interleaving); this form costs 15 % / 6 % (config C:
// 132 -> 152 us, 247 -> 261 us; of that the positive-power test is 8 / 3 us and
// the double-precision call ~0 / 3 us).  The forward and backward share the
// decisions bit for bit.
__device__ __forceinline__ bool blend_near(float power, float opacity_times_G) {
    return power > 0.0f || fabsf(opacity_times_G * 255.0f - 1.0f) < 0x1p-12f;
}
// exp(x) for |x| <= 16 in double, Taylor to degree 13 on |r| <= ln2/2
// (truncation < 2^-55 relative), rounded once to float (equal to the correctly
// rounded exp for every float in [-16, 1]).  Not inlined: the rarely taken
// re-check then adds a call instead of its double-precision registers to
// every iteration of the blend loops (inlined, the library exp cost
// render_fwd 54 -> 73 VGPRs, render_bwd 68 -> 92).
__device__ __attribute__((noinline)) float exp_rn_f32(float x) {
    const double xd = (double)x;
    const double n = __builtin_rint(xd * 1.4426950408889634);
    const double r = __builtin_fma(-n, 1.9082149292705877e-10, __builtin_fma(-n, 0.6931471803691238, xd));
    double p = 1.0 / 6227020800.0;
    p = __builtin_fma(p, r, 1.0 / 479001600.0);
    p = __builtin_fma(p, r, 1.0 / 39916800.0);
    p = __builtin_fma(p, r, 1.0 / 3628800.0);
    p = __builtin_fma(p, r, 1.0 / 362880.0);
    p = __builtin_fma(p, r, 1.0 / 40320.0);
    p = __builtin_fma(p, r, 1.0 / 5040.0);
    p = __builtin_fma(p, r, 1.0 / 720.0);
    p = __builtin_fma(p, r, 1.0 / 120.0);
    p = __builtin_fma(p, r, 1.0 / 24.0);
    p = __builtin_fma(p, r, 1.0 / 6.0);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return (float)__builtin_ldexp(p, (int)n);
}
// the exact power and G of a flagged pair (conic' = -conic/2 from the splat record)
__device__ __forceinline__ void blend_fix(float &power, float &G, float dx, float dy, float ca, float cb, float cc) {
#pragma clang fp contract(off)
    const float cx = -2.0f * ca, cy = -2.0f * cb, cz = -2.0f * cc;  // exact
    power = -0.5f * (cx * dx * dx + cz * dy * dy) - cy * dx * dy;
    G = exp_rn_f32(power);
}

// s_waitcnt vmcnt(4) expcnt(7) lgkmcnt(15): everything but the 4 youngest
// vector-memory ops (the chunk prefetch) has completed.  Issued as the builtin so
// that the compiler's waitcnt pass sees it and marks the older loads as landed.
__device__ __forceinline__ void wait_vmcnt_4() { __builtin_amdgcn_s_waitcnt(0x0F74); }

// Per-wave LDS image of the current chunk: entry k's 48-B splat record at
// byte 48k (lane-contiguous b128 stores are conflict-free at this stride).  The
// per-Gaussian loop reads the record back with uniform-address ds_reads
// (broadcast) — LDS-pipe work instead of nine or ten VALU v_readlanes.
struct ChunkStage {
    float4 rec[65][3];  // render_bwd.hip keeps its survivors in 1..64 (0 = a zero record)
};
__device__ __forceinline__ void stage_chunk(ChunkStage &st, int lane, const float4 &A, const float4 &B,
                                            const float4 &C) {
    st.rec[lane][0] = A;
    st.rec[lane][1] = B;
    st.rec[lane][2] = C;
}

// Compacted chunk image: only the entries that survived the cull, in chunk
// order (slot = first + number of survivors in lower lanes), each record's last word
// holding the entry's lane (its list position minus the chunk start).  The
// Gaussian loops then walk slots 0..n-1 with an affine index — no find-first-set
// chains on the scalar unit between one pair's LDS reads and the next's.
__device__ __forceinline__ int stage_survivors(ChunkStage &st, int lane, bool rel, uint64_t mask, const float4 &A,
                                               const float4 &B, const float4 &C, int first = 0) {
    if (rel) {
        const int slot = first + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        st.rec[slot][0] = A;
        st.rec[slot][1] = B;
        st.rec[slot][2] = make_float4(C.x, C.y, C.z, __int_as_float(lane));
    }
    return __builtin_popcountll(mask);
}

__device__ __forceinline__ float bcast(float v, int k) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}
__device__ __forceinline__ uint32_t bcast_u(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }

// blockIdx -> tile.  Workgroups are dealt round-robin over the 8 XCDs
// (blockIdx % 8 share one; a speed hint only, never relied upon), so strips of
// XCD_STRIP consecutive tiles (which share most of their Gaussians) are given
// to one XCD's L2, and the strips are dealt round-robin over the XCDs so that
// every XCD gets an even share of the heavy centre of the image.
constexpr int XCD_STRIP = 4;
template <int STRIP = XCD_STRIP>
__device__ __forceinline__ int xcd_tile(int b, int tiles) {
    const int x = b & 7, j = b >> 3;
    const int t = ((j / STRIP) * 8 + x) * STRIP + (j % STRIP);
    return t < tiles ? t : -1;
}
template <int STRIP = XCD_STRIP>
__host__ __device__ inline int xcd_grid(int tiles) {
    const int strips = (tiles + STRIP - 1) / STRIP;
    return ((strips + 7) / 8) * 8 * STRIP;
}

// (tile, quadrant) of this wave; tile < 0 = past the end of the grid
struct QuadSlot {
    int tile, w;
};
__device__ __forceinline__ QuadSlot quad_slot(int tiles) {
    if constexpr (BLEND_WAVES == 4) {
        // wave index in an SGPR: the LDS record addresses are then scalar + immediate
        return {xcd_tile(blockIdx.x, tiles), __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)};
    } else {
        const int u = xcd_tile<4 * XCD_STRIP>(blockIdx.x, 4 * tiles);
        return {u < 0 ? -1 : u >> 2, u & 3};
    }
}
__host__ inline int blend_grid(int tiles) {
    return BLEND_WAVES == 4 ? xcd_grid(tiles) : xcd_grid<4 * XCD_STRIP>(4 * tiles);
}

// ---- backward wave order (render_fwd.hip fills it, render_bwd.hip reads it)
// The backward starts each XCD's heaviest quadrants first.  A quadrant keeps the
// XCD of the forward's strip order (xcd_tile: strips of ORDER_STRIP quadrants
// dealt round-robin over the 8 XCDs), so each L2 sees the same neighbouring
// tiles in both passes.  Each forward wave files its quadrant under
// (XCD, work bucket) with one atomic; backward workgroup 8 r + x (XCD x under
// round-robin placement: a speed hint only) takes XCD x's r-th entry in
// bucket order.
constexpr int ORDER_STRIP = 4 * XCD_STRIP;  // quadrants per strip
constexpr int ORDER_NBUCKET = 32;           // work buckets per XCD, heaviest first
__host__ __device__ inline int quad_xcd(int q) { return (q / ORDER_STRIP) & 7; }
__device__ __forceinline__ int order_bucket(uint32_t work) {  // 16 blended Gaussians per bucket
    return ORDER_NBUCKET - 1 - (int)min(work >> 4, (uint32_t)ORDER_NBUCKET - 1);
}
// Workgroup 8 r + x -> XCD x's r-th quadrant in bucket order, or -1 past the end
// of that XCD's list (all lanes of the wave must be active).
__device__ __forceinline__ int ordered_quad(const uint32_t *cnt, const uint32_t *qlist, int maxc) {
    const int lane = threadIdx.x & 63, x = blockIdx.x & 7, rr = blockIdx.x >> 3;
    const uint32_t c = lane < ORDER_NBUCKET ? cnt[x * ORDER_NBUCKET + lane] : 0u;
    const uint32_t incl = wave_inclusive_scan(c);
    const int b = __builtin_popcountll(__ballot(incl <= (uint32_t)rr));  // buckets wholly before entry rr
    if (b >= ORDER_NBUCKET) return -1;
    const uint32_t start = (uint32_t)__shfl((int)(incl - c), b);
    return (int)qlist[(size_t)(x * ORDER_NBUCKET + b) * maxc + (rr - start)];
}
// quadrants per XCD list (the longest): the ordered grids are 8 times this
__host__ inline int order_max_per_xcd(int nq) {
    int mx = 0;
    for (int x = 0; x < 8; x++) {
        int c = 0;
        for (int q0 = x * ORDER_STRIP; q0 < nq; q0 += 8 * ORDER_STRIP) c += (nq - q0 < ORDER_STRIP) ? nq - q0 : ORDER_STRIP;
        mx = c > mx ? c : mx;
    }
    return mx;
}

}  // namespace gsr

// gsr_blend.hpp — pieces shared by the forward and backward blend kernels.
//
// Work unit: one wave64 = one 8x8 pixel quadrant of a 16x16 tile (lane l ->
// pixel (l & 7, l >> 3)).  A wave streams the tile's depth-sorted list in
// chunks of 64 entries, one entry per lane: the lane gathers the entry's 48-B
// splat record, tests in parallel whether the Gaussian can reach ANY pixel of
// the quadrant, and a ballot turns the chunk into a bit mask.  The survivors'
// records go to a per-wave LDS image (QuadChunk) in list order, and the wave
// walks them with uniform-address LDS reads (broadcast): no workgroup barrier.
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
// `alpha < 1/255` skip.  The blend loops evaluate power with upstream's own
// expression in upstream's operation order, without contraction (exact_power,
// the same instructions in both kernels and in the CPU restatement), so every
// power — and with it every `power > 0` decision — is the oracle's bit for bit.
// (Rounds 2-3 evaluated it as a quadrant-relative quadratic, five FMAs instead
// of ten operations; for needle-like Gaussians, whose conic's terms cancel, that
// differed from upstream's rounding by ~1e-3 and moved the image by 2e-3,
// tests/test_gpu_parity.py::test_needle_gaussians.)  exp runs in hardware
// (v_exp_f32 of power * log2 e), a few ulp from the correctly rounded expf; where
// that could move the alpha decision — alpha within 2^-12 relative of 1/255 —
// the pair takes the correctly rounded exp (blend_exact_G: exp in double,
// rounded once), so n_contrib matches the oracle's.  The loops test the flags of
// both Gaussians of an iteration with ONE wave-uniform branch (ballot), taken
// for ~1e-4 of the pairs: a per-lane branch around each Gaussian cost render_fwd
// 20 % and render_bwd 7 % (exec-mask juggling that broke the two Gaussians'
// interleaving).  Both kernels flag from the same power and G, so they re-check
// the same pairs and share every decision bit for bit (a pair that only one of
// them re-checked could be skipped by one and blended by the other, corrupting
// the backward's replay of that pixel).
__device__ __forceinline__ bool blend_near(float alpha) { return fabsf(alpha * 255.0f - 1.0f) < 0x1p-12f; }
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

// upstream's power of the staged record r0 = {mean, c'a, c'c}, r1.x = 2 c'b
// (conic' = -conic/2, exact) at pixel (fx, fy): d = mean - pixel (one rounding
// each, as upstream subtracts), then -1/2 (a dx dx + c dy dy) - b dx dy, which
// with the exactly scaled conic' reads (c'a dx) dx + (c'c dy) dy + (2c'b dx) dy:
// every product and sum rounds exactly as upstream's does (scaling by a power
// of two commutes with rounding).  The backward reuses d.
__device__ __forceinline__ float exact_power(const float4 &r0, const float4 &r1, float fx, float fy, float &dx,
                                             float &dy) {
#pragma clang fp contract(off)
    dx = r0.x - fx;
    dy = r0.y - fy;
    return ((r0.z * dx) * dx + (r0.w * dy) * dy) + (r1.x * dx) * dy;
}

// s_waitcnt vmcnt(4) expcnt(7) lgkmcnt(15): everything but the 4 youngest
// vector-memory ops (the chunk prefetch) has completed.  Issued as the builtin so
// that the compiler's waitcnt pass sees it and marks the older loads as landed.
__device__ __forceinline__ void wait_vmcnt_4() { __builtin_amdgcn_s_waitcnt(0x0F74); }

// Per-wave LDS image of a chunk's surviving Gaussians, shared by the forward and
// the backward (so both evaluate the power with the same instructions on the same
// values: their fast skip decisions, and with them their exact re-checks, agree bit
// for bit):
//   rec[k][0] = {mean.x, mean.y, c'a, c'c}, rec[k][1] = {2 c'b, opacity, r, g},
//   rec[k][2] = {b, tag, id bits, -}
// (the forward reads 40 of the 48 B: two ds_read_b128 and a ds_read_b64)
// with tag = the entry's list position + 1 (its n_contrib value) in render_fwd,
// its lane (chunk offset) in render_bwd.
// A zero record (opacity 0: alpha 0, never blended) pads an odd survivor count.
struct QuadChunk {
    float4 rec[66][3];  // render_fwd: survivors 0..ns-1, zero at ns; render_bwd: zero at 0, survivors 1..ns
};
__device__ __forceinline__ void stage_quad(float4 *rec, const float4 &A, const float4 &B, const float4 &C, int tag) {
    rec[0] = make_float4(A.x, A.y, A.z, B.x);
    rec[1] = make_float4(2.0f * A.w, B.y, B.z, B.w);
    rec[2] = make_float4(C.x, __int_as_float(tag), C.y, 0.0f);
}
__device__ __forceinline__ void stage_zero(float4 *rec, int lane) {
    if (lane < 3) rec[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// Whole-record LDS reads (volatile: the load vectorizer would otherwise split the
// records around unused fields, or merge two 8-B reads into one ds_read2_b64,
// which costs twice the LDS cycles of two ds_read_b64).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const volatile f32x4 lds_f32x4;
typedef __attribute__((address_space(3))) const volatile f32x2 lds_f32x2;
__device__ __forceinline__ float4 ld4(lds_f32x4 *p) {
    const f32x4 v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 ld2(lds_f32x2 *p) {
    const f32x2 v = *p;
    return make_float2(v.x, v.y);
}

// compacted slot of a surviving lane: first + survivors in lower lanes
__device__ __forceinline__ int survivor_slot(uint64_t mask, int first) {
    return first + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
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
#ifndef GSR_XCD_STRIP
#define GSR_XCD_STRIP 4
#endif
constexpr int XCD_STRIP = GSR_XCD_STRIP;
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

// ---- backward wave order (render_fwd.hip buckets it, render_bwd.hip files and reads it)
// The backward starts each XCD's heaviest quadrants first.  A quadrant keeps the
// XCD of the forward's strip order (xcd_tile: strips of ORDER_STRIP quadrants
// dealt round-robin over the 8 XCDs), so each L2 sees the same neighbouring
// tiles in both passes.  Each forward wave stores its quadrant's work bucket;
// the backward's first launch (bwd_prepare_kernel) files the quadrants under
// (XCD, work bucket); backward workgroup 8 r + x (XCD x under round-robin
// placement: a speed hint only) takes XCD x's r-th entry in bucket order.
constexpr int ORDER_STRIP = 4 * XCD_STRIP;  // quadrants per strip
constexpr int ORDER_NBUCKET = 32;           // work buckets per XCD, heaviest first
static_assert(ORDER_FILED == 8 * ORDER_NBUCKET, "the flag words follow the 8 x ORDER_NBUCKET counts");
__host__ __device__ inline int quad_xcd(int q) { return (q / ORDER_STRIP) & 7; }
__device__ __forceinline__ int order_bucket(uint32_t work) {  // 16 blended Gaussians per bucket
    return ORDER_NBUCKET - 1 - (int)min(work >> 4, (uint32_t)ORDER_NBUCKET - 1);
}
// Ordered workgroup 8 r + x (blk) -> XCD x's r-th quadrant in bucket order, or -1
// past the end of that XCD's list (all lanes of the wave must be active).
__device__ __forceinline__ int ordered_quad(const uint32_t *cnt, const uint32_t *qlist, int maxc, int blk) {
    const int lane = threadIdx.x & 63, x = blk & 7, rr = blk >> 3;
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

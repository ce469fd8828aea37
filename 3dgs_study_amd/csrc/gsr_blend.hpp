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
// `alpha < 1/255` skip.  The blend loops evaluate power as the quadrant-relative
// quadratic of the staged record (quad_power, the same instructions in both
// kernels) and exp in hardware (v_exp_f32 of power * log2 e): both within a few
// ulp of upstream's float expression and the correctly rounded expf.  Where that could move a skip decision — alpha
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
// the double-precision call ~0 / 3 us).  Both kernels flag from the same fast
// power and G, so they re-check the same pairs and share every decision bit for
// bit (a pair that only one of them re-checked could be skipped by one and
// blended by the other, corrupting the backward's replay of that pixel).  The
// positive-power test needs no band: upstream's float expression
// -0.5 (a dx^2 + c dy^2) - b dx dy has the sign of the exact form (<= 0) unless
// the conic's condition number exceeds ~2^21 (absolute rounding <= 4 ulp of
// a dx^2 + c dy^2, the form >= that times 1/(2 kappa)) — a 2-D covariance
// eigenvalue above ~6e5 px^2 given the 0.3 px^2 low-pass — so short of such a
// conic a fast power <= 0 never hides an upstream skip.
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
// the exact power and G of a flagged pair (conic' = -conic/2 from the splat record).
// Upstream skips a positive power: G = 0 then gives alpha 0, which both blend
// loops skip, so their fast paths need no `power > 0` select (every positive fast
// power is flagged, and a fast power <= 0 stands for upstream's, see above).
__device__ __forceinline__ void blend_fix(float &power, float &G, float dx, float dy, float ca, float cb, float cc) {
#pragma clang fp contract(off)
    const float cx = -2.0f * ca, cy = -2.0f * cb, cz = -2.0f * cc;  // exact
    power = -0.5f * (cx * dx * dx + cz * dy * dy) - cy * dx * dy;
    G = power > 0.0f ? 0.0f : exp_rn_f32(power);
}

// s_waitcnt vmcnt(4) expcnt(7) lgkmcnt(15): everything but the 4 youngest
// vector-memory ops (the chunk prefetch) has completed.  Issued as the builtin so
// that the compiler's waitcnt pass sees it and marks the older loads as landed.
__device__ __forceinline__ void wait_vmcnt_4() { __builtin_amdgcn_s_waitcnt(0x0F74); }

// Per-wave LDS image of a chunk's surviving Gaussians, shared by the forward and
// the backward (so both evaluate the power with the same instructions on the same
// values: their fast skip decisions, and with them their exact re-checks, agree bit
// for bit).  Each record carries the power as a quadratic in the pixel's offset
// (x, y) in 0..7 from the quadrant's first pixel:
//   p(x, y) = K6 + K4 x + K5 y + K1 x^2 + K2 x y + K3 y^2
// (conic' = -conic/2, centre offset (u, v) = mean - quadrant origin: K1 = c'a,
// K2 = 2 c'b, K3 = c'c, K4 = -2 (c'a u + c'b v), K5 = -2 (c'b u + c'c v),
// K6 = p(0, 0)) — five FMAs per pixel instead of the eight of d^T conic' d — and
// the mean itself, for the exact re-check (d = mean - pixel, one rounding, as
// upstream) and the backward's d.
//   rec[k][0] = {K6, K4, K5, K1}, rec[k][1] = {K2, K3, opacity, r},
//   rec[k][2] = {g, b, id bits, tag},  rec[k][3] = {mean.x, mean.y, -, -}
// with tag = the entry's list position + 1 (its n_contrib value) in render_fwd,
// its lane (chunk offset) in render_bwd.
// A zero record (opacity 0: alpha 0, never blended) pads an odd survivor count.
struct QuadChunk {
    float4 rec[66][4];  // render_fwd: survivors 0..ns-1, zero at ns; render_bwd: zero at 0, survivors 1..ns
};
__device__ __forceinline__ void stage_quad(float4 *rec, const float4 &A, const float4 &B, const float4 &C, float qx0,
                                           float qy0, int tag) {
    const float u = A.x - qx0, v = A.y - qy0;  // exact for means near the quadrant
    const float ca = A.z, cb = A.w, cc = B.x;
    const float hu = fmaf(ca, u, cb * v), hv = fmaf(cb, u, cc * v);
    rec[0] = make_float4(fmaf(u, hu, v * hv), -2.0f * hu, -2.0f * hv, ca);
    rec[1] = make_float4(2.0f * cb, cc, B.y, B.z);
    rec[2] = make_float4(B.w, C.x, C.y, __int_as_float(tag));
    rec[3] = make_float4(A.x, A.y, 0.0f, 0.0f);
}
__device__ __forceinline__ void stage_zero(float4 *rec, int lane) {
    if (lane < 4) rec[lane] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// the fast power of record (r0, r1) at quadrant offset (lx, ly): render_fwd and
// render_bwd use exactly this sequence
__device__ __forceinline__ float quad_power(const float4 &r0, const float4 &r1, float lx, float ly) {
    const float t1 = fmaf(r1.x, ly, fmaf(r0.w, lx, r0.y)), t2 = fmaf(r1.y, ly, r0.z);
    return fmaf(t2, ly, fmaf(t1, lx, r0.x));
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

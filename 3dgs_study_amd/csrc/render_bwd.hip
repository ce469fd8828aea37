// render_bwd.hip — back-to-front replay of the tile compositing (backward).
//
// Replaces upstream BACKWARD::renderCUDA (backward.cu; SURVEY.md §8a row a15,
// Appendix A.7).  Per pixel the recurrence is upstream's: start from final_T,
// walk the tile list from the back, skip entries at or beyond the pixel's
// n_contrib, recompute alpha, divide T by (1 - alpha), keep accum_rec /
// last_alpha / last_color, and produce 9 partial gradients per (pixel, Gaussian).
//
// CDNA4 mapping (gsr_blend.hpp): one independent wave64 per 8x8 quadrant.  The
// wave starts at the largest n_contrib among its own 64 pixels (entries past it
// are skipped by every pixel), streams 64-entry chunks backwards with the same
// lane-parallel exact cull as the forward, and walks the surviving Gaussians
// from the back, two Gaussians per iteration.  Upstream issues ~9 float atomics
// per contributing (pixel, Gaussian) pair; here the 2 x 9 partials are summed
// over the wave's 64 pixels by one reduce-scatter — five ds_swizzle stages
// inside each 32-lane half (the exchanges run in the LDS pipe; DPP adds and
// v_permlane swaps cost 3.5x / 7x a plain VALU op on gfx950, tests/hip/
// xlane_probe.hip) and one v_permlane32 self-swap — and ONE 9-lane atomic
// wave-instruction per Gaussian adds them to its 64-byte accumulator row: a
// single memory-side atomic request (splitting it, e.g. one per 32-lane half,
// doubled the kernel's time).
#include "gsr_blend.hpp"
#include "gsr_kernels.hpp"
#include "gsr_l1.hpp"

namespace gsr {

// Ablation switches for timing builds (results are wrong with any of them on):
// GSR_XB_NOSWZ: the exchanges read the lane's own value (no ds_swizzle),
// GSR_XB_NOTRANS: exp and rcp replaced by multiplies,
// GSR_XB_NOPAIRS: no pair loop (the chunk stream, cull and staging alone).
#ifdef GSR_XB_NOSWZ
#define GSR_SWZ(v, pat) (v)
#else
#define GSR_SWZ(v, pat) __builtin_amdgcn_ds_swizzle((v), (pat))
#endif

// Wave order: per XCD, most forward work first (the buckets the forward filed,
// gsr_blend.hpp), so that the longest replays start at once instead of forming
// the kernel's tail.

struct RenderBwdArgs {
    int W, H, gx, tiles;
    const uint32_t *order_cnt;  // [8][ORDER_NBUCKET] quadrants per (XCD, work bucket)
    uint32_t *flags;            // order_cnt + ORDER_FILED: the OrderFlag words
    const uint32_t *qlist;      // [8][ORDER_NBUCKET][maxc]
    int maxc;
    const uint2 *ranges;
    const uint32_t *point_list;
    const float4 *splats;
    const float *bg;
    const float *final_T;
    const uint32_t *n_contrib;
    const float *dL_dpix;       // [3][H][W], or NULL: the L1 loss's gradient from l1_* (GSR_FLAG_L1_SEED)
    const float *l1_image, *l1_gt, *l1_dloss;
    float l1_n;
    const int8_t *l1_signmap;  // the forward's sign(image - gt) (gsr_l1.hpp), or NULL: formed here from both
    float *accum;
    // the forward's chunk cull masks (render_fwd.hip; binning's qmask region), or NULL
    const uint64_t *qmask;
    size_t qmask_stride;
    // split replay (gsr_common.hpp; MASKS only): SEG or 0, the checkpoint slots (the
    // grid's first 4 nslots workgroups: slot b / 4, quadrant b % 4) and regions
    int seg, nslots;
    const float *ckpt, *cfin;
    const uint32_t *ctab;
};
__device__ __forceinline__ float l1_sign(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }  // torch.sign

// NB: copy the builtin's pair into scalars before bit-casting: with ROCm 7.2's
// clang, __builtin_bit_cast(float, r[1]) on the returned vector silently reads
// element 0 (caught by tests/test_gpu_parity.py; see tests/hip/permlane_probe.hip).
__device__ __forceinline__ float swap32_sum(float a, float b) {  // -> [a_lo + a_hi | b_lo + b_hi]
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t x = r[0], y = r[1];
    return __builtin_bit_cast(float, x) + __builtin_bit_cast(float, y);
}
// One ds_swizzle reduce-scatter step inside each 32-lane half: lanes with bit K
// clear keep c, the others d, and each adds its partner's (lane ^ K) copy of the
// other one.  The exchange runs in the LDS pipe; the VALU pays two selects and
// an add (a DPP add costs ~3.5 plain adds on gfx950, a v_permlane swap ~7).
template <int K>
__device__ __forceinline__ float swz_stage(float c, float d, int lane) {
    const bool hi = (lane & K) != 0;
    const float keep = hi ? d : c, send = hi ? c : d;
    return keep + __builtin_bit_cast(float, GSR_SWZ(__builtin_bit_cast(int, send), 0x1F | (K << 10)));
}

// The same step for an odd register out (c paired with a zero): every lane adds
// its partner's copy, no selects.  Lanes with bit K clear get exactly
// swz_stage<K>(c, 0)'s sum; lanes with bit K set get that sum too instead of 0,
// and no slot lane reads those copies: every slot lane's value is bit for bit
// what the zero-padded stage gives (tests/test_reduce_layout.py simulates the
// whole exchange sequence).
template <int K>
__device__ __forceinline__ float swz_fold(float c) {
    return c + __builtin_bit_cast(float, GSR_SWZ(__builtin_bit_cast(int, c), 0x1F | (K << 10)));
}


// MASKS: the forward's chunk cull masks are in a.qmask (a separate instantiation:
// one kernel carrying both the mask and the cull path ran out of VGPRs)
#ifndef GSR_BWD_WAVES
#define GSR_BWD_WAVES 6
#endif
template <bool MASKS>
__global__ void __launch_bounds__(BLEND_THREADS) __attribute__((amdgpu_waves_per_eu(GSR_BWD_WAVES))) render_bwd_kernel(RenderBwdArgs a) {
    static_assert(BLEND_WAVES == 1, "the backward wave order needs one-wave workgroups");
    // workgroup 8 r + x: XCD x's r-th quadrant in bucket order (gsr_blend.hpp)
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && lane == 0) {  // a second backward of this forward reuses the lists, and re-zeroes
        a.flags[0] = 1u;                 // ORDER_FILED
        a.flags[1] = 0u;                 // ORDER_FRESH
    }
    // Split replay (gsr_common.hpp): the grid's first 4 nslots workgroups replay
    // segment k >= 1 ([k SEG, (k + 1) SEG)) of the split lists, slot by slot (a slot's
    // tile is validated against this forward's ranges: a stale or unwritten word names
    // no segment, or the slot's own); the ordered waves replay segment 0 of every
    // quadrant, i.e. all of an unsplit list.
    const uint32_t seg = MASKS ? (uint32_t)a.seg : 0u;
    const int xb = MASKS ? 4 * a.nslots : 0;  // a multiple of 8: the ordered waves keep their XCD
    int quad = -1;
    uint32_t s0 = 0;  // the segment's first list position
    bool segment = false;
    if constexpr (MASKS) {
        if ((int)blockIdx.x < xb) {
            const uint32_t slot = blockIdx.x >> 2, t = a.ctab[slot];
            if (t >= (uint32_t)a.tiles) return;
            const uint2 rr = a.ranges[t];
            const uint32_t k = slot - rr.x / seg;
            if (slot < rr.x / seg || k == 0u || rr.x + k * seg >= rr.y) return;
            s0 = k * seg;
            quad = (int)(4 * t + (blockIdx.x & 3));
            segment = true;
        }
    }
    if (!segment) {
        quad = ordered_quad(a.order_cnt, a.qlist, a.maxc, (int)blockIdx.x - xb);
        if (quad < 0) return;
    }
    const int tile = (int)(quad >> 2), w = (int)(quad & 3);
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int qx0 = tx * TILE_X + (w & 1) * 8, qy0 = ty * TILE_Y + (w >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float fx = (float)px, fy = (float)py;
    const uint2 r = a.ranges[tile];

    const size_t HW = (size_t)a.W * a.H;
    const size_t pix = inside ? (size_t)a.W * py + px : 0;
    const float T_final = inside ? a.final_T[pix] : 0.f;
    const int last_contrib = inside ? (int)a.n_contrib[pix] : 0;
    float dpx0 = 0.f, dpx1 = 0.f, dpx2 = 0.f;
    if (inside) {
        if (a.dL_dpix) {
            dpx0 = a.dL_dpix[pix];
            dpx1 = a.dL_dpix[HW + pix];
            dpx2 = a.dL_dpix[2 * HW + pix];
        } else {  // L1 seed: gsr_l1_grad's (dloss / n) * sign(image - gt), the same operations
            const float q = a.l1_dloss[0] / a.l1_n;
            if (a.l1_signmap) {  // 3 B per pixel instead of 24 (the same signs: l1_sign_of)
                dpx0 = q * (float)a.l1_signmap[pix];
                dpx1 = q * (float)a.l1_signmap[HW + pix];
                dpx2 = q * (float)a.l1_signmap[2 * HW + pix];
            } else {
                dpx0 = q * l1_sign(a.l1_image[pix] - a.l1_gt[pix]);
                dpx1 = q * l1_sign(a.l1_image[HW + pix] - a.l1_gt[HW + pix]);
                dpx2 = q * l1_sign(a.l1_image[2 * HW + pix] - a.l1_gt[2 * HW + pix]);
            }
        }
    }
    const float bg_dot = a.bg[0] * dpx0 + a.bg[1] * dpx1 + a.bg[2] * dpx2;
    const float nTbg = -T_final * bg_dot;
    int end = last_contrib;  // wave max: the first (from the back) entry any pixel replays
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) end = max(end, __shfl_xor(end, o));
    // the segment [s0, e): the whole list unless it is split
    const uint32_t n = r.y - r.x;
    const uint32_t e = seg && n > seg ? min(s0 + seg, n) : n;
    end = min(end, (int)e);
    if (end <= (int)s0) return;

    __shared__ QuadChunk stage[BLEND_WAVES];
    QuadChunk &st = stage[0];
    // record 0: the dummy b of an odd survivor count — a zero record replays as a
    // skipped Gaussian (alpha 0, finite colour), and its atomic is never issued
    stage_zero(st.rec[0], lane);
    float T = T_final;
    // upstream's accum_rec enters dL/dalpha only as sum_c (c_c - accum_rec_c) dL/dpix_c,
    // so the replay carries its projection D = sum_c accum_rec_c dL/dpix_c (advanced
    // eagerly: after a blended Gaussian it already holds the next Gaussian's value)
    float D = 0.f;
    // A pixel that blends past the segment's end starts from the forward's state
    // there: T = T(e), and accum_rec = the colour the entries from e on composite,
    // relative to T(e): (C_final - C(e)) / T(e) (the forward's checkpoint and final
    // colour).  Others start as upstream's replay does, from final_T.
    if (e < n && last_contrib > (int)e) {
        // planes of 64 floats per (slot, quadrant): {T, C0, C1, C2}, and the final {C0, C1, C2}
        const float *ck = a.ckpt + ((size_t)split_slot(r.x + e, seg) * 4 + w) * 256 + lane;
        const float *cf = a.cfin + ((size_t)split_slot(r.x + seg, seg) * 4 + w) * 256 + lane;
        T = ck[0];
        D = ((cf[0] - ck[64]) * dpx0 + (cf[64] - ck[128]) * dpx1 + (cf[128] - ck[192]) * dpx2) / T;
    }
    const uint32_t *list = a.point_list + r.x;

    // The role-swapped reduce-scatter below leaves Gaussian a's nine sums in lanes
    // {0,8,4,12,2,10,6,14,1} (slots 0..8) and b's in {16,24,20,28,18,26,22,30,17}
    // of ONE register (and again 32 lanes up), so each Gaussian costs one atomic
    // wave-instruction: nine lanes into one 64-B accumulator row = one memory-side
    // atomic request.  (Derived by simulating the exchange stages; tests/
    // test_reduce_layout.py and the gradient parity tests check it.)
    int slot_a = -1, slot_b = -1;
    {
        constexpr int8_t LA[9] = {0, 8, 4, 12, 2, 10, 6, 14, 1};
        constexpr int8_t LB[9] = {16, 24, 20, 28, 18, 26, 22, 30, 17};
#pragma unroll
        for (int j = 0; j < 9; j++) {
            slot_a = lane == LA[j] ? j : slot_a;
            slot_b = lane == LB[j] ? j : slot_b;
        }
    }
    const bool act_a = slot_a >= 0, act_b = slot_b >= 0;
    // slot -> float of the accumulator row: the colour sums (slots 6-8) first, so
    // the exchange's colour read (sh_exchange.hip) touches one 32-B sector per row
    const int off_a = slot_a >= 6 ? slot_a - 6 : slot_a + 3, off_b = slot_b >= 6 ? slot_b - 6 : slot_b + 3;
    // lanes 16-31 (and 48-63) keep Gaussian b's sums in the first exchange stage
    const bool h16 = (lane & 16) != 0;

    // The per-pixel quantities the nine sums of one Gaussian are made of: g5 =
    // G dL/dalpha, d = mean - pixel, t = alpha T.  The opacity factor of
    // W = opacity g5 is per Gaussian: preprocess_bwd.hip applies it to the sums.
    struct Part {
        float g5, dx, dy, t;
    };
    // One Gaussian of the replay (colour r, g, record r2, list position k, d = mean -
    // pixel): power, G and alpha as render_fwd.hip computes them (exact_power, the
    // same instructions on the same staged values, and the same exact re-check near
    // the alpha threshold, done by the caller), then upstream's back-to-front step,
    // branch-free: a skipped pixel sees alpha = 0 (T and D unchanged) and zero
    // gradients.
    auto replay = [&](float power, float G, float alpha, float cr, float cg, const float4 &r2, float dx, float dy,
                      int lim) {
        const int k = __float_as_int(r2.y);  // entry lo + k = upstream `contributor`
        const bool valid = k < lim && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
        const float av = valid ? alpha : 0.0f;
#ifdef GSR_XB_NOTRANS
        const float inv_1ma = 1.f + av;
#else
        const float inv_1ma = __builtin_amdgcn_rcpf(1.f - av);
#endif
        T = T * inv_1ma;
        const float cd = fmaf(cg, dpx1, cr * dpx0) + r2.x * dpx2;  // sum_c colour_c dL/dpix_c
        const float dot = cd - D;                                      // sum_c (colour_c - accum_rec_c) dL/dpix_c
        D = fmaf(av, dot, D);
        // dL/dalpha (upstream: sum_c (c - accum_rec) dL_dpix_c * T - T_final/(1-alpha) * bg.dL_dpix)
        const float dL_dalpha = valid ? fmaf(dot, T, inv_1ma * nTbg) : 0.0f;
        // dG/d(delta) = -G conic d; with W = opacity G dL/dalpha the per-pixel terms
        // are dmean2D = -W (conic d) (W/2, H/2) and dconic = -W/2 (dx^2, dx dy,
        // dy^2); conic, (W, H), -1/2 and the opacity are per-Gaussian constants
        // applied once in preprocess_bwd.hip, so the accumulator holds sum g5 (dx,
        // dy) and sum g5 (dx^2, dx dy, dy^2).  G is finite (power <= 0 for the
        // positive-definite conic), so an invalid pixel's zero dL/dalpha zeroes them.
        Part p;
        p.g5 = G * dL_dalpha;
        p.dx = dx;
        p.dy = dy;
        p.t = av * T;  // dchannel/dcolor
        return p;
    };

    // Reduce-scatter of a pair's 18 sums and their two atomic wave instructions.
    // First stage (xor 16) with swapped roles: lanes 16-31 keep b's values and
    // send a's, and what crosses is three base quantities (g5, dx, dy) and the
    // three colour products of the Gaussian the receiving lane keeps, not its nine
    // sums: each lane forms both pixels' geometric products itself, the partner's
    // terms fused into FMAs.  Then four
    // more ds_swizzle stages (xor 8, 4, 2, 1: LDS-pipe exchanges, 3 plain VALU per
    // output register) and one final v_permlane32 self-swap adding the two halves.
    // the pair's two atomic wave-instructions: row base in SGPRs + per-lane slot;
    // lane-dependent addresses keep the compiler's atomic optimizer (a wave-scan
    // loop) out
    auto emit = [&](float v, uint32_t gida, uint32_t gidb, bool two) {
        if (act_a) atomicAdd(a.accum + (size_t)gida * ACCUM_STRIDE + off_a, v);
        if (two && act_b) atomicAdd(a.accum + (size_t)gidb * ACCUM_STRIDE + off_b, v);
    };
    auto reduce_sum = [&](const Part &pa, const Part &pb) -> float {
        const float k5 = h16 ? pb.g5 : pa.g5, s5 = h16 ? pa.g5 : pb.g5;
        const float kx = h16 ? pb.dx : pa.dx, sx = h16 ? pa.dx : pb.dx;
        const float ky = h16 ? pb.dy : pa.dy, sy = h16 ? pa.dy : pb.dy;
        const float kt = h16 ? pb.t : pa.t, st_ = h16 ? pa.t : pb.t;
        auto x16 = [&](float send) {
            return __builtin_bit_cast(float,
                                      GSR_SWZ(__builtin_bit_cast(int, send), 0x1F | (16 << 10)));
        };
        // the colour terms cross as the sender's own products t dL/dpix_c (no
        // registers held for the partner pixel's dL/dpix)
        const float r5 = x16(s5), rx = x16(sx), ry = x16(sy);
        const float rt0 = x16(st_ * dpx0), rt1 = x16(st_ * dpx1), rt2 = x16(st_ * dpx2);
        const float k0 = k5 * kx, k1 = k5 * ky;
        const float r0 = r5 * rx, r1 = r5 * ry;
        const float o0 = k0 + r0;
        const float o1 = k1 + r1;
        const float o2 = fmaf(k0, kx, r0 * rx);
        const float o3 = fmaf(k0, ky, r0 * ry);
        const float o4 = fmaf(k1, ky, r1 * ry);
        const float o5 = k5 + r5;
        const float o6 = fmaf(kt, dpx0, rt0);
        const float o7 = fmaf(kt, dpx1, rt1);
        const float o8 = fmaf(kt, dpx2, rt2);
        const float t0 = swz_stage<8>(o0, o1, lane);
        const float t1 = swz_stage<8>(o2, o3, lane);
        const float t2 = swz_stage<8>(o4, o5, lane);
        const float t3 = swz_stage<8>(o6, o7, lane);
        const float t4 = swz_fold<8>(o8);
        const float u0 = swz_stage<4>(t0, t1, lane);
        const float u1 = swz_stage<4>(t2, t3, lane);
        const float u2 = swz_fold<4>(t4);
        const float w0 = swz_stage<2>(u0, u1, lane);
        const float w1 = swz_fold<2>(u2);
        const float x0 = swz_stage<1>(w0, w1, lane);
        return swap32_sum(x0, x0);  // both halves: the full sum
    };

    // Replay one 64-entry chunk [lo, lo + 64) from the back (lane l <-> entry lo + l),
    // two Gaussians per iteration: independent LDS reads and exps (ILP), one
    // fused reduce-scatter of their 18 sums.  The survivors sit in records 1..ns
    // (record 0 is the odd pair's dummy b), so pair (a, b) = records (s + 1, s) and
    // both are read from ONE VGPR address with immediate offsets.
    // the forward's cull masks of this quadrant (chunk j of the tile's list at qm[j]), or NULL
    const uint64_t *qm = MASKS ? a.qmask + (size_t)w * a.qmask_stride + qmask_index(r.x, tile, 0) : nullptr;
    auto replay_chunk = [&](int lo, float4 A, float4 B, float4 C, uint64_t m) {
        // the chunk's entries that reach the quadrant: the forward's mask, or the
        // same exact cull on the same records; none at or past `end`
        bool rel;
        if constexpr (MASKS)
            rel = ((m >> lane) & 1ull) != 0 && lo + lane < end;  // (clearing the bits past end in m spilled VGPRs)
        else
            rel = (lo + lane < end) && quad_hit(A.x, A.y, A.z, A.w, B.x, C.z, (float)qx0, (float)qy0);
        const uint64_t mask = __ballot(rel);
        if (rel) stage_quad(st.rec[survivor_slot(mask, 1)], A, B, C, lane);
        const int ns = __builtin_popcountll(mask);
        const int lim = last_contrib - lo;  // entry lo + l replays for this pixel iff l < lim
        // byte offset of record b = k - 1 + 1 in a VGPR (asm barrier: keep it there)
        uint32_t boff = (uint32_t)(ns - 1) * (uint32_t)sizeof(st.rec[0]);
        asm volatile("" : "+v"(boff));
        const volatile char *sbase = reinterpret_cast<const volatile char *>(&st.rec[0][0]);
        // one pair's records, power, G and alpha (the exact exp near 1/255 included)
        struct Cur {
            float pa, pb, Ga, Gb, ala, alb, dxa, dya, dxb, dyb;
            float4 a1, a2, b1, b2;
        };
        auto front = [&](Cur &c) {
            // whole 16-B reads (volatile: the load vectorizer would otherwise split
            // the records into 8-B pieces around the unused fields)
            lds_f32x4 *rb = (lds_f32x4 *)(sbase + boff);
            const float4 b0 = ld4(rb + 0), a0 = ld4(rb + 3);
            c.b1 = ld4(rb + 1);
            c.b2 = ld4(rb + 2);
            c.a1 = ld4(rb + 4);
            c.a2 = ld4(rb + 5);
            boff -= 2 * (uint32_t)sizeof(st.rec[0]);
            c.pa = exact_power(a0, c.a1, fx, fy, c.dxa, c.dya);
            c.pb = exact_power(b0, c.b1, fx, fy, c.dxb, c.dyb);
#ifdef GSR_XB_NOTRANS
            c.Ga = 1.f + c.pa * 0.01f;
            c.Gb = 1.f + c.pb * 0.01f;
#else
            c.Ga = __expf(c.pa);
            c.Gb = __expf(c.pb);
#endif
            // alpha before upstream's `power > 0` skip, which the replay applies (the
            // clamp cannot move a value into or out of the re-check band)
            c.ala = fminf(0.99f, c.a1.y * c.Ga);
            c.alb = fminf(0.99f, c.b1.y * c.Gb);
            if (__builtin_expect(__ballot(blend_near(c.ala) || blend_near(c.alb)) != 0, 0)) {
                // rare: the correctly rounded exp near 1/255 (gsr_blend.hpp)
                if (blend_near(c.ala)) {
                    c.Ga = exp_rn_f32(c.pa);
                    c.ala = fminf(0.99f, c.a1.y * c.Ga);
                }
                if (blend_near(c.alb)) {
                    c.Gb = exp_rn_f32(c.pb);
                    c.alb = fminf(0.99f, c.b1.y * c.Gb);
                }
            }
        };
        // (no early-out for pairs without a contributing pixel: 98.6% of the
        // walked pairs have one at config C, the test cost more than it saved)
#ifdef GSR_XB_NOPAIRS
        if (ns < 0)  // timing build: the chunk stream and cull alone
#endif
        for (int k = ns - 1; k >= 0; k -= 2) {
            const bool two = k >= 1;  // wave-uniform
            Cur c;
            front(c);
            const Part qa = replay(c.pa, c.Ga, c.ala, c.a1.z, c.a1.w, c.a2, c.dxa, c.dya, lim);  // back to front: a before b
            const Part qb = replay(c.pb, c.Gb, c.alb, c.b1.z, c.b1.w, c.b2, c.dxb, c.dyb, lim);   // !two: b is the zero record (alpha 0)
            const uint32_t gida = __builtin_amdgcn_readfirstlane(__float_as_uint(c.a2.z));
            const uint32_t gidb = __builtin_amdgcn_readfirstlane(__float_as_uint(c.b2.z));
            emit(reduce_sum(qa, qb), gida, gidb, two);
        }
    };
    // Double-buffered backwards stream over the forward's chunks (list positions
    // [64 j, 64 j + 64), from the one holding entry end - 1 down to 0: the chunks the
    // forward culled, so its masks apply and every backward pairs the survivors
    // alike), unrolled by two so the buffers swap roles instead of being copied (see
    // render_fwd.hip).  Indices are clamped so every load is unconditional; with the
    // forward's masks a lane whose entry misses the quadrant loads the chunk's first
    // survivor's record instead (one line for all of them).  The one wait per chunk
    // also drains the previous chunk's accumulator atomics, none are waited for
    // inside the Gaussian loop.
    const int jend = (end - 1) >> 6, e1 = end - 1, js = (int)(s0 >> 6);
    auto cmask = [&](int j) -> uint64_t { return !MASKS || j < 0 ? ~0ull : qm[j]; };
    auto pick = [&](uint32_t idx, uint64_t m) -> uint32_t {
        if constexpr (!MASKS) return idx;
        const uint32_t first = __builtin_amdgcn_readlane(idx, m ? __builtin_ctzll(m) : 0);
        return ((m >> lane) & 1ull) ? idx : first;
    };
    auto at_list = [&](int j) { return list[min(max(64 * j + lane, 0), e1)]; };
    uint64_t mj = cmask(jend), mb = cmask(jend - 1), ma, mc;
    const float4 *sp = a.splats + 3 * (size_t)pick(at_list(jend), mj);
    float4 A0 = sp[0], B0 = sp[1], C0 = sp[2], A1, B1, C1;
    uint32_t idx_a, idx_b = at_list(jend - 1);
    for (int j = jend;;) {
        idx_a = at_list(j - 2);
        ma = cmask(j - 2);
        sp = a.splats + 3 * (size_t)pick(idx_b, mb);
        A1 = sp[0];
        B1 = sp[1];
        C1 = sp[2];
        wait_vmcnt_4();
        replay_chunk(64 * j, A0, B0, C0, mj);
        if (--j < js) break;
        idx_b = at_list(j - 2);
        mc = cmask(j - 2);
        sp = a.splats + 3 * (size_t)pick(idx_a, ma);
        A0 = sp[0];
        B0 = sp[1];
        C0 = sp[2];
        wait_vmcnt_4();
        replay_chunk(64 * j, A1, B1, C1, mb);
        if (--j < js) break;
        mj = ma;
        mb = mc;
    }
}

// The backward's preparation: zeroes the accumulator rows (in place of a memset
// launch) and files every quadrant under (its XCD, the work bucket the forward
// stored) for render_bwd_kernel's wave order: per wave of 64 quadrants, ONE
// returning atomic instruction, each distinct (XCD, bucket) cell's lowest lane
// reserving its peers' slots (a dependent atomic per cell cost ~20 us of latency).
// In the backward (forward == 0) it is the first launch, and skips what a forward
// called with GSR_FLAG_PREPARE_BACKWARD did already (the flag words); a second
// backward of the same forward (retain_graph) finds the lists filed and only
// zeroes.  In that forward (forward == 1) it files, after render_fwd, and marks
// the flags (its accumulator was zeroed beside render_fwd, abi.hip).
struct BwdPrepArgs {
    float4 *accum4;
    size_t n4;
    const uint8_t *qbucket;
    uint32_t *order_cnt;  // [8][ORDER_NBUCKET] + the OrderFlag words
    uint32_t *qlist;
    int nq, maxc;
    int internal;         // accum4 is geom's accumulator (ORDER_FRESH applies to it)
    int forward;
    // gsr_forward_render_l1: workgroups [file_blocks, file_blocks + l1_nb) write the
    // L1 loss's partial sums instead (l1_x NULL: none)
    int file_blocks, l1_nb;
    const float *l1_x, *l1_y;
    size_t l1_n;
    float *l1_part;
    // ... and the last of them to finish forms the loss (gsr_l1.hpp l1_finish_last_block)
    uint32_t *l1_ticket;
    float l1_invN;
    float *l1_out;
    int8_t *l1_sign;  // ... and the signs of image - gt for the seeded backward (img's l1_sign)
    // ... and workgroups after those write visible[i] = radii[i] > 0 (render()'s
    // visibility_filter), or NULL
    const int32_t *radii;
    uint8_t *visible;
    int P, vis_nb;
};
constexpr int PREP_THREADS = 256;
static_assert(PREP_THREADS == L1_THREADS, "the L1 partial blocks share the launch");
__global__ void __launch_bounds__(PREP_THREADS) bwd_prepare_kernel(BwdPrepArgs a) {
    if ((int)blockIdx.x >= a.file_blocks + a.l1_nb) {  // workgroup-uniform: a visibility block
        const int v = ((int)blockIdx.x - a.file_blocks - a.l1_nb) * PREP_THREADS * 4 + (int)threadIdx.x * 4;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (v + k < a.P) a.visible[v + k] = a.radii[v + k] > 0 ? 1 : 0;
        return;
    }
    if ((int)blockIdx.x >= a.file_blocks) {  // workgroup-uniform: an L1 partial-sum block
        l1_block_partial(a.l1_x, a.l1_y, a.l1_n, (int)blockIdx.x - a.file_blocks, a.l1_nb, a.l1_part, true,
                         a.l1_sign);
        l1_finish_last_block(a.l1_part, (int)blockIdx.x - a.file_blocks, a.l1_nb, a.l1_ticket, a.l1_invN, a.l1_out);
        return;
    }
    const size_t tid = (size_t)blockIdx.x * PREP_THREADS + threadIdx.x;
    const size_t nthreads = (size_t)a.file_blocks * PREP_THREADS;
    if (a.forward) {
        // the next kernel (a backward's first) reads these; no block of this one does
        if (tid == 0) {
            a.order_cnt[ORDER_FILED] = 1u;
            a.order_cnt[ORDER_FRESH] = 1u;
        }
    } else if (!(a.internal && a.order_cnt[ORDER_FRESH] != 0u)) {
        for (size_t i = tid; i < a.n4; i += nthreads) a.accum4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (a.nq <= 0 || (!a.forward && a.order_cnt[ORDER_FILED] != 0u)) return;  // nothing to file / already filed
    const int lane = threadIdx.x & 63;
    for (size_t q0 = tid - (size_t)lane; q0 < (size_t)a.nq; q0 += nthreads) {  // wave-uniform
        const int q = (int)q0 + lane;
        const uint32_t bk = q < a.nq ? a.qbucket[q] : 0xFFu;  // 0xFF: nothing to replay
        const int cell = bk < (uint32_t)ORDER_NBUCKET ? quad_xcd(q) * ORDER_NBUCKET + (int)bk : -1;
        // each lane's peers (the lanes filing into the same cell), from ballots alone
        uint64_t peers = 0, todo = __ballot(cell >= 0);
        while (todo) {
            const int lc = __builtin_amdgcn_readlane(cell, __builtin_ctzll(todo));
            const uint64_t m = __ballot(cell == lc);
            peers = cell == lc ? m : peers;
            todo &= ~m;
        }
        // then ONE atomic instruction: each cell's lowest lane reserves its peers' slots
        const int leader = peers ? __builtin_ctzll(peers) : lane;
        uint32_t base = 0;
        if (cell >= 0 && lane == leader) base = atomicAdd(&a.order_cnt[cell], (uint32_t)__builtin_popcountll(peers));
        base = (uint32_t)__shfl((int)base, leader);
        // (a cell never holds more than maxc quadrants: the guard only keeps a
        // mis-sequenced caller — lists filed twice — from writing past the cell)
        const uint32_t slot =
            base + __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
        if (cell >= 0 && slot < (uint32_t)a.maxc) a.qlist[(size_t)cell * a.maxc + slot] = (uint32_t)q;
    }
}

hipError_t launch_bwd_prepare(const gsr_inputs &in, void *geom, const void *img, float *accum, bool file,
                              bool internal, bool forward, hipStream_t s, const float *l1_x, const float *l1_y,
                              float *l1_out, const int32_t *radii, uint8_t *visible) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    const ImgLayout Im = img_layout(in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    BwdPrepArgs a;
    a.accum4 = reinterpret_cast<float4 *>(accum);
    a.n4 = (size_t)(in.P > 0 ? in.P : 1) * (ACCUM_STRIDE / 4);
    a.qbucket = at<uint8_t>(const_cast<void *>(img), Im.qbucket);
    a.order_cnt = at<uint32_t>(geom, G.order_cnt);
    a.qlist = at<uint32_t>(const_cast<void *>(img), Im.qlist);
    a.nq = file ? 4 * g.tiles : 0;
    a.maxc = order_max_per_xcd(4 * g.tiles);
    a.internal = internal ? 1 : 0;
    a.forward = forward ? 1 : 0;
    const size_t want = forward ? ((size_t)a.nq + PREP_THREADS - 1) / PREP_THREADS : (a.n4 + PREP_THREADS - 1) / PREP_THREADS;
    const int blocks = (int)(want < 2048 ? (want > 0 ? want : 1) : 2048);
    a.file_blocks = blocks;
    a.l1_x = l1_x;
    a.l1_y = l1_y;
    a.l1_n = (size_t)3 * in.W * in.H;
    a.l1_nb = l1_x ? l1_blocks(a.l1_n) : 0;
    a.l1_part = l1_x ? at<float>(const_cast<void *>(img), Im.l1_part) : nullptr;
    a.l1_ticket = at<uint32_t>(const_cast<void *>(img), Im.l1_ticket);
    a.l1_invN = 1.0f / (float)(double)a.l1_n;  // launch_l1_finish's invN
    a.l1_out = l1_out;
    a.l1_sign = l1_x ? at<int8_t>(const_cast<void *>(img), Im.l1_sign) : nullptr;
    a.radii = radii;
    a.visible = visible;
    a.P = in.P;
    a.vis_nb = visible ? (in.P + PREP_THREADS * 4 - 1) / (PREP_THREADS * 4) : 0;
    hipLaunchKernelGGL(bwd_prepare_kernel, dim3(blocks + a.l1_nb + a.vis_nb), dim3(PREP_THREADS), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_render_bwd(const gsr_inputs &in, const void *geom, const void *binning, const void *img,
                             const float *dL_dpix, const gsr_l1_seed *l1, float *accum, hipStream_t s,
                             int64_t qmask_cap, bool l1_signs, int seg) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    const ImgLayout Im = img_layout(in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    RenderBwdArgs a;
    a.W = in.W;
    a.H = in.H;
    a.gx = g.gx;
    a.tiles = g.tiles;
    a.ranges = at<uint2>(geom, G.off[GSR_GEOM_RANGES]);
    a.point_list = static_cast<const uint32_t *>(binning);  // GSR_BIN_POINT_LIST: offset 0 (gsr_common.hpp)
    a.splats = at<float4>(geom, G.off[GSR_GEOM_SPLATS]);
    a.bg = in.bg;
    a.final_T = at<float>(img, Im.off[GSR_IMG_FINAL_T]);
    a.n_contrib = at<uint32_t>(img, Im.off[GSR_IMG_N_CONTRIB]);
    a.dL_dpix = dL_dpix;
    a.l1_image = l1 ? l1->image : nullptr;
    a.l1_gt = l1 ? l1->gt : nullptr;
    a.l1_dloss = l1 ? l1->dloss : nullptr;
    a.l1_n = l1 ? (float)(double)l1->n : 0.f;  // gsr_l1_grad's fN
    a.l1_signmap = l1 && l1_signs ? at<int8_t>(img, Im.l1_sign) : nullptr;
    a.accum = accum;
    a.order_cnt = at<uint32_t>(geom, G.order_cnt);
    a.flags = at<uint32_t>(const_cast<void *>(geom), G.order_cnt) + ORDER_FILED;
    a.qlist = at<uint32_t>(img, Im.qlist);
    a.maxc = order_max_per_xcd(4 * g.tiles);
    a.qmask = nullptr;
    a.qmask_stride = 0;
    a.seg = a.nslots = 0;
    a.ckpt = a.cfin = nullptr;
    a.ctab = nullptr;
    if (qmask_cap > 0) {
        const BinningLayout B = binning_layout(qmask_cap, in.W, in.H);
        a.qmask = at<uint64_t>(binning, B.qmask);
        a.qmask_stride = B.qmask_stride;
        if (seg > 0) {  // the forward's checkpoints: slots 0 .. cap / seg
            a.seg = seg;
            a.nslots = (int)((qmask_cap / seg + 2 + 1) & ~1ll);  // even: 4 nslots workgroups, a multiple of 8
            a.ckpt = at<float>(binning, B.ckpt);
            a.cfin = at<float>(binning, B.cfin);
            a.ctab = at<uint32_t>(binning, B.ctab);
        }
    }
    if (a.qmask)
        hipLaunchKernelGGL(render_bwd_kernel<true>, dim3(4 * a.nslots + 8 * a.maxc), dim3(BLEND_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL(render_bwd_kernel<false>, dim3(8 * a.maxc), dim3(BLEND_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr

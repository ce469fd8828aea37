// render_fwd.hip — 16x16-tile front-to-back alpha compositing (forward).
//
// Replaces upstream FORWARD::renderCUDA (forward.cu; SURVEY.md §8a row a14,
// Appendix A.6).  Per pixel the semantics are upstream's: walk the tile's
// depth-sorted list, skip power > 0 and alpha < 1/255, stop when T would drop
// below 1e-4 (that Gaussian is not blended), record n_contrib = list position
// of the last blended Gaussian and final_T.
//
// CDNA4 mapping (gsr_blend.hpp): each wave64 owns an 8x8 quadrant and runs on
// its own — no LDS, no workgroup barrier — so a quadrant that saturates early
// retires its wave at once.  Chunks of 64 list entries are gathered one per
// lane (ids two chunks ahead, 48-B splat records one chunk ahead, hiding the
// dependent-load latency behind the current chunk's blending; one vmcnt wait per
// chunk, none in the per-Gaussian loop), culled exactly
// against the quadrant in parallel, and the surviving Gaussians are blended in
// list order with their parameters broadcast from a per-wave LDS image.
#include "gsr_blend.hpp"
#include "gsr_kernels.hpp"
#include "gsr_l1.hpp"

namespace gsr {

struct RenderFwdArgs {
    int W, H, gx, tiles;
    const uint2 *ranges;
    const uint32_t *point_list;
    const float4 *splats;
    const float *bg;
    float *out_color;
    float *final_T;
    uint32_t *n_contrib;
    uint8_t *qbucket;  // [4 * tiles] (img)
    // GSR_FLAG_PREPARE_BACKWARD: the backward's accumulator, zeroed here — this
    // kernel is bound by instruction issue, not bytes, so its 64 B per Gaussian of
    // stores ride along (a separate memset launch took 10 us at config C)
    float4 *zero4;
    size_t zero_n4;
    // the backward's wave-order counts and flag words (gsr_blend.hpp), cleared by
    // workgroup 0: this forward's quadrants are filed afresh (bwd_prepare_kernel),
    // however many forwards ran on the geom buffer since its preprocess
    uint32_t *order_cnt;
    uint32_t *l1_ticket;  // img's L1 finish ticket (gsr_l1.hpp), cleared by workgroup 0 for bwd_prepare_kernel
    // GSR_FLAG_PREPARE_BACKWARD: each chunk's cull mask, for render_bwd (binning's
    // qmask: quadrant w at w * qmask_stride, chunk slot qmask_index), or NULL
    uint64_t *qmask;
    size_t qmask_stride;
    // split replay (gsr_common.hpp; qmask set): SEG, or 0; the checkpoint regions
    int seg, seg_log2;
    float *ckpt, *cfin;  // [slot][quadrant][4 | 3][64]: {T, C} planes; the final C planes
    uint32_t *ctab;
};

#ifndef GSR_FWD_GROUP
#define GSR_FWD_GROUP 2
#endif
constexpr int FWD_GROUP_MAIN = GSR_FWD_GROUP;  // Gaussians per blend iteration (zero records after the survivors pad the last group)
// the split-replay instantiation runs where a few long lists set the kernel's time
// (config B): there a wave's serial chain, not the issue rate, is the bound, so
// more Gaussians per iteration (more independent work per step of the chain)
#ifndef GSR_FWD_GROUP_SPLIT
#define GSR_FWD_GROUP_SPLIT 3
#endif
static_assert(FWD_GROUP_MAIN >= 1 && FWD_GROUP_MAIN <= 3 && GSR_FWD_GROUP_SPLIT >= 1 && GSR_FWD_GROUP_SPLIT <= 3,
              "QuadChunk holds 64 survivors + 2 zero records");

// The survivors of a chunk are staged as QuadChunk records (gsr_blend.hpp): the
// power is upstream's expression in upstream's order (exact_power), the same
// instructions render_bwd uses.  The zero record after the survivors lets the
// odd count's second Gaussian blend nothing without a mask (render_fwd 145 ->
// 142 us at C, 374-379 -> 370 us at E).
// SPLIT: the split replay's checkpoints (gsr_common.hpp) — a separate instantiation,
// so that the unsplit kernel keeps its 64 VGPRs (8 waves per SIMD; the checkpoint
// path costs 2-4 more)
template <bool SPLIT>
__device__ __forceinline__ void render_fwd_body(const RenderFwdArgs &a) {
    constexpr int FWD_GROUP = SPLIT ? GSR_FWD_GROUP_SPLIT : FWD_GROUP_MAIN;
    auto zero_slice = [&]() {  // every workgroup its slice of the backward's accumulator
        if (a.zero4) {
            const size_t per = (a.zero_n4 + gridDim.x - 1) / gridDim.x, z0 = (size_t)blockIdx.x * per;
            const size_t z1 = z0 + per < a.zero_n4 ? z0 + per : a.zero_n4;
            for (size_t i = z0 + threadIdx.x; i < z1; i += BLEND_THREADS) a.zero4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    const QuadSlot qs = quad_slot(a.tiles);
    const int tile = qs.tile, w = qs.w, lane = threadIdx.x & 63;
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < ORDER_FILED + 2; i += BLEND_THREADS) a.order_cnt[i] = 0u;
        if (threadIdx.x < L1_TICKETS) a.l1_ticket[threadIdx.x * L1_TICKET_STRIDE] = 0u;
    }
    if (tile < 0) {
        zero_slice();
        return;
    }
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int qx0 = tx * TILE_X + (w & 1) * 8, qy0 = ty * TILE_Y + (w >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float fpx = (float)px, fpy = (float)py;
    const uint2 r = a.ranges[tile];
    const int n = (int)(r.y - r.x);

    float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
    uint32_t last = 0;
    uint32_t work = 0;  // wave-uniform: surviving Gaussians walked (~ the backward's replay work)
    // the pixel's skip threshold on alpha: upstream's 1/255 while it blends, 2
    // (above any alpha) once it has stopped or when it lies outside the image
    float thr = inside ? 1.0f / 255.0f : 2.0f;
    __shared__ QuadChunk stage[BLEND_WAVES];
    QuadChunk &st = stage[BLEND_WAVES == 1 ? 0 : w];
    if (__any(inside) && n > 0) {
        const uint32_t *list = a.point_list + r.x;
        const int nm1 = n - 1;
        uint64_t *qm = a.qmask ? a.qmask + (size_t)w * a.qmask_stride + qmask_index(r.x, tile, 0) : nullptr;
        // Blend one 64-entry chunk starting at list position pos (lane l <-> entry
        // pos + l); returns true once every pixel of the quadrant is saturated.
        auto blend_chunk = [&](int pos, float4 A, float4 B, float4 C) -> bool {
            const bool rel = (pos + lane < n) && quad_hit(A.x, A.y, A.z, A.w, B.x, C.z, (float)qx0, (float)qy0);
            const uint64_t mask = __ballot(rel);
            // the backward replays exactly these entries (the same cull on the same
            // records): one 8-B store per chunk spares it the cull and the gathers of
            // the entries that miss the quadrant
            if (qm && lane == 0) qm[pos >> 6] = mask;
            if (rel) stage_quad(st.rec[survivor_slot(mask, 0)], A, B, C, pos + lane + 1);
            const int ns = __builtin_popcountll(mask);
            stage_zero(st.rec[ns], lane);
            if (FWD_GROUP > 2) stage_zero(st.rec[ns + 1], lane);
            work += ns;
            // FWD_GROUP Gaussians per iteration: their LDS reads, powers and exps are
            // independent, so each wave has that much instruction-level parallelism
            // to cover LDS and transcendental latency; only the T recurrence is serial.
            for (int k = 0; k < ns; k += FWD_GROUP) {
                float pw[FWD_GROUP], al[FWD_GROUP], cr[FWD_GROUP], cg[FWD_GROUP], cb[FWD_GROUP], op[FWD_GROUP];
                int li[FWD_GROUP];
                bool near = false, all_done = false;
#pragma unroll
                for (int g = 0; g < FWD_GROUP; g++) {
                    const int kg = k + g;  // ns itself: the zero record
                    lds_f32x4 *rp = (lds_f32x4 *)&st.rec[kg][0];
                    const float4 r0 = ld4(rp), r1 = ld4(rp + 1);
                    const float2 r2 = ld2((lds_f32x2 *)(rp + 2));  // {b, tag}: 8 of the record's last 16 B
                    li[g] = __float_as_int(r2.y);
                    float dx, dy;
                    pw[g] = exact_power(r0, r1, fpx, fpy, dx, dy);
                    op[g] = r1.y;
                    // alpha before upstream's `power > 0` skip, which the step below
                    // applies with the alpha skip (the clamp cannot move a value into
                    // or out of the re-check band)
                    al[g] = fminf(0.99f, op[g] * __expf(pw[g]));
                    near = near || blend_near(al[g]);
                    cr[g] = r1.z;
                    cg[g] = r1.w;
                    cb[g] = r2.x;
                }
                if (__builtin_expect(__ballot(near) != 0, 0)) {  // rare: the correctly rounded exp (gsr_blend.hpp)
#pragma unroll
                    for (int g = 0; g < FWD_GROUP; g++)
                        if (blend_near(al[g])) al[g] = fminf(0.99f, op[g] * exp_rn_f32(pw[g]));
                }
                // a = the alpha this pixel takes: 0 when upstream would skip the
                // Gaussian (power > 0 or alpha < 1/255, or the pixel finished: thr =
                // 2); a zero alpha leaves T and C unchanged.
                // Selects on VGPRs only: the per-Gaussian SALU work of bool masks and
                // exec juggling, one scalar unit per CU, bounded this loop.
                float av[FWD_GROUP], tt[FWD_GROUP];
#pragma unroll
                for (int g = 0; g < FWD_GROUP; g++) av[g] = (al[g] < thr || pw[g] > 0.0f) ? 0.0f : al[g];
                // Upstream's stop test: T (1 - a) < 1e-4 means that Gaussian is not
                // blended and the pixel stops.  All the group's products are formed up
                // front: T (1 - a0) (1 - a1) ..., rounded step by step, never grows (a
                // factor <= 1 never rounds a product up past its other factor), so the
                // last test alone says whether any fires.  A finished pixel (thr = 2:
                // a = 0) or one outside the image keeps T >= 1e-4 and never fires, so
                // the rare branch runs at most once per stopping pixel; it only zeroes
                // the alphas that upstream's step would not blend and picks the T each
                // step leaves — the blend below is the same arithmetic in the same order
                // either way.
#pragma unroll
                for (int g = 0; g < FWD_GROUP; g++) tt[g] = (g ? tt[g - 1] : T) * (1 - av[g]);
                if (__builtin_expect(__ballot(tt[FWD_GROUP - 1] < 0.0001f) != 0, 0)) {
#pragma unroll
                    for (int g = 0; g < FWD_GROUP; g++) {
                        const bool sg = tt[g] < 0.0001f;  // once one fires, the later ones do
                        av[g] = sg ? 0.0f : av[g];
                        tt[g] = sg ? (g ? tt[g - 1] : T) : tt[g];
                        if (g == FWD_GROUP - 1) thr = sg ? 2.0f : thr;
                    }
                    all_done = !__any(thr < 1.0f);  // thr only changes here
                }
#pragma unroll
                for (int g = 0; g < FWD_GROUP; g++) {
                    const float w = av[g] * (g ? tt[g - 1] : T);
                    C0 += cr[g] * w;
                    C1 += cg[g] * w;
                    C2 += cb[g] * w;
                }
                T = tt[FWD_GROUP - 1];
#pragma unroll
                for (int g = 0; g < FWD_GROUP; g++) last = av[g] > 0.0f ? (uint32_t)li[g] : last;  // tag: position + 1
                if (all_done) return true;
            }
            return false;
        };
        // Double-buffered stream, unrolled by two so the buffers swap roles instead
        // of being copied (a register copy of an in-flight load would force a full
        // vmcnt drain).  Indices are clamped: every load is unconditional, so the
        // single wait per chunk keeps exactly the 4 prefetch loads in flight.
        // Split replay (gsr_common.hpp): a list longer than SEG stores each pixel's
        // state {T, C} before every SEG-th entry (at the chunk's start, ahead of its
        // prefetch: the one wait per chunk then also covers the stores), and the final
        // colour once at the end; the backward replays the segments in waves of their
        // own.  SEG is a power of two, so the test and the slot come from the chunk
        // position alone (a loop-carried "next checkpoint" lived in a VGPR: render_fwd
        // 64 -> 68 VGPRs, 8 -> 7 waves per SIMD).
        const bool split = SPLIT && n > a.seg;
        const int smask = split ? a.seg - 1 : 0x7fffffff;
        auto checkpoint = [&](int pos) {
            const uint32_t slot = (r.x + (uint32_t)pos) >> a.seg_log2;  // split_slot
            // four planes of 64 floats, a dword store straight from each state register
            // (the lane offset made here: hoisted, a per-lane address costs the loop registers)
            uint32_t lo = (uint32_t)lane * 4u;  // bytes: the stores take a scalar base + 32-bit offset
            asm volatile("" : "+v"(lo));
            char *ck = reinterpret_cast<char *>(a.ckpt + ((size_t)slot * 4 + w) * 256);
            *reinterpret_cast<float *>(ck + lo) = T;
            *reinterpret_cast<float *>(ck + 256 + lo) = C0;
            *reinterpret_cast<float *>(ck + 512 + lo) = C1;
            *reinterpret_cast<float *>(ck + 768 + lo) = C2;
            if (lane == 0) a.ctab[slot] = (uint32_t)tile;  // every quadrant that gets here: the same word
        };
        const float4 *sp = a.splats + 3 * (size_t)list[min(lane, nm1)];
        float4 A0 = sp[0], B0 = sp[1], C0_ = sp[2], A1, B1, C1_;
        uint32_t idx_a, idx_b = list[min(64 + lane, nm1)];
        for (int pos = 0;;) {
            if (SPLIT && (pos & smask) == 0 && pos > 0) checkpoint(pos);
            idx_a = list[min(pos + 128 + lane, nm1)];
            sp = a.splats + 3 * (size_t)idx_b;
            A1 = sp[0];
            B1 = sp[1];
            C1_ = sp[2];
            wait_vmcnt_4();
            if (blend_chunk(pos, A0, B0, C0_)) break;
            if ((pos += 64) >= n) break;
            if (SPLIT && (pos & smask) == 0 && pos > 0) checkpoint(pos);
            idx_b = list[min(pos + 128 + lane, nm1)];
            sp = a.splats + 3 * (size_t)idx_a;
            A0 = sp[0];
            B0 = sp[1];
            C0_ = sp[2];
            wait_vmcnt_4();
            if (blend_chunk(pos, A1, B1, C1_)) break;
            if ((pos += 64) >= n) break;
        }
        if (split) {
            float *cf = a.cfin + ((size_t)((r.x + (uint32_t)a.seg) >> a.seg_log2) * 4 + w) * 256;
            cf[lane] = C0;
            cf[64 + lane] = C1;
            cf[128 + lane] = C2;
        }
    }
    // the quadrant's work bucket for the backward's wave order (filed by bwd_prepare_kernel,
    // render_bwd.hip): a plain byte store (an atomic filing here, one returning atomic per
    // wave on 256 counters, held every wave until its return: +19 us at config E)
    // (0xFF: no Gaussian reached the quadrant, every n_contrib is 0 and the backward
    // has nothing to replay — not filed, so no backward wave is spent on it)
    if (lane == 0) a.qbucket[4 * tile + w] = work ? (uint8_t)order_bucket(work) : (uint8_t)0xFF;
    if (inside) {
        const size_t pix = (size_t)a.W * py + px;
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[HW + pix] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix] = C2 + T * a.bg[2];
    }
    // last: the zeroing stores go out behind the outputs, after the last wait (at the
    // kernel's start they sat in the chunk loop's vmcnt waits: 128-129 vs 126-127 us)
    zero_slice();
}

__global__ void __launch_bounds__(BLEND_THREADS) __attribute__((amdgpu_waves_per_eu(7))) render_fwd_kernel(RenderFwdArgs a) {
    render_fwd_body<false>(a);
}
// the split-replay form (checkpoints, groups of GSR_FWD_GROUP_SPLIT).  (Records two
// chunks ahead in a third buffer, 85 VGPRs at 5 waves per SIMD: render_fwd 42.8 ->
// 51.7 us at config B — the long lists' waves do not run alone enough for the
// lost occupancy to pay.)
__global__ void __launch_bounds__(BLEND_THREADS) __attribute__((amdgpu_waves_per_eu(7))) render_fwd_split_kernel(RenderFwdArgs a) {
    render_fwd_body<true>(a);
}

hipError_t launch_render_fwd(const gsr_inputs &in, void *geom, const void *binning, void *img, float *out_color,
                             float *acc_zero, size_t acc_bytes, hipStream_t s, int64_t qmask_cap, int seg) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    const ImgLayout Im = img_layout(in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    RenderFwdArgs a;
    a.W = in.W;
    a.H = in.H;
    a.gx = g.gx;
    a.tiles = g.tiles;
    a.ranges = at<uint2>(geom, G.off[GSR_GEOM_RANGES]);
    a.point_list = static_cast<const uint32_t *>(binning);  // GSR_BIN_POINT_LIST: offset 0 (gsr_common.hpp)
    a.splats = at<float4>(geom, G.off[GSR_GEOM_SPLATS]);
    a.bg = in.bg;
    a.out_color = out_color;
    a.final_T = at<float>(img, Im.off[GSR_IMG_FINAL_T]);
    a.n_contrib = at<uint32_t>(img, Im.off[GSR_IMG_N_CONTRIB]);
    a.qbucket = at<uint8_t>(img, Im.qbucket);
    a.zero4 = reinterpret_cast<float4 *>(acc_zero);
    a.zero_n4 = acc_zero ? acc_bytes / sizeof(float4) : 0;
    a.order_cnt = at<uint32_t>(geom, G.order_cnt);
    a.l1_ticket = at<uint32_t>(img, Im.l1_ticket);
    a.qmask = nullptr;
    a.qmask_stride = 0;
    a.seg = a.seg_log2 = 0;
    a.ckpt = a.cfin = nullptr;
    a.ctab = nullptr;
    if (binning && qmask_cap > 0) {
        const BinningLayout B = binning_layout(qmask_cap, in.W, in.H);
        a.qmask = at<uint64_t>(const_cast<void *>(binning), B.qmask);
        a.qmask_stride = B.qmask_stride;
        if (seg > 0) {
            a.seg = seg;
            a.seg_log2 = __builtin_ctz((unsigned)seg);
            a.ckpt = at<float>(const_cast<void *>(binning), B.ckpt);
            a.cfin = at<float>(const_cast<void *>(binning), B.cfin);
            a.ctab = at<uint32_t>(const_cast<void *>(binning), B.ctab);
        }
    }
    if (a.seg)
        hipLaunchKernelGGL(render_fwd_split_kernel, dim3(blend_grid(g.tiles)), dim3(BLEND_THREADS), 0, s, a);
    else
        hipLaunchKernelGGL(render_fwd_kernel, dim3(blend_grid(g.tiles)), dim3(BLEND_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr

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
// from the back.  Upstream issues ~9 float atomics per contributing
// (pixel, Gaussian) pair; here the 9 partials are summed over the wave's 64
// pixels by a reduce-scatter (v_permlane32_swap, v_permlane16_swap, then DPP row
// shifts: 28 VALU for all nine sums instead of 63) and ONE 9-lane atomic
// wave-instruction adds them to the Gaussian's 64-byte accumulator row.
#include "gsr_blend.hpp"
#include "gsr_kernels.hpp"

namespace gsr {

struct RenderBwdArgs {
    int W, H, gx, tiles;
    const uint2 *ranges;
    const uint32_t *point_list;
    const float4 *splats;
    const float *bg;
    const float *final_T;
    const uint32_t *n_contrib;
    const float *dL_dpix;
    float *accum;
};

// NB: copy the builtin's pair into scalars before bit-casting: with ROCm 7.2's
// clang, __builtin_bit_cast(float, r[1]) on the returned vector silently reads
// element 0 (caught by tests/test_gpu_parity.py; see tests/hip/permlane_probe.hip).
__device__ __forceinline__ float swap32_sum(float a, float b) {  // -> [a_lo + a_hi | b_lo + b_hi]
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t x = r[0], y = r[1];
    return __builtin_bit_cast(float, x) + __builtin_bit_cast(float, y);
}
__device__ __forceinline__ float swap16_sum(float a, float b) {  // rows: [a0+a1 | b0+b1 | a2+a3 | b2+b3]
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                                                    false, false);
    const uint32_t x = r[0], y = r[1];
    return __builtin_bit_cast(float, x) + __builtin_bit_cast(float, y);
}
__device__ __forceinline__ float row_sum_to_lane15(float v) {  // sum of each 16-lane row lands in its lane 15
    v += dpp_f32<DPP_ROW_SHR1>(v);
    v += dpp_f32<DPP_ROW_SHR2>(v);
    v += dpp_f32<DPP_ROW_SHR4>(v);  // only lane 15 is consumed: no bank masks needed,
    v += dpp_f32<DPP_ROW_SHR8>(v);  // so each step is one v_add_f32_dpp
    return v;
}

__global__ void __launch_bounds__(BLEND_THREADS) render_bwd_kernel(RenderBwdArgs a) {
    const int tile = xcd_tile(blockIdx.x, a.tiles);
    if (tile < 0) return;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
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
        dpx0 = a.dL_dpix[pix];
        dpx1 = a.dL_dpix[HW + pix];
        dpx2 = a.dL_dpix[2 * HW + pix];
    }
    const float bg_dot = a.bg[0] * dpx0 + a.bg[1] * dpx1 + a.bg[2] * dpx2;
    const float ddelx_dx = 0.5f * (float)a.W, ddely_dy = 0.5f * (float)a.H;
    int end = last_contrib;  // wave max: the first (from the back) entry any pixel replays
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) end = max(end, __shfl_xor(end, o));
    if (end <= 0) return;

    __shared__ ChunkStage stage[BLEND_THREADS / 64];
    ChunkStage &st = stage[w];
    float T = T_final;
    float R0 = 0.f, R1 = 0.f, R2 = 0.f;
    const bool row_last = (lane & 15) == 15;
    // accumulator slot of the sum each row-last lane holds: lanes 15/31/47/63 -> +0/+2/+1/+3
    const int slot = ((lane >> 4) & 1) * 2 + (lane >> 5);
    const uint32_t *list = a.point_list + r.x;

    // Replay one 64-entry chunk [lo, lo + 64) from the back (lane l <-> entry lo + l).
    auto replay_chunk = [&](int lo, float4 A, float4 B, float4 C) {
        stage_chunk(st, lane, A, B, C);
        const bool rel = (lo + lane >= 0) && quad_hit(A.x, A.y, A.z, A.w, B.x, C.z, (float)qx0, (float)qy0);
        uint64_t mask = __ballot(rel);
        while (mask) {
            const int k = 63 - __builtin_clzll(mask);
            mask &= ~(1ull << k);
            const int entry = lo + k;  // upstream `contributor` for this entry
            const float4 p0 = st.rec[k][0], p1 = st.rec[k][1];
            const float2 p2 = *reinterpret_cast<const float2 *>(&st.rec[k][2]);
            const float gx_ = p0.x, gy_ = p0.y, cx = p0.z, cy = p0.w;
            const float cz = p1.x, op = p1.y;
            const float dx = gx_ - fx, dy = gy_ - fy;
            const float power = -0.5f * (cx * dx * dx + cz * dy * dy) - cy * dx * dy;
            const float G = __expf(power);
            const float alpha = fminf(0.99f, op * G);
            const bool valid = entry < last_contrib && !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            if (!__any(valid)) continue;
            const float cr = p1.z, cg = p1.w, cb = p2.x;
            const uint32_t gid = __float_as_uint(p2.y);
            // Branch-free replay step: a skipped pixel sees alpha = 0 (T and the
            // running colour R unchanged) and zero gradients.  R is upstream's
            // accum_rec advanced eagerly: after a blended Gaussian it already holds
            // last_alpha * last_color + (1 - last_alpha) * accum_rec.
            const float av = valid ? alpha : 0.0f;
            const float Gv = valid ? G : 0.0f;
            const float om = 1.f - av;
            const float inv_1ma = __builtin_amdgcn_rcpf(om);
            T = T * inv_1ma;
            const float dchannel_dcolor = av * T;
            const float e0 = cr - R0, e1 = cg - R1, e2 = cb - R2;
            const float dot = e0 * dpx0 + e1 * dpx1 + e2 * dpx2;
            R0 = av * cr + om * R0;
            R1 = av * cg + om * R1;
            R2 = av * cb + om * R2;
            const float dL_dalpha = valid ? dot * T + (-T_final * inv_1ma) * bg_dot : 0.0f;
            const float g6 = dchannel_dcolor * dpx0;
            const float g7 = dchannel_dcolor * dpx1;
            const float g8 = dchannel_dcolor * dpx2;
            const float dL_dG = op * dL_dalpha;
            const float gdx = Gv * dx, gdy = Gv * dy;
            const float dG_ddelx = -gdx * cx - gdy * cy;
            const float dG_ddely = -gdy * cz - gdx * cy;
            const float g0 = dL_dG * dG_ddelx * ddelx_dx;
            const float g1 = dL_dG * dG_ddely * ddely_dy;
            const float hG = -0.5f * dL_dG;
            const float g2 = gdx * dx * hG;
            const float g3 = gdx * dy * hG;
            const float g4 = gdy * dy * hG;
            const float g5 = Gv * dL_dalpha;
            // reduce-scatter of the nine sums over 64 lanes (convergent: all lanes active)
            const float h0 = swap32_sum(g0, g1);  // lanes 0-31: g0, 32-63: g1
            const float h1 = swap32_sum(g2, g3);
            const float h2 = swap32_sum(g4, g5);
            const float h3 = swap32_sum(g6, g7);
            const float h4 = swap32_sum(g8, 0.f);
            const float k0 = row_sum_to_lane15(swap16_sum(h0, h1));   // lanes 15/31/47/63: g0 g2 g1 g3
            const float k1 = row_sum_to_lane15(swap16_sum(h2, h3));   //                    g4 g6 g5 g7
            const float k2 = row_sum_to_lane15(swap16_sum(h4, 0.f));  //                    g8
            // three atomic wave-instructions straight from the lanes holding the sums
            // (uniform row base in SGPRs, per-lane slot offset), no gather into lanes 0-8
            float *row = a.accum + (size_t)gid * ACCUM_STRIDE;
            if (row_last) {
                atomicAdd(row + slot, k0);
                atomicAdd(row + slot + 4, k1);
                if (lane == 15) atomicAdd(row + slot + 8, k2);  // slot = 0 here; a lane-dependent
                // address keeps the compiler's atomic optimizer (a wave-scan loop) out
            }
        }
    };
    // Double-buffered backwards stream, unrolled by two so the buffers swap roles
    // instead of being copied (see render_fwd.hip).  Indices are clamped so every
    // load is unconditional; the one wait per chunk also drains the previous
    // chunk's accumulator atomics, none are waited for inside the Gaussian loop.
    const float4 *sp = a.splats + 3 * (size_t)list[max(end - 64 + lane, 0)];
    float4 A0 = sp[0], B0 = sp[1], C0 = sp[2], A1, B1, C1;
    uint32_t idx_a, idx_b = list[max(end - 128 + lane, 0)];
    for (int lo = end - 64;;) {
        idx_a = list[max(lo - 128 + lane, 0)];
        sp = a.splats + 3 * (size_t)idx_b;
        A1 = sp[0];
        B1 = sp[1];
        C1 = sp[2];
        wait_vmcnt_4();
        replay_chunk(lo, A0, B0, C0);
        if ((lo -= 64) + 64 <= 0) break;
        idx_b = list[max(lo - 128 + lane, 0)];
        sp = a.splats + 3 * (size_t)idx_a;
        A0 = sp[0];
        B0 = sp[1];
        C0 = sp[2];
        wait_vmcnt_4();
        replay_chunk(lo, A1, B1, C1);
        if ((lo -= 64) + 64 <= 0) break;
    }
}

hipError_t launch_render_bwd(const gsr_inputs &in, const void *geom, const void *binning, int64_t I,
                             const void *img, const float *dL_dpix, float *accum, hipStream_t s) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    const ImgLayout Im = img_layout(in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    RenderBwdArgs a;
    a.W = in.W;
    a.H = in.H;
    a.gx = g.gx;
    a.tiles = g.tiles;
    a.ranges = at<uint2>(geom, G.off[GSR_GEOM_RANGES]);
    a.point_list = at<uint32_t>(binning, binning_layout(I, in.W, in.H).off[GSR_BIN_POINT_LIST]);
    a.splats = at<float4>(geom, G.off[GSR_GEOM_SPLATS]);
    a.bg = in.bg;
    a.final_T = at<float>(img, Im.off[GSR_IMG_FINAL_T]);
    a.n_contrib = at<uint32_t>(img, Im.off[GSR_IMG_N_CONTRIB]);
    a.dL_dpix = dL_dpix;
    a.accum = accum;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(xcd_grid(g.tiles)), dim3(BLEND_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr

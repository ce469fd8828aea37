// render_bwd.hip — back-to-front replay of the tile compositing (backward).
//
// Replaces upstream BACKWARD::renderCUDA (backward.cu; SURVEY.md §8a row a15,
// Appendix A.7).  Per pixel the recurrence is upstream's: start from final_T,
// walk the tile list from the back, skip entries at or beyond the pixel's
// n_contrib, recompute alpha, divide T by (1 - alpha), keep accum_rec /
// last_alpha / last_color, and produce 9 partial gradients per (pixel, Gaussian).
//
// CDNA4 mapping:
//  * the walk starts at the tile's max n_contrib (written by the forward), not
//    at the end of the list: entries past it are skipped by every pixel anyway;
//  * 8x8 quadrant per wave + the conservative alpha box give a wave-uniform
//    skip (all pixels of the quadrant would `continue` on alpha < 1/255);
//  * upstream issues ~9 float atomics per contributing (pixel, Gaussian) pair.
//    Here the 9 partials are summed over the wave's 64 pixels with DPP row
//    reductions (no LDS), and ONE wave-instruction of 9 lanes adds the sums to
//    the Gaussian's 64-byte accumulator row: one memory-side atomic request per
//    (wave, Gaussian) instead of up to 576.
#include "gsr_kernels.hpp"
#include "gsr_wave.hpp"

namespace gsr {

constexpr int RB_THREADS = 256;
constexpr int RB_BATCH = 256;

struct RenderBwdArgs {
    int W, H, gx;
    const uint2 *ranges;
    const uint32_t *point_list;
    const float4 *splats;
    const float *bg;
    const float *final_T;
    const uint32_t *n_contrib;
    const uint32_t *tile_maxc;
    const float *dL_dpix;
    float *accum;
};

__global__ void __launch_bounds__(RB_THREADS) render_bwd_kernel(RenderBwdArgs a) {
    __shared__ float4 sA[RB_BATCH];
    __shared__ float4 sB[RB_BATCH];
    __shared__ float4 sC[RB_BATCH];
    __shared__ uint32_t sId[RB_BATCH];
    const int tile = blockIdx.x;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int qx0 = tx * TILE_X + (w & 1) * 8, qy0 = ty * TILE_Y + (w >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float fx = (float)px, fy = (float)py;
    const float qxlo = (float)qx0, qxhi = (float)(qx0 + 7), qylo = (float)qy0, qyhi = (float)(qy0 + 7);
    const uint2 r = a.ranges[tile];
    const int maxc = (int)a.tile_maxc[tile];

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
    // wave-level upper bound of the list positions any of its pixels replays
    int wave_maxc = last_contrib;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) wave_maxc = max(wave_maxc, __shfl_xor(wave_maxc, o));

    float T = T_final;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
    float last_alpha = 0.f, lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;

    for (int end = maxc; end > 0; end -= RB_BATCH) {
        const int cnt = min(RB_BATCH, end);
        const int lo = end - cnt;
        __syncthreads();
        if ((int)threadIdx.x < cnt) {
            const uint32_t id = a.point_list[r.x + lo + threadIdx.x];
            const float4 *sp = a.splats + 3 * (size_t)id;
            sA[threadIdx.x] = sp[0];
            sB[threadIdx.x] = sp[1];
            sC[threadIdx.x] = sp[2];
            sId[threadIdx.x] = id;
        }
        __syncthreads();
        const int jstart = min(cnt, wave_maxc - lo) - 1;
        for (int j = jstart; j >= 0; j--) {
            const int k = lo + j;  // upstream `contributor` for this entry
            const float4 A = sA[j];
            const float4 E = sC[j];
            if (A.x + E.y < qxlo || A.x - E.y > qxhi || A.y + E.z < qylo || A.y - E.z > qyhi) continue;
            const float4 B = sB[j];
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f, g4 = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool valid = k < last_contrib;
            const float dx = A.x - fx, dy = A.y - fy;
            const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
            valid = valid && !(power > 0.0f);
            const float G = __expf(power);
            const float alpha = fminf(0.99f, B.y * G);
            valid = valid && !(alpha < 1.0f / 255.0f);
            if (valid) {
                T = T / (1.f - alpha);
                const float dchannel_dcolor = alpha * T;
                float dL_dalpha = 0.0f;
                acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                lc0 = B.z;
                lc1 = B.w;
                lc2 = E.x;
                dL_dalpha += (B.z - acc0) * dpx0;
                dL_dalpha += (B.w - acc1) * dpx1;
                dL_dalpha += (E.x - acc2) * dpx2;
                g6 = dchannel_dcolor * dpx0;
                g7 = dchannel_dcolor * dpx1;
                g8 = dchannel_dcolor * dpx2;
                dL_dalpha *= T;
                last_alpha = alpha;
                dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                const float dL_dG = B.y * dL_dalpha;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * A.z - gdy * A.w;
                const float dG_ddely = -gdy * B.x - gdx * A.w;
                g0 = dL_dG * dG_ddelx * ddelx_dx;
                g1 = dL_dG * dG_ddely * ddely_dy;
                g2 = -0.5f * gdx * dx * dL_dG;
                g3 = -0.5f * gdx * dy * dL_dG;
                g4 = -0.5f * gdy * dy * dL_dG;
                g5 = G * dL_dalpha;
            }
#ifdef GSR_BWD_LANE_ATOMICS
            if (valid) {
                float *row = a.accum + (size_t)sId[j] * ACCUM_STRIDE;
                atomicAdd(row + 0, g0); atomicAdd(row + 1, g1); atomicAdd(row + 2, g2);
                atomicAdd(row + 3, g3); atomicAdd(row + 4, g4); atomicAdd(row + 5, g5);
                atomicAdd(row + 6, g6); atomicAdd(row + 7, g7); atomicAdd(row + 8, g8);
            }
            continue;
#endif
            if (__any(valid)) {
                // all nine reductions complete in convergent code before any lane selects
                const float s0 = wave_sum(g0), s1 = wave_sum(g1), s2 = wave_sum(g2);
                const float s3 = wave_sum(g3), s4 = wave_sum(g4), s5 = wave_sum(g5);
                const float s6 = wave_sum(g6), s7 = wave_sum(g7), s8 = wave_sum(g8);
                float v = s0;
                v = lane == 1 ? s1 : v;
                v = lane == 2 ? s2 : v;
                v = lane == 3 ? s3 : v;
                v = lane == 4 ? s4 : v;
                v = lane == 5 ? s5 : v;
                v = lane == 6 ? s6 : v;
                v = lane == 7 ? s7 : v;
                v = lane == 8 ? s8 : v;
                if (lane < ACC_NVALS) atomicAdd(a.accum + (size_t)sId[j] * ACCUM_STRIDE + lane, v);
            }
        }
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
    a.ranges = at<uint2>(geom, G.off[GSR_GEOM_RANGES]);
    a.point_list = at<uint32_t>(binning, binning_layout(I, in.W, in.H).off[GSR_BIN_POINT_LIST]);
    a.splats = at<float4>(geom, G.off[GSR_GEOM_SPLATS]);
    a.bg = in.bg;
    a.final_T = at<float>(img, Im.off[GSR_IMG_FINAL_T]);
    a.n_contrib = at<uint32_t>(img, Im.off[GSR_IMG_N_CONTRIB]);
    a.tile_maxc = at<uint32_t>(img, Im.off[GSR_IMG_TILE_MAX_CONTRIB]);
    a.dL_dpix = dL_dpix;
    a.accum = accum;
    hipLaunchKernelGGL(render_bwd_kernel, dim3(g.tiles), dim3(RB_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr

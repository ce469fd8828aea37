// render_fwd.hip — 16x16-tile front-to-back alpha compositing (forward).
//
// Replaces upstream FORWARD::renderCUDA (forward.cu; SURVEY.md §8a row a14,
// Appendix A.6).  Per pixel the semantics are upstream's: walk the tile's
// depth-sorted list, skip power > 0 and alpha < 1/255, stop when T would drop
// below 1e-4 (that Gaussian is not blended), record n_contrib = list position
// of the last blended Gaussian and final_T.
//
// CDNA4 mapping: one 256-thread workgroup (4 wave64) per tile; wave w owns an
// 8x8 pixel quadrant so that a Gaussian's alpha>=1/255 box (precomputed by
// preprocess, conservative) can be tested once per wave: a wave-uniform skip
// of a Gaussian whose box misses the quadrant changes no pixel, because every
// pixel of the quadrant would reject it with alpha < 1/255.  Splat records
// (48 B, gathered through point_list) are staged 256 at a time in LDS; the
// workgroup stops staging once every pixel is saturated, and each wave stops
// iterating once its own 64 pixels are.
#include "gsr_kernels.hpp"
#include "gsr_wave.hpp"

namespace gsr {

constexpr int RF_THREADS = 256;
constexpr int RF_BATCH = 256;

struct RenderFwdArgs {
    int W, H, gx;
    const uint2 *ranges;
    const uint32_t *point_list;
    const float4 *splats;
    const float *bg;
    float *out_color;
    float *final_T;
    uint32_t *n_contrib;
    uint32_t *tile_maxc;
};

__global__ void __launch_bounds__(RF_THREADS) render_fwd_kernel(RenderFwdArgs a) {
    __shared__ float4 sA[RF_BATCH];  // x, y, conic.x, conic.y
    __shared__ float4 sB[RF_BATCH];  // conic.z, opacity, r, g
    __shared__ float4 sC[RF_BATCH];  // b, ext_x, ext_y, -
    __shared__ uint32_t smax;
    const int tile = blockIdx.x;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int qx0 = tx * TILE_X + (w & 1) * 8, qy0 = ty * TILE_Y + (w >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float fx = (float)px, fy = (float)py;
    const float qxlo = (float)qx0, qxhi = (float)(qx0 + 7), qylo = (float)qy0, qyhi = (float)(qy0 + 7);
    const uint2 r = a.ranges[tile];
    const int n = (int)(r.y - r.x);
    if (threadIdx.x == 0) smax = 0;

    float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f;
    uint32_t last = 0;
    bool done = !inside;
    for (int base = 0; base < n; base += RF_BATCH) {
        if (__syncthreads_count(done) == RF_THREADS) break;
        const int k = base + (int)threadIdx.x;
        if (k < n) {
            const uint32_t id = a.point_list[r.x + k];
            const float4 *sp = a.splats + 3 * (size_t)id;
            sA[threadIdx.x] = sp[0];
            sB[threadIdx.x] = sp[1];
            sC[threadIdx.x] = sp[2];
        }
        __syncthreads();
        const int cnt = min(RF_BATCH, n - base);
        for (int j = 0; j < cnt; j++) {
            if (!__any(!done)) break;
            const float4 A = sA[j];
            const float4 E = sC[j];
            if (A.x + E.y < qxlo || A.x - E.y > qxhi || A.y + E.z < qylo || A.y - E.z > qyhi) continue;
            if (done) continue;
            const float4 B = sB[j];
            const float dx = A.x - fx, dy = A.y - fy;
            const float power = -0.5f * (A.z * dx * dx + B.x * dy * dy) - A.w * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, B.y * __expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1 - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            C0 += B.z * alpha * T;
            C1 += B.w * alpha * T;
            C2 += E.x * alpha * T;
            T = test_T;
            last = (uint32_t)(base + j + 1);
        }
    }
    if (inside) {
        const size_t pix = (size_t)a.W * py + px;
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[HW + pix] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix] = C2 + T * a.bg[2];
    }
    atomicMax(&smax, last);
    __syncthreads();
    if (threadIdx.x == 0) a.tile_maxc[tile] = smax;
}

hipError_t launch_render_fwd(const gsr_inputs &in, const void *geom, const void *binning, int64_t I, void *img,
                             float *out_color, hipStream_t s) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    const ImgLayout Im = img_layout(in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    RenderFwdArgs a;
    a.W = in.W;
    a.H = in.H;
    a.gx = g.gx;
    a.ranges = at<uint2>(geom, G.off[GSR_GEOM_RANGES]);
    a.point_list = binning ? at<uint32_t>(binning, binning_layout(I, in.W, in.H).off[GSR_BIN_POINT_LIST]) : nullptr;
    a.splats = at<float4>(geom, G.off[GSR_GEOM_SPLATS]);
    a.bg = in.bg;
    a.out_color = out_color;
    a.final_T = at<float>(img, Im.off[GSR_IMG_FINAL_T]);
    a.n_contrib = at<uint32_t>(img, Im.off[GSR_IMG_N_CONTRIB]);
    a.tile_maxc = at<uint32_t>(img, Im.off[GSR_IMG_TILE_MAX_CONTRIB]);
    hipLaunchKernelGGL(render_fwd_kernel, dim3(g.tiles), dim3(RF_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace gsr

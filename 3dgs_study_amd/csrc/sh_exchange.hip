// sh_exchange.hip — dL/dSH summed over views from the views' colour gradients.
//
// View-parallel training (3dgs_study_amd/multiview.py) needs
// every rank to hold sum_v dL_v/dsh.  Per view, upstream's SH backward
// (backward.cu computeColorFromSH) makes that gradient the outer product
//     dL_v/dsh[k][c] = basis_k(dir_v) * dRGB_v[c],   dir_v = normalize(mean - campos_v)
// with dRGB_v the clamp-masked colour gradient (zero for culled Gaussians).
// So instead of all-reducing 12·M bytes per Gaussian (192 B at SH3: 76 % of
// the gradient), the ranks all-gather the 12-byte dRGB_v of their views plus
// each view's camera centre, and this kernel rebuilds the sum locally — the
// same products as preprocess_bwd (shared sh_basis, fp contraction off), added
// in view order, so every rank computes bit-identical gradients.
//
// records: nviews rows of view_stride floats:
//   [campos.x, campos.y, campos.z, (float)sh_degree, dRGB [P][3], padding]
// Outputs are the two leaf gradients of GaussianModel's SH storage
// (scene/gaussian_model.py:106-110): dsh_dc [P,1,3] and dsh_rest [P,M-1,3].
#pragma clang fp contract(off)

#include "gsr_kernels.hpp"
#include "gsr_math.hpp"
#include "gsr_rows.hpp"

namespace gsr {

constexpr int SX_THREADS = 128;

// One thread per Gaussian; 3·M sums in registers; the f_rest rows leave through
// LDS (coalesced 16-B stores) like the SH rows of preprocess_bwd.
template <int MC>
__global__ void __launch_bounds__(SX_THREADS) sh_from_colors_kernel(int P, int nviews, int64_t stride,
                                                                     const float *__restrict__ means3D,
                                                                     const float *__restrict__ rec,
                                                                     float *__restrict__ dsh_dc,
                                                                     float *__restrict__ dsh_rest) {
    constexpr int RW = 3 * (MC - 1);  // f_rest row width
    __shared__ __attribute__((aligned(16))) float lds[RW > 0 ? SX_THREADS * (RW + 1) : 1];
    const int g0 = blockIdx.x * SX_THREADS;
    const int n = min(SX_THREADS, P - g0);
    const int idx = g0 + (int)threadIdx.x;
    const bool live = idx < P;
    const int li = live ? idx : P - 1;
    const float mx = means3D[3 * (size_t)li], my = means3D[3 * (size_t)li + 1], mz = means3D[3 * (size_t)li + 2];
    float acc[3 * MC];
#pragma unroll
    for (int k = 0; k < 3 * MC; k++) acc[k] = 0.f;
    // Views in groups of VB: the group's colour rows are loaded before any of its
    // products, so the loads of VB views are in flight together (one view at a
    // time left the kernel waiting on each view's load: 97 us for 8 views at
    // 1M Gaussians, vs 34 us for one; groups of 4: 83 us, of 8: 79 us).  Sums
    // stay in view order.
    constexpr int VB = 8;
    for (int v0 = 0; v0 < nviews; v0 += VB) {
        float dv[VB][3];
#pragma unroll
        for (int j = 0; j < VB; j++) {
            const int v = min(v0 + j, nviews - 1);
            const float *d3 = rec + (size_t)v * (size_t)stride + 4 + 3 * (size_t)li;
#pragma unroll
            for (int c = 0; c < 3; c++) dv[j][c] = d3[c];
        }
#pragma unroll
        for (int j = 0; j < VB; j++) {
            if (v0 + j >= nviews) break;
            const float *r = rec + (size_t)(v0 + j) * (size_t)stride;
            const float *d = dv[j];
            // a zero colour gradient (culled or clamped in this view) adds exactly
            // nothing: skipped, so a mean at the view's camera centre (zero-length
            // direction, NaN basis) cannot poison the sum; upstream gives a culled
            // Gaussian no SH gradient at all
            if (d[0] == 0.f && d[1] == 0.f && d[2] == 0.f) continue;
            const int deg = (int)r[3];
            const float ox = mx - r[0], oy = my - r[1], oz = mz - r[2];
            const float len = sqrtf((ox * ox + oy * oy) + oz * oz);
            float b[16];
            sh_basis(deg, ox / len, oy / len, oz / len, b);
            const int ncoef = min((deg + 1) * (deg + 1), MC);
#pragma unroll
            for (int k = 0; k < MC; k++)
                if (k < ncoef) {
#pragma unroll
                    for (int c = 0; c < 3; c++) acc[3 * k + c] += b[k] * d[c];
                }
        }
    }
    if (live) {
#pragma unroll
        for (int c = 0; c < 3; c++) dsh_dc[3 * (size_t)idx + c] = acc[c];
    }
    // (per-thread dword stores of the 180-B rows instead of the LDS stage: 71 vs
    // 34 us for one view)
    if constexpr (RW > 0) {
        float *row = lds + threadIdx.x * (RW + 1);
#pragma unroll
        for (int k = 0; k < RW; k++) row[k] = acc[3 + k];
        __syncthreads();
        lds_to_rows<SX_THREADS, RW>(lds, g0, n, RW, dsh_rest);
    }
}

// The clamp-masked colour gradient of one view straight from render_bwd's
// accumulator rows (dcolor at floats 0..2: one 32-B sector), before preprocess_bwd runs, so the
// exchange can start while preprocess_bwd computes: preprocess_bwd's own masking
// (dcol * (clamped ? 0 : 1), zero for culled Gaussians), bit for bit.
__global__ void __launch_bounds__(256) colors_from_accum_kernel(int P, const int32_t *__restrict__ radii,
                                                                const uint8_t *__restrict__ clamped,
                                                                const float *__restrict__ accum,
                                                                float *__restrict__ drgb) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const bool vis = radii[i] > 0;
    const uint32_t cl = clamped[i];
    // one 16-B load of the row's head (the colour sums, floats 0..2)
    const float4 row = *reinterpret_cast<const float4 *>(accum + (size_t)i * ACCUM_STRIDE);
    const float c[3] = {row.x, row.y, row.z};
#pragma unroll
    for (int k = 0; k < 3; k++) drgb[3 * (size_t)i + k] = vis ? c[k] * ((cl >> k) & 1u ? 0.f : 1.f) : 0.f;
}

hipError_t launch_colors_from_accum(int P, const int32_t *radii, const uint8_t *clamped, const float *accum,
                                    float *drgb, hipStream_t s) {
    hipLaunchKernelGGL(colors_from_accum_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, clamped, accum,
                       drgb);
    return hipGetLastError();
}

hipError_t launch_sh_grad_from_colors(int P, int M, int nviews, int64_t view_stride, const float *means3D,
                                      const float *records, float *dsh_dc, float *dsh_rest, hipStream_t s) {
    const dim3 grid((P + SX_THREADS - 1) / SX_THREADS);
    switch (M) {
        case 16:
            hipLaunchKernelGGL(sh_from_colors_kernel<16>, grid, dim3(SX_THREADS), 0, s, P, nviews, view_stride,
                               means3D, records, dsh_dc, dsh_rest);
            break;
        case 9:
            hipLaunchKernelGGL(sh_from_colors_kernel<9>, grid, dim3(SX_THREADS), 0, s, P, nviews, view_stride,
                               means3D, records, dsh_dc, dsh_rest);
            break;
        case 4:
            hipLaunchKernelGGL(sh_from_colors_kernel<4>, grid, dim3(SX_THREADS), 0, s, P, nviews, view_stride,
                               means3D, records, dsh_dc, dsh_rest);
            break;
        case 1:
            hipLaunchKernelGGL(sh_from_colors_kernel<1>, grid, dim3(SX_THREADS), 0, s, P, nviews, view_stride,
                               means3D, records, dsh_dc, dsh_rest);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gsr

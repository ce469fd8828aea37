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

// One view (the forced one-rank exchange, and any rank group whose records hold a
// single view): the sum is one outer product basis (x) dRGB per Gaussian, so the
// workgroup stages the 15 basis values and the 3 colour gradients (18 floats, not
// the 45 products) and forms each product as it writes the f_rest rows — 2.5x less
// LDS and no 48 accumulators, so more workgroups in flight.  Bit for bit the
// general kernel's result: its sum over one view is 0 + b * d (the 0 + turns a -0
// product into +0, so it is kept), a skipped view (zero dRGB) leaves +0, and a
// coefficient above the view's degree stays exactly 0 whatever d holds.
constexpr int SX1_THREADS = 256, SX1_S = 19;  // LDS stride: 15 basis + 3 colour, odd
template <int MC>
__global__ void __launch_bounds__(SX1_THREADS) sh_from_colors_one_kernel(int P, const float *__restrict__ means3D,
                                                                         const float *__restrict__ rec,
                                                                         float *__restrict__ dsh_dc,
                                                                         float *__restrict__ dsh_rest) {
    static_assert(MC == 16, "the write-out divides by the degree-3 row width, 45");
    constexpr int RW = 3 * (MC - 1);
    __shared__ float lds[SX1_THREADS * SX1_S];
    const int g0 = blockIdx.x * SX1_THREADS;
    const int n = min(SX1_THREADS, P - g0);
    const int idx = g0 + (int)threadIdx.x;
    if (idx < P) {
        const float d[3] = {rec[4 + 3 * (size_t)idx], rec[4 + 3 * (size_t)idx + 1], rec[4 + 3 * (size_t)idx + 2]};
        const bool zero = d[0] == 0.f && d[1] == 0.f && d[2] == 0.f;
        float b[16];
#pragma unroll
        for (int k = 0; k < 16; k++) b[k] = 0.f;
        const int deg = (int)rec[3];
        if (!zero) {
            const float ox = means3D[3 * (size_t)idx] - rec[0], oy = means3D[3 * (size_t)idx + 1] - rec[1],
                        oz = means3D[3 * (size_t)idx + 2] - rec[2];
            const float len = sqrtf((ox * ox + oy * oy) + oz * oz);
            sh_basis(deg, ox / len, oy / len, oz / len, b);
        }
#pragma unroll
        for (int c = 0; c < 3; c++) dsh_dc[3 * (size_t)idx + c] = 0.f + b[0] * d[c];
        float *row = lds + threadIdx.x * SX1_S;
#pragma unroll
        for (int k = 1; k < MC; k++) row[k - 1] = b[k];
#pragma unroll
        for (int c = 0; c < 3; c++) row[15 + c] = d[c];
    }
    if constexpr (RW > 0) {
        const int deg = (int)rec[3];  // one record: the degree is uniform
        const int nk = min((deg + 1) * (deg + 1), MC) - 1;  // live f_rest coefficients
        __syncthreads();
        // the workgroup's f_rest rows [g0, g0 + n) as float4s (the rows of 256
        // Gaussians are 16-B aligned: 45 x 4 x 256 B), each element b[k] * d[c]
        float4 *out4 = reinterpret_cast<float4 *>(dsh_rest + (size_t)g0 * RW);
        const int n4 = n * RW / 4;
        auto elem = [&](int e) {
            const int g = (int)(((uint32_t)e * 11651u) >> 19);  // e / 45 for e < 11520 (256 rows)
            const int j = e - g * RW;
            const int k = (int)(((uint32_t)j * 43u) >> 7);       // j / 3 for j < 45
            const float *row = lds + g * SX1_S;
            return k < nk ? 0.f + row[k] * row[15 + (j - 3 * k)] : 0.f;
        };
        for (int i = threadIdx.x; i < n4; i += SX1_THREADS)
            out4[i] = make_float4(elem(4 * i), elem(4 * i + 1), elem(4 * i + 2), elem(4 * i + 3));
        for (int e = (n4 << 2) + threadIdx.x; e < n * RW; e += SX1_THREADS) dsh_rest[(size_t)g0 * RW + e] = elem(e);
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
    float c[3] = {0.f, 0.f, 0.f};
    if (vis) {  // a culled Gaussian's row and clamp bits are not read (its colour gradient is 0)
        const uint32_t cl = clamped[i];
        // one 16-B load of the row's head (the colour sums, floats 0..2)
        const float4 row = *reinterpret_cast<const float4 *>(accum + (size_t)i * ACCUM_STRIDE);
        const float r[3] = {row.x, row.y, row.z};
#pragma unroll
        for (int k = 0; k < 3; k++) c[k] = r[k] * ((cl >> k) & 1u ? 0.f : 1.f);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) drgb[3 * (size_t)i + k] = c[k];
}

hipError_t launch_colors_from_accum(int P, const int32_t *radii, const uint8_t *clamped, const float *accum,
                                    float *drgb, hipStream_t s) {
    hipLaunchKernelGGL(colors_from_accum_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, clamped, accum,
                       drgb);
    return hipGetLastError();
}

hipError_t launch_sh_grad_from_colors(int P, int M, int nviews, int64_t view_stride, const float *means3D,
                                      const float *records, float *dsh_dc, float *dsh_rest, hipStream_t s) {
    if (nviews == 1 && M == 16) {  // the one-view form (the degree-3 storage)
        hipLaunchKernelGGL(sh_from_colors_one_kernel<16>, dim3((P + SX1_THREADS - 1) / SX1_THREADS), dim3(SX1_THREADS),
                           0, s, P, means3D, records, dsh_dc, dsh_rest);
        return hipGetLastError();
    }
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

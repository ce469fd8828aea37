// gsr_rows.hpp — coalesced staging of per-Gaussian rows through LDS.
//
// The SH block of a Gaussian is a 12·M-byte row (192 B at SH degree 3).  The
// preprocess kernels load a degree-3 row per thread straight into registers
// (12 x 16 B; preprocess.hip).  For the other widths, and for the SH rebuild of
// the view exchange (sh_exchange.hip, 180-B rows whose per-thread stores were
// 2x slower), the workgroup streams its contiguous slice of rows with
// 16-byte-per-lane accesses through LDS rows padded to an odd number of dwords
// (bank-conflict-free per-lane row access).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

// row r, column c of a [rows][RW] block -> padded LDS index.  RWC > 0: the row
// width is a compile-time constant and the division is a multiply-shift (the
// SH row of degree 3 is 48 floats); RWC = 0: run-time width, float reciprocal
// with exact integer fix-ups.
template <int RWC>
__device__ __forceinline__ int lds_row_index(int e, int RW, float invRW) {
    if constexpr (RWC > 0) {
        const int r = (int)((uint32_t)e / (uint32_t)RWC);
        return r * (RWC + 1) + (e - r * RWC);
    } else {
        int r = (int)((float)e * invRW);
        r += ((r + 1) * RW <= e) ? 1 : 0;
        r -= (r * RW > e) ? 1 : 0;
        return r * (RW + 1) + (e - r * RW);
    }
}

// Copy rows [g0, g0 + n) of a row-major float [*, RW] array into LDS rows of
// stride RW + 1.  All threads of the workgroup must call it.
template <int THREADS, int RWC = 0>
__device__ inline void rows_to_lds(const float *__restrict__ src, int g0, int n, int RW_, float *lds) {
    const int RW = RWC > 0 ? RWC : RW_;
    const int total = n * RW;
    const float invRW = 1.0f / (float)RW;
    const float *base = src + (size_t)g0 * RW;
    if ((((uintptr_t)base) & 15u) == 0) {
        const float4 *b4 = reinterpret_cast<const float4 *>(base);
        const int n4 = total >> 2;
        // batches of BATCH loads in flight per lane before the first LDS store
        // (a load-store-load loop would expose the full HBM latency per float4)
        constexpr int BATCH = 12;
        for (int i0 = threadIdx.x; i0 < n4; i0 += THREADS * BATCH) {
            float4 v[BATCH];
#pragma unroll
            for (int b = 0; b < BATCH; b++) {
                const int i = i0 + b * THREADS;
                if (i < n4) v[b] = b4[i];
            }
#pragma unroll
            for (int b = 0; b < BATCH; b++) {
                const int i = i0 + b * THREADS;
                if (i < n4) {
                    const int e = i << 2;
                    lds[lds_row_index<RWC>(e, RW, invRW)] = v[b].x;
                    lds[lds_row_index<RWC>(e + 1, RW, invRW)] = v[b].y;
                    lds[lds_row_index<RWC>(e + 2, RW, invRW)] = v[b].z;
                    lds[lds_row_index<RWC>(e + 3, RW, invRW)] = v[b].w;
                }
            }
        }
        for (int e = (n4 << 2) + threadIdx.x; e < total; e += THREADS) lds[lds_row_index<RWC>(e, RW, invRW)] = base[e];
    } else {
        for (int e = threadIdx.x; e < total; e += THREADS) lds[lds_row_index<RWC>(e, RW, invRW)] = base[e];
    }
}

// Rows [g0, g0 + n) of a row-major float [*, w] array into columns [c0, c0 + w) of
// LDS rows of stride S: the SH storage's two leaves (_features_dc, w = 3, and
// _features_rest, w = 3M - 3; gsr_inputs.sh_rest) staged side by side as one padded
// row per Gaussian.  All threads of the workgroup must call it.
template <int THREADS>
__device__ inline void rows_to_lds_cols(const float *__restrict__ src, int g0, int n, int w, int c0, int S,
                                        float *lds) {
    const int total = n * w;
    const float invw = 1.0f / (float)w;
    const float *base = src + (size_t)g0 * w;
    for (int e = threadIdx.x; e < total; e += THREADS) {
        int r = (int)((float)e * invw);
        r += ((r + 1) * w <= e) ? 1 : 0;
        r -= (r * w > e) ? 1 : 0;
        lds[r * S + c0 + (e - r * w)] = base[e];
    }
}

// One Gaussian's degree-3 SH row (48 floats) from the split storage: 3 floats of
// _features_dc and 45 of _features_rest (180-B rows, 4-byte aligned: the loads are
// the compiler's to merge).
__device__ __forceinline__ void load_sh_row_split(const float *__restrict__ dc, const float *__restrict__ rest,
                                                  size_t li, float r[48]) {
#pragma unroll
    for (int k = 0; k < 3; k++) r[k] = dc[3 * li + k];
#pragma unroll
    for (int k = 0; k < 45; k++) r[3 + k] = rest[45 * li + k];
}

// The reverse: LDS rows (stride RW + 1) -> global rows [g0, g0 + n).
template <int THREADS, int RWC = 0>
__device__ inline void lds_to_rows(const float *lds, int g0, int n, int RW_, float *__restrict__ dst) {
    const int RW = RWC > 0 ? RWC : RW_;
    const int total = n * RW;
    const float invRW = 1.0f / (float)RW;
    float *base = dst + (size_t)g0 * RW;
    if ((((uintptr_t)base) & 15u) == 0) {
        float4 *b4 = reinterpret_cast<float4 *>(base);
        const int n4 = total >> 2;
        for (int i = threadIdx.x; i < n4; i += THREADS) {
            const int e = i << 2;
            float4 v;
            v.x = lds[lds_row_index<RWC>(e, RW, invRW)];
            v.y = lds[lds_row_index<RWC>(e + 1, RW, invRW)];
            v.z = lds[lds_row_index<RWC>(e + 2, RW, invRW)];
            v.w = lds[lds_row_index<RWC>(e + 3, RW, invRW)];
            b4[i] = v;
        }
        for (int e = (n4 << 2) + threadIdx.x; e < total; e += THREADS) base[e] = lds[lds_row_index<RWC>(e, RW, invRW)];
    } else {
        for (int e = threadIdx.x; e < total; e += THREADS) base[e] = lds[lds_row_index<RWC>(e, RW, invRW)];
    }
}


// Columns [c0, c0 + w) of LDS rows (stride S) -> global rows [g0, g0 + n) of width
// w, overwritten or (add) added to what is there (AccumulateGrad's grad += new):
// the SH cat's two leaves, dsh_dc (w = 3) and dsh_rest (w = 3M - 3).
template <int THREADS>
__device__ inline void lds_cols_to_rows(const float *lds, int S, int c0, int w, int g0, int n,
                                        float *__restrict__ dst, bool add) {
    const int total = n * w;
    const float invw = 1.0f / (float)w;
    float *base = dst + (size_t)g0 * w;
    for (int e = threadIdx.x; e < total; e += THREADS) {
        int r = (int)((float)e * invw);
        r += ((r + 1) * w <= e) ? 1 : 0;
        r -= (r * w > e) ? 1 : 0;
        const float v = lds[r * S + c0 + (e - r * w)];
        base[e] = add ? base[e] + v : v;
    }
}

// The reverse into M coefficient planes: LDS rows (stride RW + 1, RW = 3M) of
// Gaussians [g0, g0 + n) -> plane k = dst + k * plane_stride, floats
// [3 g0, 3 (g0 + n)) of each, i.e. dL/dsh laid out [M][P][3] (the tensor
// [P,M,3] with strides (3, 3P, 1); diff_gaussian_rasterization hands that view
// to autograd so the SH cat backward's f_dc slice needs no copy).  16-B stores
// when the planes are 16-B aligned.
template <int THREADS>
__device__ inline void lds_to_planes(const float *lds, int g0, int n, int M, size_t plane_stride,
                                     float *__restrict__ dst) {
    const int RW1 = 3 * M + 1;
    const int cnt = 3 * n;
    const bool vec = (plane_stride & 3) == 0 && ((uintptr_t)dst & 15u) == 0;  // 3 g0 is a multiple of 4
    auto at_e = [&](int e, int k) {
        const int g = (int)(((uint32_t)e * 43691u) >> 17);  // e / 3 for e < 98304
        return lds[g * RW1 + 3 * k + (e - 3 * g)];
    };
    for (int k = 0; k < M; k++) {
        float *base = dst + (size_t)k * plane_stride + (size_t)g0 * 3;
        int e0 = 0;
        if (vec) {
            const int n4 = cnt >> 2;
            for (int i = threadIdx.x; i < n4; i += THREADS) {
                const int e = i << 2;
                reinterpret_cast<float4 *>(base)[i] = make_float4(at_e(e, k), at_e(e + 1, k), at_e(e + 2, k), at_e(e + 3, k));
            }
            e0 = n4 << 2;
        }
        for (int e = e0 + threadIdx.x; e < cnt; e += THREADS) base[e] = at_e(e, k);
    }
}

}  // namespace gsr

// gsr_l1.hpp — the L1 loss mean|x - y|'s per-workgroup partial sums, shared by
// train_ops.hip's l1_kernel (the loss on its own) and render_bwd.hip's
// bwd_prepare_kernel (the loss computed in the same launch as the backward's
// quadrant filing, gsr_forward_render_l1): one block decomposition, so both give
// the same partials and, through l1_ssim_finish_kernel, the same loss bits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace gsr {

constexpr int L1_THREADS = 256, L1_BLOCKS = 1024;

__host__ __device__ inline int l1_blocks(size_t n) {
    const size_t want = (n / 4 + L1_THREADS - 1) / L1_THREADS;
    return (int)(want < (size_t)L1_BLOCKS ? (want > 0 ? want : 1) : L1_BLOCKS);
}

// Block blk of nblk (L1_THREADS threads): sum |x - y| over its grid-stride share
// (16-B loads; block 0 also takes the tail of a length that is not a multiple of 4)
// into partials[2 blk] (and 0 into partials[2 blk + 1], the SSIM slot).
__device__ __forceinline__ void l1_block_partial(const float *x, const float *y, size_t n, int blk, int nblk,
                                                 float *partials) {
    __shared__ float wsum[L1_THREADS / 64];
    const size_t n4 = n >> 2, stride = (size_t)nblk * L1_THREADS;
    const float4 *x4 = reinterpret_cast<const float4 *>(x), *y4 = reinterpret_cast<const float4 *>(y);
    float acc = 0.f;
    for (size_t i = (size_t)blk * L1_THREADS + threadIdx.x; i < n4; i += stride) {
        const float4 a = x4[i], b = y4[i];
        acc += (fabsf(a.x - b.x) + fabsf(a.y - b.y)) + (fabsf(a.z - b.z) + fabsf(a.w - b.w));
    }
    if (blk == 0)
        for (size_t i = (n4 << 2) + threadIdx.x; i < n; i += L1_THREADS) acc += fabsf(x[i] - y[i]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float tot = 0.f;
#pragma unroll
        for (int k = 0; k < L1_THREADS / 64; k++) tot += wsum[k];
        partials[2 * blk] = tot;
        partials[2 * blk + 1] = 0.f;
    }
}

}  // namespace gsr

// gsr_l1.hpp — the L1 loss mean|x - y|'s per-workgroup partial sums, shared by
// train_ops.hip's l1_kernel (the loss on its own) and render_bwd.hip's
// bwd_prepare_kernel (the loss computed in the same launch as the backward's
// quadrant filing, gsr_forward_render_l1): one block decomposition, so both give
// the same partials and, through l1_ssim_finish_kernel, the same loss bits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace gsr {

#ifndef GSR_L1_BLOCKS
#define GSR_L1_BLOCKS 1024  // at most 1024: the finish emulates a 1024-thread reduction
#endif
constexpr int L1_THREADS = 256, L1_BLOCKS = GSR_L1_BLOCKS;
static_assert(L1_BLOCKS <= 1024, "the finish reads at most 1024 partials");
typedef float l1_v4f __attribute__((ext_vector_type(4)));

__host__ __device__ inline int l1_blocks(size_t n) {
    const size_t want = (n / 4 + L1_THREADS - 1) / L1_THREADS;
    return (int)(want < (size_t)L1_BLOCKS ? (want > 0 ? want : 1) : L1_BLOCKS);
}

// Block blk of nblk (L1_THREADS threads): sum |x - y| over its grid-stride share
// (16-B loads; block 0 also takes the tail of a length that is not a multiple of 4)
// into partials[2 blk] (and 0 into partials[2 blk + 1], the SSIM slot).
// write_through: the two words leave as agent-scope (sc1) stores, for a consumer in
// the same launch (l1_finish_last_block).
__device__ __forceinline__ float l1_sign_of(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }  // torch.sign
// sign (or NULL): sign(x - y) per element as an int8 (the L1 loss's pixel gradient
// up to its scale, for the seeded backward: 1 B instead of the 8 B of both inputs)
__device__ __forceinline__ void l1_block_partial(const float *x, const float *y, size_t n, int blk, int nblk,
                                                 float *partials, bool write_through = false,
                                                 int8_t *sign = nullptr) {
    __shared__ float wsum[L1_THREADS / 64];
    const size_t n4 = n >> 2, stride = (size_t)nblk * L1_THREADS;
    const float4 *x4 = reinterpret_cast<const float4 *>(x), *y4 = reinterpret_cast<const float4 *>(y);
    float acc = 0.f;
    for (size_t i = (size_t)blk * L1_THREADS + threadIdx.x; i < n4; i += stride) {
        // both images are read once here: non-temporal, so they do not displace what
        // the render backward is about to gather (render_bwd -1.5 to -2 us at config C)
        const l1_v4f av = __builtin_nontemporal_load(reinterpret_cast<const l1_v4f *>(x4 + i));
        const l1_v4f bv = __builtin_nontemporal_load(reinterpret_cast<const l1_v4f *>(y4 + i));
        const float4 a = make_float4(av.x, av.y, av.z, av.w), b = make_float4(bv.x, bv.y, bv.z, bv.w);
        acc += (fabsf(a.x - b.x) + fabsf(a.y - b.y)) + (fabsf(a.z - b.z) + fabsf(a.w - b.w));
        if (sign) {
            const uint32_t s = (uint32_t)(uint8_t)(int8_t)l1_sign_of(a.x - b.x) |
                               (uint32_t)(uint8_t)(int8_t)l1_sign_of(a.y - b.y) << 8 |
                               (uint32_t)(uint8_t)(int8_t)l1_sign_of(a.z - b.z) << 16 |
                               (uint32_t)(uint8_t)(int8_t)l1_sign_of(a.w - b.w) << 24;
            reinterpret_cast<uint32_t *>(sign)[i] = s;
        }
    }
    if (blk == 0)
        for (size_t i = (n4 << 2) + threadIdx.x; i < n; i += L1_THREADS) {
            acc += fabsf(x[i] - y[i]);
            if (sign) sign[i] = (int8_t)l1_sign_of(x[i] - y[i]);
        }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float tot = 0.f;
#pragma unroll
        for (int k = 0; k < L1_THREADS / 64; k++) tot += wsum[k];
        if (write_through) {
            __hip_atomic_store(&partials[2 * blk], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&partials[2 * blk + 1], 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            partials[2 * blk] = tot;
            partials[2 * blk + 1] = 0.f;
        }
    }
}

// The L1 loss's finish inside the partial sums' own launch: each block, after its
// write-through partials, takes a ticket (agent-scope add after its stores drained);
// the block that draws the last one reads every partial (sc1 loads: MI355X_MICROARCH
// hand-off table, row 1) and forms the loss exactly as l1_ssim_finish_kernel does
// with lambda 0 — its 1024 threads' double sums, emulated 4 per thread in the same
// order, so the same bits — saving the finish launch and its boundary.  Tickets are
// two-level: 1024 adds on one word serialise (~88 per us), so block b adds to group
// b mod 8's word and each group's last block to the top word.  The L1_TICKETS words
// are zeroed by the launch before (render_fwd_kernel).
constexpr int L1_TICKET_GROUPS = 8, L1_TICKETS = L1_TICKET_GROUPS + 1;
constexpr int L1_TICKET_STRIDE = 32;  // words: each ticket on a 128-B line of its own
__device__ __forceinline__ void l1_finish_last_block(const float *partials, int blk, int nb, uint32_t *tickets,
                                                     float invN, float *out) {
    __shared__ int last;
    __shared__ double ws[16];
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's partials have landed
        const int g = blk % L1_TICKET_GROUPS, ng = nb < L1_TICKET_GROUPS ? nb : L1_TICKET_GROUPS;
        const uint32_t in_group = (uint32_t)((nb - g + L1_TICKET_GROUPS - 1) / L1_TICKET_GROUPS);
        bool l = false;
        if (__hip_atomic_fetch_add(&tickets[g * L1_TICKET_STRIDE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            in_group - 1u)
            l = __hip_atomic_fetch_add(&tickets[L1_TICKET_GROUPS * L1_TICKET_STRIDE], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)ng - 1u;
        last = l;
    }
    __syncthreads();
    if (!last) return;
    // virtual thread v = threadIdx.x + 256 j of the finish kernel's 1024: partial v
    // (nb <= L1_BLOCKS = 1024), reduced per virtual wave by the same xor butterfly
    static_assert(L1_THREADS == 256, "four virtual finish threads per thread");
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int v = (int)threadIdx.x + 256 * j;
        double l1 = v < nb ? (double)__hip_atomic_load(&partials[2 * v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) l1 += __shfl_xor(l1, o);
        if ((threadIdx.x & 63) == 0) ws[4 * j + w] = l1;  // virtual wave v / 64 = 4 j + w
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0;
        for (int k = 0; k < 16; k++) a += ws[k];
        const double lambda = 0.0, b = 0.0;
        const float lam = 0.0f;
        (void)lambda;
        out[0] = (float)((1.0 - lam) * a * invN + lam * (1.0 - b * invN));
        out[1] = (float)(a * invN);
        out[2] = (float)(b * invN);
    }
}

}  // namespace gsr

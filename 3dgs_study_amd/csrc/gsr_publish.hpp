// gsr_publish.hpp — num_rendered from the preprocess workgroups' instance sums,
// published into the geom control words and the caller's pinned host words.  One
// 1024-thread workgroup: an extra workgroup of the depth sort's first digit scan
// (binning.hip), which runs right after preprocess — no launch of its own.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gsr_common.hpp"

namespace gsr {

// Which candidate key range decides the depth sort: base = the smallest key with
// its low byte cleared, three passes when every candidate lies within 2^24 of it.
__device__ __forceinline__ uint2 dsort_base_passes(uint32_t kmin, uint32_t kmax) {
    const bool any = kmin <= kmax;
    const uint32_t base = any ? (kmin & ~0xffu) : 0u;
    return make_uint2(base, any && kmax - base > 0xffffffu ? 4u : 3u);
}

constexpr int TOTAL_THREADS = 1024;
// (THREADS: the workgroup's size — 1024 in the digit scan, 256 in depth_keys_kernel
// when the first depth pass is grouped).  dctrl (or NULL): also the depth sort's
// key base and pass count, from the workgroups' candidate key ranges (sums .y =
// smallest, .z = largest depth key bits of a Gaussian in front of the near plane),
// into the sort's control words and the host's CTRL_DSORT_PASSES
template <int THREADS = TOTAL_THREADS>
__device__ __forceinline__ void publish_total(const uint4 *sums, int n, uint32_t *ctrl, uint32_t *host_ctrl,
                                              uint32_t *dctrl = nullptr) {
    __shared__ unsigned long long part[THREADS / 64];
    __shared__ uint32_t perr[THREADS / 64], pmin[THREADS / 64], pmax[THREADS / 64];
    unsigned long long t = 0;
    uint32_t e = 0, kmin = 0xffffffffu, kmax = 0u;
    // 8 loads in flight per thread (one at a time: 12 us for config E's 19.5k
    // workgroup records, on the host's critical path)
    constexpr int U = 8;
    for (int i0 = threadIdx.x; i0 < n; i0 += THREADS * U) {
        uint4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const int i = i0 + j * THREADS;
            v[j] = i < n ? sums[i] : make_uint4(0u, 0xffffffffu, 0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            t += v[j].x & 0x7fffffffu;
            e |= v[j].x >> 31;
            kmin = min(kmin, v[j].y);
            kmax = max(kmax, v[j].z);
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        t += __shfl_xor(t, o);
        e |= __shfl_xor(e, o);
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    if ((threadIdx.x & 63) == 0) {
        part[threadIdx.x >> 6] = t;
        perr[threadIdx.x >> 6] = e;
        pmin[threadIdx.x >> 6] = kmin;
        pmax[threadIdx.x >> 6] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < THREADS / 64; k++) {
            t += part[k];
            e |= perr[k];
            kmin = min(kmin, pmin[k]);
            kmax = max(kmax, pmax[k]);
        }
        const uint32_t w[3] = {(uint32_t)t, (uint32_t)(t >> 32), e};
        for (int k = 0; k < 3; k++) {
            ctrl[k] = w[k];
            __hip_atomic_store(&host_ctrl[k], w[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (dctrl) {
            const uint2 bp = dsort_base_passes(kmin, kmax);
            dctrl[DCTRL_KEY_BASE] = bp.x;
            dctrl[DCTRL_PASSES] = bp.y;
            __hip_atomic_store(&host_ctrl[CTRL_DSORT_PASSES], bp.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __threadfence_system();
    }
}

}  // namespace gsr

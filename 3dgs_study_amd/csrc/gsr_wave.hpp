// gsr_wave.hpp — wave64 / workgroup primitives for CDNA4 (gfx950).
// DPP row operations reduce across the 64 lanes without touching LDS:
// row_shr:N shifts inside 16-lane rows, row_bcast:15/31 carry row totals
// across rows (GFX9 family, available on gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

// DPP control codes (GFX9 encoding)
constexpr int DPP_QUAD_XOR1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int DPP_ROW_ROR8 = 0x128;
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_SHL1 = 0x101;
constexpr int DPP_ROW_SHL2 = 0x102;
constexpr int DPP_ROW_SHR1 = 0x111;
constexpr int DPP_ROW_SHR2 = 0x112;
constexpr int DPP_ROW_SHR3 = 0x113;
constexpr int DPP_ROW_SHR4 = 0x114;
constexpr int DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142;
constexpr int DPP_ROW_BCAST31 = 0x143;

template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ float dpp_f32(float v) {
    // lanes outside ROW_MASK/BANK_MASK, or whose source is out of the row, read 0
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK,
                                                                  BANK_MASK, true));
}
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, BANK_MASK, true);
}

// Sum over the 64 lanes; the total lands in lane 63 (all lanes must be active).
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    v += dpp_f32<DPP_ROW_SHR1>(v);
    v += dpp_f32<DPP_ROW_SHR2>(v);
    v += dpp_f32<DPP_ROW_SHR4, 0xf, 0xe>(v);
    v += dpp_f32<DPP_ROW_SHR8, 0xf, 0xc>(v);
    v += dpp_f32<DPP_ROW_BCAST15, 0xa>(v);
    v += dpp_f32<DPP_ROW_BCAST31, 0xc>(v);
    return v;
}

// Wave-uniform sum over the 64 lanes.  Call from convergent code only: the
// lane-63 read must see every lane's contribution (a readlane placed inside a
// lane-divergent branch lets the compiler sink the final DPP add into that
// branch, leaving lane 63 stale).
__device__ __forceinline__ float wave_sum(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wave_sum_to_lane63(v)), 63));
}

// Inclusive prefix sum across the wave (all lanes active).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    v += dpp_u32<DPP_ROW_SHR1>(v);
    v += dpp_u32<DPP_ROW_SHR2>(v);
    v += dpp_u32<DPP_ROW_SHR4>(v);
    v += dpp_u32<DPP_ROW_SHR8>(v);
    v += dpp_u32<DPP_ROW_BCAST15, 0xa>(v);
    v += dpp_u32<DPP_ROW_BCAST31, 0xc>(v);
    return v;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Workgroup inclusive scan (THREADS multiple of 64). `wsum` is LDS scratch of
// THREADS/64 words.  Returns the inclusive prefix; *total gets the block sum.
template <int THREADS>
__device__ __forceinline__ uint32_t block_inclusive_scan(uint32_t v, uint32_t *wsum, uint32_t *total) {
    constexpr int NW = THREADS / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t s = wave_inclusive_scan(v);
    if (lane == 63) wsum[w] = s;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        uint32_t x = wsum[i];
        pre += (i < w) ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return s + pre;
}

template <int THREADS>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *wsum) {
    uint32_t tot;
    block_inclusive_scan<THREADS>(v, wsum, &tot);
    return tot;
}

// Exclusive scan of v[0, n) in place by one workgroup; returns the total.  Per
// round each wave takes 64 * PER consecutive entries with coalesced loads (all
// in flight at once), scans them as PER wave scans chained by the running wave
// total, and one exchange of the wave totals places the waves: a block scan
// (two barriers) per THREADS entries left the 256 digit scans of the config-E
// tile sort at ~28 us each.
template <int THREADS, int PER>
__device__ __forceinline__ uint32_t block_exclusive_scan_inplace(uint32_t *v, int n, uint32_t *wsum) {
    constexpr int NW = THREADS / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += THREADS * PER) {
        const int wb = base + w * 64 * PER + lane;
        uint32_t x[PER], ex[PER], run = 0;
#pragma unroll
        for (int j = 0; j < PER; j++) x[j] = wb + 64 * j < n ? v[wb + 64 * j] : 0u;
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const uint32_t s = wave_inclusive_scan(x[j]);
            ex[j] = run + s - x[j];
            run += (uint32_t)__builtin_amdgcn_readlane((int)s, 63);
        }
        if (lane == 0) wsum[w] = run;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t t = wsum[k];
            pre += k < w ? t : 0u;
            tot += t;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; j++)
            if (wb + 64 * j < n) v[wb + 64 * j] = carry + pre + ex[j];
        carry += tot;
    }
    return carry;
}

}  // namespace gsr

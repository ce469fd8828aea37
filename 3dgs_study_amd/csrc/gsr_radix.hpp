// gsr_radix.hpp — wave-level stable ranking and block placement shared by the
// binning kernels (binning.hip: the depth sort and the LSD tile sort; rowspan.hip:
// the row-span binning).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gsr_common.hpp"

namespace gsr {

// Lanes of the wave whose digit equals this lane's (restricted to `live`),
// comparing the NB low digit bits (the digit is masked, so comparing more bits
// than the pass has is harmless).  Per bit: s = the sign-extended bit (0 or ~0,
// one v_bfe_i32), one ballot of s, and per mask half m &= ~(ballot ^ s) as ONE
// v_bitop3_b32 (truth table 0x90: m & (ballot == s)): 4 VALU per bit.  (A runtime
// bit count with a per-lane select of ballot / ~ballot compiled to ~11.)
__device__ __forceinline__ uint32_t and_xnor(uint32_t m, uint32_t bal, uint32_t s) {
    return __builtin_amdgcn_bitop3_b32(m, bal, s, 0x90);  // the builtin: the compiler pads its hazards
}
template <int NB>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t live) {
    uint32_t lo = (uint32_t)live, hi = (uint32_t)(live >> 32);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t s = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);  // feeds the ballot too
        const uint64_t bal = __ballot(s != 0u);
        lo = and_xnor(lo, (uint32_t)bal, s);
        hi = and_xnor(hi, (uint32_t)(bal >> 32), s);
    }
    return ((uint64_t)hi << 32) | lo;
}
// number of set bits of m below this lane
__device__ __forceinline__ uint32_t count_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Workgroup -> radix block.  The per-block digit counts live column-major
// (hist[digit][block], so the digit scan reads rows); neighbouring blocks share
// their 32-B sectors.  Workgroups are dealt round-robin over the 8 XCDs, so give
// each XCD a contiguous run of blocks: a sector's partial writes (upsweep) and
// reads (downsweep) then meet in one L2 instead of crossing to HBM once per
// block.  A bijection on [0, NB); placement is a speed hint only.
__device__ __forceinline__ uint32_t radix_block(int NB) {
    const uint32_t x = blockIdx.x & 7u, j = blockIdx.x >> 3;
    const uint32_t q = (uint32_t)NB >> 3, r = (uint32_t)NB & 7u;
    return x * q + min(x, r) + j;
}
// The same placement over the first n of a grid of at least n workgroups, for a
// block count the device computed (the grid was sized by a bound): false for the
// workgroups beyond it, which are the highest-numbered ones.
__device__ __forceinline__ bool radix_block_of(uint32_t n, uint32_t *blk) {
    const uint32_t x = blockIdx.x & 7u, j = blockIdx.x >> 3;
    const uint32_t q = n >> 3, r = n & 7u;
    if (j >= q + (x < r ? 1u : 0u)) return false;
    *blk = x * q + min(x, r) + j;
    return true;
}

}  // namespace gsr

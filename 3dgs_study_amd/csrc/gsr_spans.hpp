// gsr_spans.hpp — a Gaussian's tile footprint as row spans (rowspan.hip; the row
// counts in binning.hip's rank_gather_kernel).
//
// preprocess.hip stores per Gaussian its tile rect {x0 | x1 << 16, y0 | y1 << 16}
// (upstream's getRect) and a 64-bit row-major mask of the rect tiles it keeps:
// all ones = every tile of the rect (the rect footprint, and every rect of more
// than 64 tiles), else the tight footprint's tiles — per tile row one contiguous
// run, the ellipse's extent over the row's band.  Either way the footprint is,
// per tile row, one span of columns [xa, xb) or nothing.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

struct Foot {
    uint32_t x0, x1, y0, y1;
    uint64_t m;
    bool full;
};
__device__ __forceinline__ Foot foot_of(uint4 q) {
    Foot f;
    f.x0 = q.x & 0xffffu;
    f.x1 = q.x >> 16;
    f.y0 = q.y & 0xffffu;
    f.y1 = q.y >> 16;
    f.m = ((uint64_t)q.w << 32) | q.z;
    f.full = f.m == ~0ull;
    if (f.x1 <= f.x0) f.y1 = f.y0;  // an empty rect has no rows
    return f;
}
// the kept tiles of rect row k (0 <= k < y1 - y0) of a masked footprint, as bits
// from column x0 up (a masked rect has at most 64 tiles, so k * w < 64)
__device__ __forceinline__ uint64_t foot_row_bits(const Foot &f, uint32_t k) {
    const uint32_t w = f.x1 - f.x0;
    return (f.m >> (k * w)) & (w >= 64u ? ~0ull : ((1ull << w) - 1ull));
}
__device__ __forceinline__ bool foot_row_kept(const Foot &f, uint32_t k) { return f.full || foot_row_bits(f, k) != 0ull; }
// tile rows with at least one kept tile = the Gaussian's spans
__device__ __forceinline__ uint32_t foot_spans(const Foot &f) {
    if (f.full) return f.y1 - f.y0;
    uint32_t n = 0;
    for (uint32_t k = 0; k < f.y1 - f.y0; k++) n += foot_row_kept(f, k) ? 1u : 0u;
    return n;
}
// the span of rect row k: columns [xa, xb), packed xa | xb << 16
__device__ __forceinline__ uint32_t foot_row_span(const Foot &f, uint32_t k) {
    if (f.full) return f.x0 | (f.x1 << 16);
    const uint64_t b = foot_row_bits(f, k);
    const uint32_t xa = f.x0 + (uint32_t)__builtin_ctzll(b), xb = f.x0 + 64u - (uint32_t)__builtin_clzll(b);
    return xa | (xb << 16);
}

// The rect footprint's record as one word, for grids of at most 256 x 256 tiles:
// x0 | (x1 - 1) << 8 | y0 << 16 | (y1 - 1) << 24 (every tile of the rect), 0xff for
// an empty rect (x0 = 255 > x1 - 1 = 0).  The depth sort carries it beside each
// Gaussian's id (binning.hip), so the rank-ordered footprints need no random gather.
__device__ __forceinline__ uint32_t rect_word(uint4 q) {
    const uint32_t x0 = q.x & 0xffffu, x1 = q.x >> 16, y0 = q.y & 0xffffu, y1 = q.y >> 16;
    if (x1 <= x0 || y1 <= y0) return 0xffu;
    return x0 | ((x1 - 1u) << 8) | (y0 << 16) | ((y1 - 1u) << 24);
}
__device__ __forceinline__ Foot foot_of_word(uint32_t w) {
    Foot f;
    f.x0 = w & 0xffu;
    f.x1 = ((w >> 8) & 0xffu) + 1u;
    f.y0 = (w >> 16) & 0xffu;
    f.y1 = (w >> 24) + 1u;
    f.m = ~0ull;
    f.full = true;
    if (f.x1 <= f.x0) f.y1 = f.y0;  // empty
    return f;
}

}  // namespace gsr

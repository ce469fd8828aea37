// gsr_colour.hpp — the colour half of preprocess (forward.cu computeColorFromSH),
// shared by preprocess.hip (the fused kernel's colour stage, the side-stream
// colour kernel) and binning.hip (colour riders on the depth sort's downsweeps,
// gsr_colour_mode 2).  Every includer compiles it with FP contraction off (the
// pragma precedes its includes), so every copy gives the same bits.
#pragma once

#include "gsr_common.hpp"
#include "gsr_rows.hpp"

namespace gsr {

// SH -> RGB for one Gaussian, per channel (forward.cu computeColorFromSH).
__device__ inline float sh_channel(const float *sh, int c, int deg, float x, float y, float z) {
#define SH(k) sh[3 * (k) + c]
    float result = SH_C0 * SH(0);
    if (deg > 0) {
        result = ((result - (SH_C1 * y) * SH(1)) + (SH_C1 * z) * SH(2)) - (SH_C1 * x) * SH(3);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            result = ((((result + (SH_C2_0 * xy) * SH(4)) + (SH_C2_1 * yz) * SH(5)) +
                       (SH_C2_2 * ((2.0f * zz - xx) - yy)) * SH(6)) +
                      (SH_C2_3 * xz) * SH(7)) +
                     (SH_C2_4 * (xx - yy)) * SH(8);
            if (deg > 2) {
                result = ((((((result + ((SH_C3_0 * y) * (3.0f * xx - yy)) * SH(9)) + ((SH_C3_1 * xy) * z) * SH(10)) +
                            ((SH_C3_2 * y) * ((4.0f * zz - xx) - yy)) * SH(11)) +
                           ((SH_C3_3 * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy)) * SH(12)) +
                          ((SH_C3_4 * x) * ((4.0f * zz - xx) - yy)) * SH(13)) +
                         ((SH_C3_5 * z) * (xx - yy)) * SH(14)) +
                        ((SH_C3_6 * x) * (xx - 3.0f * yy)) * SH(15);
            }
        }
    }
#undef SH
    return result + 0.5f;
}

// One workgroup's Gaussians [blk * PRE_THREADS, +PRE_THREADS) of the kept ones
// (radii > 0): each thread loads its own 192-B row into registers (no LDS, no
// barrier: lanes without a Gaussian return at once), evaluates the colour, and
// writes the record's colour words (floats 6, 7, 8), the clamp bits and, when a
// backward follows, the SH direction Jacobian.  SPLIT: the rows are the two leaves.
template <bool SPLIT>
__device__ __forceinline__ void colour_rows48(const ColourRide &c, int blk) {
    const int idx = blk * PRE_THREADS + (int)threadIdx.x;
    if (idx >= c.P || c.radii[idx] <= 0) return;
    float4 rowv[12];
    if constexpr (SPLIT) {
        float r[48];
        load_sh_row_split(c.sh, c.sh_rest, (size_t)idx, r);
#pragma unroll
        for (int b = 0; b < 12; b++) rowv[b] = make_float4(r[4 * b], r[4 * b + 1], r[4 * b + 2], r[4 * b + 3]);
    } else {
        const float4 *r4 = reinterpret_cast<const float4 *>(c.sh + (size_t)idx * 48);
#pragma unroll
        for (int b = 0; b < 12; b++) rowv[b] = r4[b];
    }
    const float px = c.means3D[3 * idx], py = c.means3D[3 * idx + 1], pz = c.means3D[3 * idx + 2];
    const float dx = px - c.campos[0], dy = py - c.campos[1], dz = pz - c.campos[2];
    const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
    const float x = dx / len, y = dy / len, z = dz / len;
    const float *sh = reinterpret_cast<const float *>(rowv);
    float rgb[3];
    uint8_t clampbits = 0;
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const float v = sh_channel(sh, ch, c.D, x, y, z);
        clampbits |= (v < 0) ? (uint8_t)(1u << ch) : (uint8_t)0;
        rgb[ch] = fmaxf(v, 0.0f);
    }
    if (c.shjac) {
        float J[9];
        sh_dir_jacobian(sh, c.D, x, y, z, J);
#pragma unroll
        for (int k = 0; k < 9; k++) store_jac(c.shjac + (size_t)k * c.P + idx, J[k]);
    }
    float *rec = reinterpret_cast<float *>(c.splats + 3 * (size_t)idx);
    *reinterpret_cast<float2 *>(rec + 6) = make_float2(rgb[0], rgb[1]);
    rec[8] = rgb[2];
    c.clamped[idx] = clampbits;
}

}  // namespace gsr

// gsr_math.hpp — per-Gaussian math shared by the forward preprocess and the
// backward preprocess kernels.  Operation order mirrors oracle/gsr_oracle.c
// (upstream auxiliary.h / forward.cu) term for term; include
// it only from translation units compiled under `#pragma clang fp contract(off)`
// so that the integer outputs derived from it (radii, tile rects) agree with
// the oracle bit for bit.
#pragma once

#include "gsr_common.hpp"

namespace gsr {

struct f3 {
    float x, y, z;
};
struct f4 {
    float x, y, z, w;
};

// v_cvt_i32_f32 semantics (saturating, NaN -> 0) made explicit so that the
// compiler cannot assume an in-range conversion.
__device__ inline int f2i_sat(float v) {
    if (!(v == v)) return 0;
    if (v >= 2147483647.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

// auxiliary.h ndc2Pix: double literals -> evaluated in double.
__device__ inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

__device__ inline f3 xform_point4x3(const f3 p, const Mat4 &M) {
    const float *m = M.m;
    return f3{m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
}
__device__ inline f4 xform_point4x4(const f3 p, const Mat4 &M) {
    const float *m = M.m;
    return f4{m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
}
__device__ inline f3 xform_vec4x3_transpose(const f3 p, const Mat4 &M) {
    const float *m = M.m;
    return f3{m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
              m[8] * p.x + m[9] * p.y + m[10] * p.z};
}

// auxiliary.h getRect (radius arrives as int, (int) truncates toward zero).
struct TileRect {
    unsigned x0, y0, x1, y1;
};
__device__ inline unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ inline int imax_(int a, int b) { return a > b ? a : b; }
__device__ inline TileRect get_rect(float px, float py, int r, int gx, int gy) {
    TileRect t;
    t.x0 = umin_((unsigned)gx, (unsigned)imax_(0, f2i_sat((px - (float)r) / (float)TILE_X)));
    t.y0 = umin_((unsigned)gy, (unsigned)imax_(0, f2i_sat((py - (float)r) / (float)TILE_Y)));
    t.x1 = umin_((unsigned)gx, (unsigned)imax_(0, f2i_sat((((px + (float)r) + (float)TILE_X) - 1.0f) / (float)TILE_X)));
    t.y1 = umin_((unsigned)gy, (unsigned)imax_(0, f2i_sat((((py + (float)r) + (float)TILE_Y) - 1.0f) / (float)TILE_Y)));
    return t;
}

__device__ inline M3 m3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7, float a8) {
    M3 R;
    R.m[0][0] = a0; R.m[0][1] = a1; R.m[0][2] = a2;
    R.m[1][0] = a3; R.m[1][1] = a4; R.m[1][2] = a5;
    R.m[2][0] = a6; R.m[2][1] = a7; R.m[2][2] = a8;
    return R;
}
__device__ inline M3 m3_mul(const M3 &A, const M3 &B) {  // glm operator*
    M3 R;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++)
            R.m[j][i] = A.m[0][i] * B.m[j][0] + A.m[1][i] * B.m[j][1] + A.m[2][i] * B.m[j][2];
    return R;
}
__device__ inline M3 m3_transpose(const M3 &A) {
    M3 R;
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int i = 0; i < 3; i++) R.m[j][i] = A.m[i][j];
    return R;
}
__device__ inline M3 quat_to_rot(float r, float x, float y, float z) {
    return m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

// GaussianModel's activations (scene/gaussian_model.py:107-126) as torch's GPU
// kernels evaluate them, for inputs given as the stored parameters
// (gsr_inputs.activations): sigmoid 1 / (1 + exp(-x)) and exp with the accurate
// expf (torch's std::exp), F.normalize as x / clamp_min(||x||, 1e-12) with the
// norm's squares summed pairwise, ((x0^2 + x1^2) + (x2^2 + x3^2)) — the order
// torch's vector-norm reduction uses for four floats (tools/act_probe.py: equal on
// 1M of 1M rows; sequential sums and fma chains miss 8-17 %).  No contraction.
__device__ __forceinline__ float act_sigmoid(float x) {
#pragma clang fp contract(off)
    return 1.0f / (1.0f + expf(-x));
}
__device__ __forceinline__ float act_exp(float x) { return expf(x); }
// q <- x / max(n, eps) in place; returns n = ||x|| (LinalgVectorNormBackward0's result)
__device__ __forceinline__ float act_normalize(float q[4]) {
#pragma clang fp contract(off)
    const float s0 = q[0] * q[0], s1 = q[1] * q[1], s2 = q[2] * q[2], s3 = q[3] * q[3];
    const float n = sqrtf((s0 + s1) + (s2 + s3));
    const float d = n != n ? n : fmaxf(n, 1e-12f);  // clamp_min keeps a NaN
#pragma unroll
    for (int k = 0; k < 4; k++) q[k] = q[k] / d;
    return n;
}
constexpr float ACT_ROTATION_EPS = 1e-12f;  // F.normalize's default eps

// forward.cu computeCov3D: Sigma = (S R)^T (S R) in glm terms; q used as given.
__device__ inline void compute_cov3d(float sx, float sy, float sz, float mod, float qr, float qx, float qy, float qz,
                                     float cov[6]) {
    M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * sx;
    S.m[1][1] = mod * sy;
    S.m[2][2] = mod * sz;
    M3 R = quat_to_rot(qr, qx, qy, qz);
    M3 Mm = m3_mul(S, R);
    M3 Mt = m3_transpose(Mm);
    M3 Sig = m3_mul(Mt, Mm);
    cov[0] = Sig.m[0][0];
    cov[1] = Sig.m[0][1];
    cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1];
    cov[4] = Sig.m[1][2];
    cov[5] = Sig.m[2][2];
}

// forward.cu computeCov2D (EWA splatting, tan-FoV clamp, +0.3 low-pass).
__device__ inline f3 compute_cov2d(const f3 mean, float fx, float fy, float tanx, float tany, const float c3[6],
                                   const Mat4 &V) {
    f3 t = xform_point4x3(mean, V);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    M3 J = m3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    const float *v = V.m;
    M3 W = m3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    M3 T = m3_mul(W, J);
    M3 Vk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    M3 X = m3_mul(m3_transpose(T), m3_transpose(Vk));
    M3 cov = m3_mul(X, T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    return f3{cov.m[0][0], cov.m[0][1], cov.m[1][1]};
}

}  // namespace gsr

/*
 * gsr_oracle.c — CPU restatement of the differentiable Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path (3dgs_study_amd/csrc).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path never calls
 * it, and there is no CPU fallback built on it.
 *
 * What it restates.  The reference (PoplarPoplar/3dgs_study) drives the
 * rasterizer through gaussian_renderer/__init__.py:47-106, but the rasterizer
 * itself lives in the un-vendored git submodule
 *   submodules/diff-gaussian-rasterization   (.gitmodules:4-6,
 *   fork github.com/PoplarPoplar/diff-gaussian-rasterization, commit unknown)
 * whose directory is empty in the snapshot.  The algorithm below therefore
 * restates the public upstream graphdeco-inria/diff-gaussian-rasterization
 * design with the 2-output API that the reference calls
 * (tagged [UPSTREAM-SPEC] there):
 *   cuda_rasterizer/auxiliary.h      ndc2Pix, getRect, transformPoint*, dnormvdv
 *   cuda_rasterizer/forward.cu       preprocessCUDA, computeCov3D, computeCov2D,
 *                                    computeColorFromSH, renderCUDA
 *   cuda_rasterizer/rasterizer_impl.cu duplicateWithKeys, SortPairs, identifyTileRanges
 *   cuda_rasterizer/backward.cu      renderCUDA, computeCov2DCUDA, preprocessCUDA,
 *                                    computeCov3D, computeColorFromSH
 * PARITY STATUS: the CUDA original cannot be built or run here (source absent,
 * no network).  The Python-side pieces it shares with the reference are pinned
 * by golden vectors captured from the reference in this container
 * (tests/golden/make_golden.py): eval_sh (utils/sh_utils.py:57-112), the 3D
 * covariance (utils/general_utils.py:72-128, scene/gaussian_model.py:27-32) and
 * the camera matrices (utils/graphics_utils.py:49-133, scene/cameras.py:95-121).
 * The analytic backward is pinned against float64 autograd of the same
 * forward (tests/test_oracle_autograd.py).  The blend/sort stages are pinned by
 * the analytic known-answer tests of SURVEY.md A.10 only.
 *
 * Threads: liboracle.so (the checker) is single-threaded.  The same source
 * built with -fopenmp (liboracle_mt.so, bench.py's CPU baseline on all host
 * cores) runs the per-Gaussian loops, the per-tile blend loops and the sort in
 * parallel; its forward is bit-identical to the single-threaded one, its
 * render backward sums per-thread partial gradients (a different float order).
 *
 * Floating point: compile with -ffp-contract=off.  The integer outputs
 * (radii, rects, tiles_touched, keys) are derived with the same operation
 * order as the HIP preprocess kernel, which is also built without
 * contraction, so those integers must agree bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define BLOCK_X 16
#define BLOCK_Y 16
#define NUM_CH 3

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* exp for the blend's alpha: the correctly rounded float exp, taken as the
 * double-precision exp rounded once (checked equal to the correctly rounded
 * value for every float in [-16, 1]; glibc's expf differs on ~6e-5 of them).
 * Upstream's CUDA expf is accurate to 2 ulp and not reproducible off the GPU,
 * so the restatement pins the exact value: the HIP blend kernels take the same
 * `alpha < 1/255` decisions (gsr_blend.hpp blend_g). */
static float exp_rn(float x) {
    volatile double d = exp((double)x); /* volatile: no narrowing to expf */
    return (float)d;
}

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;

/* Float -> int conversion as the GPU performs it (v_cvt_i32_f32 saturates and
 * maps NaN to 0); a plain C cast is undefined out of range. */
static int f2i_sat(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

/* auxiliary.h: ndc2Pix uses double literals -> evaluated in double. */
static float ndc2Pix(float v, int S) { return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5); }

static f3 transformPoint4x3(f3 p, const float *m) {
    f3 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]};
    return t;
}
static f4 transformPoint4x4(f3 p, const float *m) {
    f4 t = {m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
            m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]};
    return t;
}
static f3 transformVec4x3Transpose(f3 p, const float *m) {
    f3 t = {m[0] * p.x + m[1] * p.y + m[2] * p.z, m[4] * p.x + m[5] * p.y + m[6] * p.z,
            m[8] * p.x + m[9] * p.y + m[10] * p.z};
    return t;
}

static unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }
static int imax_(int a, int b) { return a > b ? a : b; }

/* auxiliary.h getRect: the radius arrives as an int, (int) truncates. */
static void getRect(float px, float py, int max_radius, unsigned gx, unsigned gy, unsigned rmin[2],
                    unsigned rmax[2]) {
    rmin[0] = umin_(gx, (unsigned)imax_(0, f2i_sat((px - (float)max_radius) / (float)BLOCK_X)));
    rmin[1] = umin_(gy, (unsigned)imax_(0, f2i_sat((py - (float)max_radius) / (float)BLOCK_Y)));
    rmax[0] = umin_(gx, (unsigned)imax_(0, f2i_sat((((px + (float)max_radius) + (float)BLOCK_X) - 1.0f) / (float)BLOCK_X)));
    rmax[1] = umin_(gy, (unsigned)imax_(0, f2i_sat((((py + (float)max_radius) + (float)BLOCK_Y) - 1.0f) / (float)BLOCK_Y)));
}

/* 3x3 matrices in glm layout: m[col][row]. */
typedef struct { float m[3][3]; } mat3;

static mat3 mat3_mul(const mat3 *A, const mat3 *B) { /* glm operator* */
    mat3 R;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++)
            R.m[j][i] = A->m[0][i] * B->m[j][0] + A->m[1][i] * B->m[j][1] + A->m[2][i] * B->m[j][2];
    return R;
}
static mat3 mat3_transpose(const mat3 *A) {
    mat3 R;
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < 3; i++) R.m[j][i] = A->m[i][j];
    return R;
}
/* glm::mat3(a0..a8) fills column by column. */
static mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7, float a8) {
    mat3 R;
    R.m[0][0] = a0; R.m[0][1] = a1; R.m[0][2] = a2;
    R.m[1][0] = a3; R.m[1][1] = a4; R.m[1][2] = a5;
    R.m[2][0] = a6; R.m[2][1] = a7; R.m[2][2] = a8;
    return R;
}

static mat3 quat_to_R(float r, float x, float y, float z) {
    return mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                     2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                     2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

/* forward.cu computeCov3D: Sigma = (S*R)^T (S*R) in glm terms, q used as given. */
static void computeCov3D(const float *scale, float mod, const float *rot, float *cov3D) {
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    mat3 R = quat_to_R(rot[0], rot[1], rot[2], rot[3]);
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_transpose(&M);
    mat3 Sigma = mat3_mul(&Mt, &M);
    cov3D[0] = Sigma.m[0][0];
    cov3D[1] = Sigma.m[0][1];
    cov3D[2] = Sigma.m[0][2];
    cov3D[3] = Sigma.m[1][1];
    cov3D[4] = Sigma.m[1][2];
    cov3D[5] = Sigma.m[2][2];
}

/* forward.cu computeCov2D (EWA with tan-FoV clamp and 0.3 low-pass). */
static f3 computeCov2D(f3 mean, float fx, float fy, float tanx, float tany, const float *c3, const float *vm) {
    f3 t = transformPoint4x3(mean, vm);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    mat3 J = mat3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    mat3 W = mat3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
    mat3 T = mat3_mul(&W, &J);
    mat3 V = mat3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    mat3 Tt = mat3_transpose(&T), Vt = mat3_transpose(&V);
    mat3 X = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&X, &T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    f3 r = {cov.m[0][0], cov.m[0][1], cov.m[1][1]};
    return r;
}

/* forward.cu computeColorFromSH, per channel, glm evaluation order. */
static void computeColorFromSH(int idx, int deg, int max_coeffs, const float *means, const float *campos,
                               const float *shs, uint8_t *clamped, float *out_rgb) {
    float dx = means[3 * idx + 0] - campos[0];
    float dy = means[3 * idx + 1] - campos[1];
    float dz = means[3 * idx + 2] - campos[2];
    float len = sqrtf((dx * dx + dy * dy) + dz * dz);
    float x = dx / len, y = dy / len, z = dz / len;
    const float *sh = shs + (size_t)idx * max_coeffs * 3;
    for (int c = 0; c < 3; c++) {
#define SH(k) sh[3 * (k) + c]
        float result = SH_C0 * SH(0);
        if (deg > 0) {
            result = ((result - (SH_C1 * y) * SH(1)) + (SH_C1 * z) * SH(2)) - (SH_C1 * x) * SH(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z;
                float xy = x * y, yz = y * z, xz = x * z;
                result = ((((result + (SH_C2[0] * xy) * SH(4)) + (SH_C2[1] * yz) * SH(5)) +
                           (SH_C2[2] * ((2.0f * zz - xx) - yy)) * SH(6)) +
                          (SH_C2[3] * xz) * SH(7)) +
                         (SH_C2[4] * (xx - yy)) * SH(8);
                if (deg > 2) {
                    result = ((((((result + ((SH_C3[0] * y) * (3.0f * xx - yy)) * SH(9)) +
                                 ((SH_C3[1] * xy) * z) * SH(10)) +
                                ((SH_C3[2] * y) * ((4.0f * zz - xx) - yy)) * SH(11)) +
                               ((SH_C3[3] * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy)) * SH(12)) +
                              ((SH_C3[4] * x) * ((4.0f * zz - xx) - yy)) * SH(13)) +
                             ((SH_C3[5] * z) * (xx - yy)) * SH(14)) +
                            ((SH_C3[6] * x) * (xx - 3.0f * yy)) * SH(15);
                }
            }
        }
#undef SH
        result += 0.5f;
        clamped[3 * idx + c] = (result < 0);
        out_rgb[c] = fmaxf(result, 0.0f);
    }
}

/* ------------------------------------------------------------------------ */
/* Forward                                                                   */
/* ------------------------------------------------------------------------ */

/* forward.cu preprocessCUDA (+ auxiliary.h in_frustum).  Returns 0, or 1 if a
 * point was culled although `prefiltered` was set (upstream traps there). */
int oracle_preprocess(int P, int D, int M, const float *means3D, const float *scales, float scale_modifier,
                      const float *rotations, const float *opacities, const float *shs, uint8_t *clamped,
                      const float *cov3D_precomp, const float *colors_precomp, const float *viewmatrix,
                      const float *projmatrix, const float *campos, int W, int H, float tan_fovx, float tan_fovy,
                      int *radii, float *means2D, float *depths, float *cov3Ds, float *rgb, float *conic_opacity,
                      uint32_t *tiles_touched, int32_t *rects, int prefiltered) {
    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);
    const unsigned gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int idx = 0; idx < P; idx++) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        if (rects) { rects[4 * idx + 0] = rects[4 * idx + 1] = rects[4 * idx + 2] = rects[4 * idx + 3] = 0; }
        f3 p_orig = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        f4 p_hom = transformPoint4x4(p_orig, projmatrix);
        float p_w = 1.0f / (p_hom.w + 0.0000001f);
        f3 p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};
        f3 p_view = transformPoint4x3(p_orig, viewmatrix);
        if (p_view.z <= 0.2f) {
            if (prefiltered) bad = 1;
            continue;
        }
        const float *cov3D;
        if (cov3D_precomp) {
            cov3D = cov3D_precomp + 6 * (size_t)idx;
        } else {
            computeCov3D(scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx, cov3Ds + 6 * (size_t)idx);
            cov3D = cov3Ds + 6 * (size_t)idx;
        }
        f3 cov = computeCov2D(p_orig, focal_x, focal_y, tan_fovx, tan_fovy, cov3D, viewmatrix);
        float det = (cov.x * cov.z - cov.y * cov.y);
        if (det == 0.0f) continue;
        float det_inv = 1.f / det;
        float conic[3] = {cov.z * det_inv, -cov.y * det_inv, cov.x * det_inv};
        float mid = 0.5f * (cov.x + cov.z);
        float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        float pix_x = ndc2Pix(p_proj.x, W), pix_y = ndc2Pix(p_proj.y, H);
        unsigned rmin[2], rmax[2];
        getRect(pix_x, pix_y, f2i_sat(my_radius), gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (!colors_precomp) {
            computeColorFromSH(idx, D, M, means3D, campos, shs, clamped, rgb + 3 * (size_t)idx);
        }
        depths[idx] = p_view.z;
        radii[idx] = f2i_sat(my_radius);
        means2D[2 * idx + 0] = pix_x;
        means2D[2 * idx + 1] = pix_y;
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = opacities[idx];
        tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
        if (rects) {
            rects[4 * idx + 0] = (int32_t)rmin[0];
            rects[4 * idx + 1] = (int32_t)rmin[1];
            rects[4 * idx + 2] = (int32_t)rmax[0];
            rects[4 * idx + 3] = (int32_t)rmax[1];
        }
    }
    return bad;
}

/* cub::DeviceScan::InclusiveSum on uint32. Returns the total (num_rendered). */
int64_t oracle_inclusive_scan(int P, const uint32_t *in, uint32_t *out) {
    uint32_t acc = 0;
    for (int i = 0; i < P; i++) {
        acc += in[i];
        out[i] = acc;
    }
    return P > 0 ? (int64_t)out[P - 1] : 0;
}

/* rasterizer_impl.cu duplicateWithKeys: one (key,value) per touched tile. */
void oracle_duplicate_with_keys(int P, const float *means2D, const float *depths, const uint32_t *offsets,
                                const int *radii, int W, int H, uint64_t *keys, uint32_t *values) {
    const unsigned gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
#pragma omp parallel for schedule(dynamic, 1024)
    for (int idx = 0; idx < P; idx++) {
        if (radii[idx] <= 0) continue;
        uint32_t off = (idx == 0) ? 0 : offsets[idx - 1];
        unsigned rmin[2], rmax[2];
        getRect(means2D[2 * idx], means2D[2 * idx + 1], radii[idx], gx, gy, rmin, rmax);
        for (unsigned y = rmin[1]; y < rmax[1]; y++)
            for (unsigned x = rmin[0]; x < rmax[0]; x++) {
                uint64_t key = (uint64_t)(y * gx + x);
                key <<= 32;
                uint32_t dbits;
                memcpy(&dbits, &depths[idx], 4);
                key |= dbits;
                keys[off] = key;
                values[off] = (uint32_t)idx;
                off++;
            }
    }
}

typedef struct { uint64_t key; uint32_t val; uint32_t pos; } kv_t;
static int kv_cmp(const void *a, const void *b) {
    const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

#ifdef _OPENMP
#include <omp.h>
/* Threaded form of the same stable sort: a stable counting sort by tile (the
 * key's high word; per-thread histograms over contiguous chunks), then every
 * tile's run sorted by (key, emission position) — the qsort's order exactly. */
static void sort_pairs_mt(int64_t n, const uint64_t *keys_in, const uint32_t *vals_in, uint64_t *keys_out,
                          uint32_t *vals_out) {
    uint32_t ntiles = 0;
    for (int64_t i = 0; i < n; i++) {
        const uint32_t t = (uint32_t)(keys_in[i] >> 32) + 1;
        ntiles = t > ntiles ? t : ntiles;
    }
    const int nt = omp_get_max_threads();
    int64_t *hist = (int64_t *)calloc((size_t)nt * ntiles + 1, sizeof(int64_t));
    int64_t *start = (int64_t *)calloc((size_t)ntiles + 1, sizeof(int64_t));
    kv_t *tmp = (kv_t *)malloc(sizeof(kv_t) * (size_t)(n > 0 ? n : 1));
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num();
        const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        int64_t *h = hist + (size_t)t * ntiles;
        for (int64_t i = lo; i < hi; i++) h[keys_in[i] >> 32]++;
#pragma omp barrier
#pragma omp single
        {
            int64_t acc = 0;
            for (uint32_t b = 0; b < ntiles; b++) {
                start[b] = acc;
                for (int u = 0; u < nt; u++) {
                    const int64_t c = hist[(size_t)u * ntiles + b];
                    hist[(size_t)u * ntiles + b] = acc;
                    acc += c;
                }
            }
            start[ntiles] = acc;
        }
        for (int64_t i = lo; i < hi; i++) {
            kv_t *e = &tmp[h[keys_in[i] >> 32]++];
            e->key = keys_in[i];
            e->val = vals_in[i];
            e->pos = (uint32_t)i;
        }
#pragma omp barrier
#pragma omp for schedule(dynamic, 16)
        for (int64_t b = 0; b < (int64_t)ntiles; b++) {
            const int64_t s0 = start[b], s1 = start[b + 1];
            qsort(tmp + s0, (size_t)(s1 - s0), sizeof(kv_t), kv_cmp);
            for (int64_t i = s0; i < s1; i++) {
                keys_out[i] = tmp[i].key;
                vals_out[i] = tmp[i].val;
            }
        }
    }
    free(tmp);
    free(start);
    free(hist);
}
#endif

/* cub::DeviceRadixSort::SortPairs is stable: equal keys keep emission order. */
void oracle_sort_pairs(int64_t n, const uint64_t *keys_in, const uint32_t *vals_in, uint64_t *keys_out,
                       uint32_t *vals_out) {
#ifdef _OPENMP
    if (omp_get_max_threads() > 1) {
        sort_pairs_mt(n, keys_in, vals_in, keys_out, vals_out);
        return;
    }
#endif
    kv_t *tmp = (kv_t *)malloc(sizeof(kv_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; i++) {
        tmp[i].key = keys_in[i];
        tmp[i].val = vals_in[i];
        tmp[i].pos = (uint32_t)i;
    }
    qsort(tmp, (size_t)n, sizeof(kv_t), kv_cmp);
    for (int64_t i = 0; i < n; i++) {
        keys_out[i] = tmp[i].key;
        vals_out[i] = tmp[i].val;
    }
    free(tmp);
}

/* rasterizer_impl.cu identifyTileRanges (ranges zeroed first). */
void oracle_identify_tile_ranges(int64_t n, const uint64_t *keys, int num_tiles, uint32_t *ranges) {
    memset(ranges, 0, sizeof(uint32_t) * 2 * (size_t)num_tiles);
    for (int64_t idx = 0; idx < n; idx++) {
        uint32_t currtile = (uint32_t)(keys[idx] >> 32);
        if (idx == 0)
            ranges[2 * currtile + 0] = 0;
        else {
            uint32_t prevtile = (uint32_t)(keys[idx - 1] >> 32);
            if (currtile != prevtile) {
                ranges[2 * prevtile + 1] = (uint32_t)idx;
                ranges[2 * currtile + 0] = (uint32_t)idx;
            }
        }
        if (idx == n - 1) ranges[2 * currtile + 1] = (uint32_t)n;
    }
}

/* forward.cu renderCUDA: front-to-back alpha blending per pixel. */
void oracle_render_forward(const uint32_t *ranges, const uint32_t *point_list, int W, int H, const float *means2D,
                           const float *colors, const float *conic_opacity, float *final_T, uint32_t *n_contrib,
                           const float *bg, float *out_color) {
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ty++)
        for (int tx = 0; tx < gx; tx++) {
            const uint32_t *range = ranges + 2 * (ty * gx + tx);
            for (int ly = 0; ly < BLOCK_Y; ly++)
                for (int lx = 0; lx < BLOCK_X; lx++) {
                    int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= W || py >= H) continue;
                    float pfx = (float)px, pfy = (float)py;
                    float T = 1.0f;
                    uint32_t contributor = 0, last_contributor = 0;
                    float C[NUM_CH] = {0, 0, 0};
                    for (uint32_t k = range[0]; k < range[1]; k++) {
                        contributor++;
                        uint32_t id = point_list[k];
                        float dxp = means2D[2 * id] - pfx, dyp = means2D[2 * id + 1] - pfy;
                        const float *co = conic_opacity + 4 * (size_t)id;
                        float power = -0.5f * (co[0] * dxp * dxp + co[2] * dyp * dyp) - co[1] * dxp * dyp;
                        if (power > 0.0f) continue;
                        float alpha = fminf(0.99f, co[3] * exp_rn(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        float test_T = T * (1 - alpha);
                        if (test_T < 0.0001f) break; /* done: this one is not blended */
                        for (int ch = 0; ch < NUM_CH; ch++) C[ch] += colors[3 * (size_t)id + ch] * alpha * T;
                        T = test_T;
                        last_contributor = contributor;
                    }
                    size_t pix_id = (size_t)W * py + px;
                    final_T[pix_id] = T;
                    n_contrib[pix_id] = last_contributor;
                    for (int ch = 0; ch < NUM_CH; ch++)
                        out_color[(size_t)ch * H * W + pix_id] = C[ch] + T * bg[ch];
                }
        }
}

/* ------------------------------------------------------------------------ */
/* Backward                                                                  */
/* ------------------------------------------------------------------------ */

/* backward.cu renderCUDA: back-to-front replay; accumulates (float, in pixel
 * order) into dL_dmean2D [P][3], dL_dconic [P][4] (x,y,w used), dL_dopacity
 * [P], dL_dcolors [P][3].  Output arrays must be zeroed by the caller. */
static void render_backward_tiles(const uint32_t *ranges, const uint32_t *point_list, int W, int H, const float *bg,
                                  const float *means2D, const float *conic_opacity, const float *colors,
                                  const float *final_Ts, const uint32_t *n_contrib, const float *dL_dpixels,
                                  float *dL_dmean2D, float *dL_dconic, float *dL_dopacity, float *dL_dcolors,
                                  int tile_lo, int tile_step) {
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const float ddelx_dx = (float)(0.5 * W);
    const float ddely_dy = (float)(0.5 * H);
    for (int tile = tile_lo; tile < gx * gy; tile += tile_step) {
        const int ty = tile / gx, tx = tile % gx;
        {
            const uint32_t *range = ranges + 2 * (ty * gx + tx);
            for (int ly = 0; ly < BLOCK_Y; ly++)
                for (int lx = 0; lx < BLOCK_X; lx++) {
                    int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= W || py >= H) continue;
                    size_t pix_id = (size_t)W * py + px;
                    float pfx = (float)px, pfy = (float)py;
                    const float T_final = final_Ts[pix_id];
                    float T = T_final;
                    uint32_t contributor = range[1] - range[0];
                    const uint32_t last_contributor = n_contrib[pix_id];
                    float accum_rec[NUM_CH] = {0, 0, 0}, dL_dpixel[NUM_CH], last_color[NUM_CH] = {0, 0, 0};
                    float last_alpha = 0;
                    for (int ch = 0; ch < NUM_CH; ch++) dL_dpixel[ch] = dL_dpixels[(size_t)ch * H * W + pix_id];
                    for (int64_t k = (int64_t)range[1] - 1; k >= (int64_t)range[0]; k--) {
                        contributor--;
                        if (contributor >= last_contributor) continue;
                        uint32_t gid = point_list[k];
                        float dxp = means2D[2 * gid] - pfx, dyp = means2D[2 * gid + 1] - pfy;
                        const float *co = conic_opacity + 4 * (size_t)gid;
                        float power = -0.5f * (co[0] * dxp * dxp + co[2] * dyp * dyp) - co[1] * dxp * dyp;
                        if (power > 0.0f) continue;
                        float G = exp_rn(power);
                        float alpha = fminf(0.99f, co[3] * G);
                        if (alpha < 1.0f / 255.0f) continue;
                        T = T / (1.f - alpha);
                        float dchannel_dcolor = alpha * T;
                        float dL_dalpha = 0.0f;
                        for (int ch = 0; ch < NUM_CH; ch++) {
                            float c = colors[3 * (size_t)gid + ch];
                            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                            last_color[ch] = c;
                            float dL_dchannel = dL_dpixel[ch];
                            dL_dalpha += (c - accum_rec[ch]) * dL_dchannel;
                            dL_dcolors[3 * (size_t)gid + ch] += dchannel_dcolor * dL_dchannel;
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        float bg_dot_dpixel = 0;
                        for (int ch = 0; ch < NUM_CH; ch++) bg_dot_dpixel += bg[ch] * dL_dpixel[ch];
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot_dpixel;
                        float dL_dG = co[3] * dL_dalpha;
                        float gdx = G * dxp, gdy = G * dyp;
                        float dG_ddelx = -gdx * co[0] - gdy * co[1];
                        float dG_ddely = -gdy * co[2] - gdx * co[1];
                        dL_dmean2D[3 * (size_t)gid + 0] += dL_dG * dG_ddelx * ddelx_dx;
                        dL_dmean2D[3 * (size_t)gid + 1] += dL_dG * dG_ddely * ddely_dy;
                        dL_dconic[4 * (size_t)gid + 0] += -0.5f * gdx * dxp * dL_dG;
                        dL_dconic[4 * (size_t)gid + 1] += -0.5f * gdx * dyp * dL_dG;
                        dL_dconic[4 * (size_t)gid + 3] += -0.5f * gdy * dyp * dL_dG;
                        dL_dopacity[gid] += G * dL_dalpha;
                    }
                }
        }
    }
}

void oracle_render_backward_p(int P, const uint32_t *ranges, const uint32_t *point_list, int W, int H,
                              const float *bg, const float *means2D, const float *conic_opacity, const float *colors,
                              const float *final_Ts, const uint32_t *n_contrib, const float *dL_dpixels,
                              float *dL_dmean2D, float *dL_dconic, float *dL_dopacity, float *dL_dcolors) {
#ifdef _OPENMP
    const int nt = omp_get_max_threads();
    if (nt > 1) {
        /* each thread replays the tiles it takes into its own zeroed partials;
         * the partials are then added in thread order */
        const size_t per = (size_t)P * 11;
        float *part = (float *)calloc(per * (size_t)nt, sizeof(float));
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num();
            float *q = part + per * (size_t)t;
            const int ntile = ((W + BLOCK_X - 1) / BLOCK_X) * ((H + BLOCK_Y - 1) / BLOCK_Y);
#pragma omp for schedule(dynamic, 2)
            for (int tile = 0; tile < ntile; tile++)  /* one tile per call */
                render_backward_tiles(ranges, point_list, W, H, bg, means2D, conic_opacity, colors, final_Ts,
                                      n_contrib, dL_dpixels, q, q + 3 * (size_t)P, q + 7 * (size_t)P,
                                      q + 8 * (size_t)P, tile, ntile);
#pragma omp for schedule(static)
            for (int64_t i = 0; i < (int64_t)P; i++) {
                for (int u = 0; u < nt; u++) {
                    const float *r = part + per * (size_t)u;
                    for (int c = 0; c < 3; c++) dL_dmean2D[3 * i + c] += r[3 * i + c];
                    for (int c = 0; c < 4; c++) dL_dconic[4 * i + c] += r[3 * (size_t)P + 4 * i + c];
                    dL_dopacity[i] += r[7 * (size_t)P + i];
                    for (int c = 0; c < 3; c++) dL_dcolors[3 * i + c] += r[8 * (size_t)P + 3 * i + c];
                }
            }
        }
        free(part);
        return;
    }
#endif
    render_backward_tiles(ranges, point_list, W, H, bg, means2D, conic_opacity, colors, final_Ts, n_contrib,
                          dL_dpixels, dL_dmean2D, dL_dconic, dL_dopacity, dL_dcolors, 0, 1);
}

/* backward.cu computeCov2DCUDA: dL/dconic -> dL/dcov3D and (assigned) dL/dmean3D. */
void oracle_cov2d_backward(int P, const float *means, const int *radii, const float *cov3Ds, float h_x, float h_y,
                           float tan_fovx, float tan_fovy, const float *view_matrix, const float *dL_dconics,
                           float *dL_dmeans, float *dL_dcov) {
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        const float *c3 = cov3Ds + 6 * (size_t)idx;
        f3 mean = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
        f3 g = {dL_dconics[4 * idx], dL_dconics[4 * idx + 1], dL_dconics[4 * idx + 3]};
        f3 t = transformPoint4x3(mean, view_matrix);
        const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
        const float txtz = t.x / t.z, tytz = t.y / t.z;
        t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
        t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
        const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
        const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
        mat3 J = mat3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0, 0, 0);
        const float *vm = view_matrix;
        mat3 W = mat3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
        mat3 V = mat3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
        mat3 T = mat3_mul(&W, &J);
        mat3 Tt = mat3_transpose(&T), Vt = mat3_transpose(&V);
        mat3 X = mat3_mul(&Tt, &Vt);
        mat3 cov2D = mat3_mul(&X, &T);
        float a = cov2D.m[0][0] += 0.3f;
        float b = cov2D.m[0][1];
        float c = cov2D.m[1][1] += 0.3f;
        float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float *dc = dL_dcov + 6 * (size_t)idx;
#define TT(i, j) T.m[i][j]
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * g.x + 2 * b * c * g.y + (denom - a * c) * g.z);
            dL_dc = denom2inv * (-a * a * g.z + 2 * a * b * g.y + (denom - a * c) * g.x);
            dL_db = denom2inv * 2 * (b * c * g.x - (denom + 2 * b * b) * g.y + a * b * g.z);
            dc[0] = (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc);
            dc[3] = (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc);
            dc[5] = (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc);
            dc[1] = 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                    2 * TT(1, 0) * TT(1, 1) * dL_dc;
            dc[2] = 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                    2 * TT(1, 0) * TT(1, 2) * dL_dc;
            dc[4] = 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                    2 * TT(1, 1) * TT(1, 2) * dL_dc;
        } else {
            for (int i = 0; i < 6; i++) dc[i] = 0;
        }
#define VV(i, j) V.m[i][j]
        float dL_dT00 = 2 * (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_da +
                        (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_db;
        float dL_dT01 = 2 * (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_da +
                        (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_db;
        float dL_dT02 = 2 * (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_da +
                        (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_db;
        float dL_dT10 = 2 * (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_dc +
                        (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_db;
        float dL_dT11 = 2 * (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_dc +
                        (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_db;
        float dL_dT12 = 2 * (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_dc +
                        (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_db;
#undef TT
#undef VV
        float dL_dJ00 = W.m[0][0] * dL_dT00 + W.m[0][1] * dL_dT01 + W.m[0][2] * dL_dT02;
        float dL_dJ02 = W.m[2][0] * dL_dT00 + W.m[2][1] * dL_dT01 + W.m[2][2] * dL_dT02;
        float dL_dJ11 = W.m[1][0] * dL_dT10 + W.m[1][1] * dL_dT11 + W.m[1][2] * dL_dT12;
        float dL_dJ12 = W.m[2][0] * dL_dT10 + W.m[2][1] * dL_dT11 + W.m[2][2] * dL_dT12;
        float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
        float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
        float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                       (2 * h_y * t.y) * tz3 * dL_dJ12;
        f3 dt = {dL_dtx, dL_dty, dL_dtz};
        f3 dm = transformVec4x3Transpose(dt, view_matrix);
        dL_dmeans[3 * idx + 0] = dm.x;
        dL_dmeans[3 * idx + 1] = dm.y;
        dL_dmeans[3 * idx + 2] = dm.z;
    }
}

/* backward.cu computeColorFromSH (backward). */
static void sh_backward(int idx, int deg, int max_coeffs, const float *means, const float *campos, const float *shs,
                        const uint8_t *clamped, const float *dL_dcolor, float *dL_dmeans, float *dL_dshs) {
    float ox = means[3 * idx] - campos[0], oy = means[3 * idx + 1] - campos[1], oz = means[3 * idx + 2] - campos[2];
    float len = sqrtf((ox * ox + oy * oy) + oz * oz);
    float x = ox / len, y = oy / len, z = oz / len;
    const float *sh = shs + (size_t)idx * max_coeffs * 3;
    float *dsh = dL_dshs + (size_t)idx * max_coeffs * 3;
    float dRGB[3], dRGBdx[3] = {0, 0, 0}, dRGBdy[3] = {0, 0, 0}, dRGBdz[3] = {0, 0, 0};
    for (int c = 0; c < 3; c++) dRGB[c] = dL_dcolor[3 * idx + c] * (clamped[3 * idx + c] ? 0.f : 1.f);
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; c++) {
#define SH(k) sh[3 * (k) + c]
        dsh[c] = SH_C0 * dRGB[c];
        if (deg > 0) {
            dsh[3 * 1 + c] = (-SH_C1 * y) * dRGB[c];
            dsh[3 * 2 + c] = (SH_C1 * z) * dRGB[c];
            dsh[3 * 3 + c] = (-SH_C1 * x) * dRGB[c];
            dRGBdx[c] = -SH_C1 * SH(3);
            dRGBdy[c] = -SH_C1 * SH(1);
            dRGBdz[c] = SH_C1 * SH(2);
            if (deg > 1) {
                dsh[3 * 4 + c] = (SH_C2[0] * xy) * dRGB[c];
                dsh[3 * 5 + c] = (SH_C2[1] * yz) * dRGB[c];
                dsh[3 * 6 + c] = (SH_C2[2] * (2.f * zz - xx - yy)) * dRGB[c];
                dsh[3 * 7 + c] = (SH_C2[3] * xz) * dRGB[c];
                dsh[3 * 8 + c] = (SH_C2[4] * (xx - yy)) * dRGB[c];
                dRGBdx[c] += SH_C2[0] * y * SH(4) + SH_C2[2] * 2.f * -x * SH(6) + SH_C2[3] * z * SH(7) +
                             SH_C2[4] * 2.f * x * SH(8);
                dRGBdy[c] += SH_C2[0] * x * SH(4) + SH_C2[1] * z * SH(5) + SH_C2[2] * 2.f * -y * SH(6) +
                             SH_C2[4] * 2.f * -y * SH(8);
                dRGBdz[c] += SH_C2[1] * y * SH(5) + SH_C2[2] * 2.f * 2.f * z * SH(6) + SH_C2[3] * x * SH(7);
                if (deg > 2) {
                    dsh[3 * 9 + c] = (SH_C3[0] * y * (3.f * xx - yy)) * dRGB[c];
                    dsh[3 * 10 + c] = (SH_C3[1] * xy * z) * dRGB[c];
                    dsh[3 * 11 + c] = (SH_C3[2] * y * (4.f * zz - xx - yy)) * dRGB[c];
                    dsh[3 * 12 + c] = (SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)) * dRGB[c];
                    dsh[3 * 13 + c] = (SH_C3[4] * x * (4.f * zz - xx - yy)) * dRGB[c];
                    dsh[3 * 14 + c] = (SH_C3[5] * z * (xx - yy)) * dRGB[c];
                    dsh[3 * 15 + c] = (SH_C3[6] * x * (xx - 3.f * yy)) * dRGB[c];
                    dRGBdx[c] += (SH_C3[0] * SH(9) * 3.f * 2.f * xy + SH_C3[1] * SH(10) * yz +
                                  SH_C3[2] * SH(11) * -2.f * xy + SH_C3[3] * SH(12) * -3.f * 2.f * xz +
                                  SH_C3[4] * SH(13) * (-3.f * xx + 4.f * zz - yy) + SH_C3[5] * SH(14) * 2.f * xz +
                                  SH_C3[6] * SH(15) * 3.f * (xx - yy));
                    dRGBdy[c] += (SH_C3[0] * SH(9) * 3.f * (xx - yy) + SH_C3[1] * SH(10) * xz +
                                  SH_C3[2] * SH(11) * (-3.f * yy + 4.f * zz - xx) + SH_C3[3] * SH(12) * -3.f * 2.f * yz +
                                  SH_C3[4] * SH(13) * -2.f * xy + SH_C3[5] * SH(14) * -2.f * yz +
                                  SH_C3[6] * SH(15) * -3.f * 2.f * xy);
                    dRGBdz[c] += (SH_C3[1] * SH(10) * xy + SH_C3[2] * SH(11) * 4.f * 2.f * yz +
                                  SH_C3[3] * SH(12) * 3.f * (2.f * zz - xx - yy) + SH_C3[4] * SH(13) * 4.f * 2.f * xz +
                                  SH_C3[5] * SH(14) * (xx - yy));
                }
            }
        }
#undef SH
    }
    float ddx = (dRGBdx[0] * dRGB[0] + dRGBdx[1] * dRGB[1]) + dRGBdx[2] * dRGB[2];
    float ddy = (dRGBdy[0] * dRGB[0] + dRGBdy[1] * dRGB[1]) + dRGBdy[2] * dRGB[2];
    float ddz = (dRGBdz[0] * dRGB[0] + dRGBdz[1] * dRGB[1]) + dRGBdz[2] * dRGB[2];
    /* auxiliary.h dnormvdv */
    float sum2 = ox * ox + oy * oy + oz * oz;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    float dmx = ((+sum2 - ox * ox) * ddx - oy * ox * ddy - oz * ox * ddz) * invsum32;
    float dmy = (-ox * oy * ddx + (sum2 - oy * oy) * ddy - oz * oy * ddz) * invsum32;
    float dmz = (-ox * oz * ddx - oy * oz * ddy + (sum2 - oz * oz) * ddz) * invsum32;
    dL_dmeans[3 * idx + 0] += dmx;
    dL_dmeans[3 * idx + 1] += dmy;
    dL_dmeans[3 * idx + 2] += dmz;
}

/* backward.cu computeCov3D (backward): dL/dcov3D -> dL/dscale, dL/drot (q as given). */
static void cov3d_backward(int idx, const float *scale, float mod, const float *rot, const float *dL_dcov3Ds,
                           float *dL_dscales, float *dL_drots) {
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = quat_to_R(r, x, y, z);
    mat3 S = mat3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    S.m[0][0] = s[0];
    S.m[1][1] = s[1];
    S.m[2][2] = s[2];
    mat3 M = mat3_mul(&S, &R);
    const float *d = dL_dcov3Ds + 6 * (size_t)idx;
    mat3 dL_dSigma = mat3_cols(d[0], 0.5f * d[1], 0.5f * d[2], 0.5f * d[1], d[3], 0.5f * d[4], 0.5f * d[2],
                               0.5f * d[4], d[5]);
    mat3 twoM;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) twoM.m[i][j] = 2.0f * M.m[i][j];
    mat3 dL_dM = mat3_mul(&twoM, &dL_dSigma);
    mat3 Rt = mat3_transpose(&R);
    mat3 dMt = mat3_transpose(&dL_dM);
    for (int k = 0; k < 3; k++)
        dL_dscales[3 * idx + k] = (Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1]) + Rt.m[k][2] * dMt.m[k][2];
    for (int k = 0; k < 3; k++)
        for (int j = 0; j < 3; j++) dMt.m[k][j] *= s[k];
#define D(i, j) dMt.m[i][j]
    float dq0 = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    float dq1 = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) -
                4 * x * (D(2, 2) + D(1, 1));
    float dq2 = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) -
                4 * y * (D(2, 2) + D(0, 0));
    float dq3 = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) -
                4 * z * (D(1, 1) + D(0, 0));
#undef D
    dL_drots[4 * idx + 0] = dq0;
    dL_drots[4 * idx + 1] = dq1;
    dL_drots[4 * idx + 2] = dq2;
    dL_drots[4 * idx + 3] = dq3;
}

/* backward.cu preprocessCUDA: 2D-mean, SH and cov3D backward.  dL_dmeans
 * holds the cov2D part (assigned earlier) and is accumulated into. */
void oracle_preprocess_backward(int P, int D, int M, const float *means, const int *radii, const float *shs,
                                const uint8_t *clamped, const float *scales, const float *rotations,
                                float scale_modifier, const float *proj, const float *campos,
                                const float *dL_dmean2D, float *dL_dmeans, const float *dL_dcolor,
                                const float *dL_dcov3D, float *dL_dsh, float *dL_dscale, float *dL_drot) {
#pragma omp parallel for schedule(static)
    for (int idx = 0; idx < P; idx++) {
        if (!(radii[idx] > 0)) continue;
        f3 m = {means[3 * idx], means[3 * idx + 1], means[3 * idx + 2]};
        f4 m_hom = transformPoint4x4(m, proj);
        float m_w = 1.0f / (m_hom.w + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        float gx = dL_dmean2D[3 * idx], gy = dL_dmean2D[3 * idx + 1];
        float dmx = (proj[0] * m_w - proj[3] * mul1) * gx + (proj[1] * m_w - proj[3] * mul2) * gy;
        float dmy = (proj[4] * m_w - proj[7] * mul1) * gx + (proj[5] * m_w - proj[7] * mul2) * gy;
        float dmz = (proj[8] * m_w - proj[11] * mul1) * gx + (proj[9] * m_w - proj[11] * mul2) * gy;
        dL_dmeans[3 * idx + 0] += dmx;
        dL_dmeans[3 * idx + 1] += dmy;
        dL_dmeans[3 * idx + 2] += dmz;
        if (shs) sh_backward(idx, D, M, means, campos, shs, clamped, dL_dcolor, dL_dmeans, dL_dsh);
        if (scales)
            cov3d_backward(idx, scales + 3 * (size_t)idx, scale_modifier, rotations + 4 * (size_t)idx, dL_dcov3D,
                           dL_dscale, dL_drot);
    }
}

/* auxiliary.h in_frustum via checkFrustum (_C.mark_visible). */
void oracle_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present) {
    for (int idx = 0; idx < P; idx++) {
        f3 p = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
        f3 pv = transformPoint4x3(p, viewmatrix);
        present[idx] = !(pv.z <= 0.2f);
    }
}

/* Stand-alone SH->RGB and cov3D (for golden-vector checks against the
 * reference's utils/sh_utils.py:eval_sh and utils/general_utils.py). */
void oracle_sh_to_rgb(int P, int deg, int max_coeffs, const float *means, const float *campos, const float *shs,
                      uint8_t *clamped, float *rgb) {
    for (int idx = 0; idx < P; idx++) computeColorFromSH(idx, deg, max_coeffs, means, campos, shs, clamped, rgb + 3 * (size_t)idx);
}
void oracle_cov3d(int P, const float *scales, float mod, const float *rotations, float *cov3D) {
    for (int idx = 0; idx < P; idx++) computeCov3D(scales + 3 * (size_t)idx, mod, rotations + 4 * (size_t)idx, cov3D + 6 * (size_t)idx);
}

/* View-parallel SH exchange (3dgs_study_amd/multiview.py; not upstream): the sum
 * over views of backward.cu computeColorFromSH's dL/dsh for colour gradients
 * that are already clamp-masked, added in view order.  dsh_sum [P][M][3]. */
void oracle_sh_grad_sum(int P, int nviews, int M, const float *means, const float *campos, const int *degs,
                        const float *drgb, float *dsh_sum) {
    float *zeros_sh = (float *)calloc((size_t)P * M * 3, sizeof(float));
    uint8_t *noclamp = (uint8_t *)calloc((size_t)P * 3, 1);
    float *dmean = (float *)calloc((size_t)P * 3, sizeof(float));
    float *dsh = (float *)calloc((size_t)P * M * 3, sizeof(float));
    for (size_t i = 0; i < (size_t)P * M * 3; i++) dsh_sum[i] = 0.f;
    for (int v = 0; v < nviews; v++) {
        memset(dsh, 0, (size_t)P * M * 3 * sizeof(float));
        const float *d = drgb + (size_t)v * P * 3;
        for (int i = 0; i < P; i++) {
            /* a view whose colour gradient is zero (culled, clamped) adds nothing; upstream
             * never evaluates the basis for a culled Gaussian (NaN at the camera centre) */
            if (d[3 * i] == 0.f && d[3 * i + 1] == 0.f && d[3 * i + 2] == 0.f) continue;
            sh_backward(i, degs[v], M, means, campos + 3 * v, zeros_sh, noclamp, d, dmean, dsh);
        }
        for (size_t i = 0; i < (size_t)P * M * 3; i++) dsh_sum[i] += dsh[i];
    }
    free(zeros_sh);
    free(noclamp);
    free(dmean);
    free(dsh);
}

/* threads the parallel loops use (1 in the single-threaded checker build) */
int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

// preprocess_bwd.hip — per-Gaussian backward (fused).
//
// Replaces upstream BACKWARD::computeCov2DCUDA + BACKWARD::preprocessCUDA
// (+ computeColorFromSH / computeCov3D backward) of backward.cu (SURVEY.md
// §8a rows a16/a17, Appendix A.8) with ONE kernel: it reads the Gaussian's
// accumulator row written by render_bwd, recomputes cov3D/cov2D (instead of
// storing cov3D in the forward: 24 B/Gaussian written + read saved), and
// writes every output tensor exactly once, zeros for culled Gaussians, so the
// caller needs no memset of the 8 gradient tensors.
#pragma clang fp contract(off)

#include "gsr_kernels.hpp"
#include "gsr_math.hpp"
#include "gsr_rows.hpp"

namespace gsr {

struct PreBwdArgs {
    gsr_inputs in;
    float focal_x, focal_y;
    const int32_t *radii;
    const uint8_t *clamped;
    const float *splat_f;  // the forward's splat records as floats (opacity at 12 i + 5), when in.opacities is NULL
    const float *accum;
    const float *shjac;     // [9][P] the forward's SH direction Jacobian (valid iff ctrl[CTRL_SHJAC])
    const uint32_t *ctrl;   // geom control words
    BwdOutputs o;
};

// backward.cu computeColorFromSH (backward), given the colour's derivatives with
// respect to the normalised view direction (J[3 axis + c], sh_dir_jacobian: stored
// by the forward, or computed here from the SH row): dsh (b[k] * dRGB[c] for the
// active coefficients, zeros for the rest of the M) and the direction term of
// dL/dmean3D.  `dsh` may be the row the Jacobian was computed from.
// the direction term of dL/dmean3D from d colour / d direction (auxiliary.h dnormvdv)
__device__ __forceinline__ void sh_dir_term(const float J[9], float ox, float oy, float oz, const float dRGB[3],
                                            f3 &dmean) {
    const float ddx = (J[0] * dRGB[0] + J[1] * dRGB[1]) + J[2] * dRGB[2];
    const float ddy = (J[3] * dRGB[0] + J[4] * dRGB[1]) + J[5] * dRGB[2];
    const float ddz = (J[6] * dRGB[0] + J[7] * dRGB[1]) + J[8] * dRGB[2];
    const float sum2 = ox * ox + oy * oy + oz * oz;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    dmean.x += ((+sum2 - ox * ox) * ddx - oy * ox * ddy - oz * ox * ddz) * invsum32;
    dmean.y += (-ox * oy * ddx + (sum2 - oy * oy) * ddy - oz * oy * ddz) * invsum32;
    dmean.z += (-ox * oz * ddx - oy * oz * ddy + (sum2 - oz * oz) * ddz) * invsum32;
}
// the basis of the view direction o / |o| (sh_basis: the products dsh = b[k] * dRGB[c])
__device__ __forceinline__ void sh_dir_basis(int deg, float ox, float oy, float oz, float b[16]) {
    const float len = sqrtf((ox * ox + oy * oy) + oz * oz);
    sh_basis(deg, ox / len, oy / len, oz / len, b);
}
__device__ __forceinline__ void sh_backward_j(const float J[9], float *dsh, int deg, int M, float ox, float oy,
                                              float oz, const float dRGB[3], f3 &dmean) {
    const int ncoef = (deg + 1) * (deg + 1);
    float b[16];
    sh_dir_basis(deg, ox, oy, oz, b);
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const float d = dRGB[c];
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (k < ncoef) dsh[3 * k + c] = b[k] * d;
    }
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (k >= ncoef && k < M) dsh[3 * k + 0] = dsh[3 * k + 1] = dsh[3 * k + 2] = 0.f;
    for (int k = max(ncoef, 16); k < M; k++) dsh[3 * k + 0] = dsh[3 * k + 1] = dsh[3 * k + 2] = 0.f;
    sh_dir_term(J, ox, oy, oz, dRGB, dmean);
}
// The same from the SH row itself (no stored Jacobian): every coefficient is read
// (into J) before any gradient is written, so `sh` and `dsh` may alias.
__device__ __forceinline__ void sh_backward(const float *sh, float *dsh, int deg, int M, float ox, float oy, float oz,
                                            const float dRGB[3], f3 &dmean) {
    const float len = sqrtf((ox * ox + oy * oy) + oz * oz);
    float J[9];
    sh_dir_jacobian(sh, deg, ox / len, oy / len, oz / len, J);
    sh_backward_j(J, dsh, deg, M, ox, oy, oz, dRGB, dmean);
}

constexpr int PB_THREADS = 256;

// dL/dSH of a degree-3 row (48 floats in registers) into the two leaves of the
// caller's SH cat (gsr_leaf_grads): floats 0-2 to dsh_dc [P,1,3], floats 3-47 to
// dsh_rest [P,15,3].  The 180-B rest rows pass through a per-wave LDS image of 32
// rows at a time and leave as coalesced 16-B stores over the wave's contiguous
// slice (per-lane stores at a 180-B stride ran 2x slower in sh_exchange.hip).
// Every thread of the workgroup calls it (barriers).
__device__ __forceinline__ void leaf_sh_store_direct(const gsr_leaf_grads &L, int P, int idx, bool live,
                                                     const float rowv[48]) {
    __shared__ __attribute__((aligned(16))) float stage[PB_THREADS / 64][32 * 45];
    const bool add = (L.accumulate & 1) != 0;
    if (live)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            float *p = L.dsh_dc + 3 * (size_t)idx + c;
            *p = add ? *p + rowv[c] : rowv[c];
        }
    const int lane = threadIdx.x & 63;
    float *buf = stage[threadIdx.x >> 6];
    const size_t wave_g0 = (size_t)blockIdx.x * PB_THREADS + (threadIdx.x & ~63u);
    const size_t limit = (size_t)45 * P;  // floats in dsh_rest
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if ((lane >> 5) == h)
#pragma unroll
            for (int j = 0; j < 45; j++) buf[(lane & 31) * 45 + j] = rowv[3 + j];
        __syncthreads();
        const size_t f0 = (wave_g0 + 32 * h) * 45;  // the half's first float in dsh_rest
#pragma unroll
        for (int m = 0; m < 6; m++) {
            const int i = lane + 64 * m;  // float4 of the half's 32 x 45 floats
            if (i < 360) {
                const size_t f = f0 + 4 * (size_t)i;
                const float4 v = *reinterpret_cast<const float4 *>(buf + 4 * i);
                if (f + 4 <= limit) {
                    float4 *d = reinterpret_cast<float4 *>(L.dsh_rest + f);
                    if (add) {
                        const float4 o = *d;
                        *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
                    } else {
                        *d = v;
                    }
                } else {
                    const float vv[4] = {v.x, v.y, v.z, v.w};
                    for (int c = 0; c < 4; c++)
                        if (f + c < limit) L.dsh_rest[f + c] = add ? L.dsh_rest[f + c] + vv[c] : vv[c];
                }
            }
        }
        __syncthreads();
    }
}

// The same leaves from each Gaussian's basis and colour gradient instead of its
// 48-float dsh row (preprocess_bwd_kernel<48, *, true>): leaf_sh_store_direct's
// half-wave LDS image and coalesced 16-B stores, with each lane's 45 rest floats
// formed as b[k] * dRGB[c] — the products sh_backward_j forms, so the same bits —
// as they go into LDS, so no row is held in registers (77 instead of 125 VGPRs: 6
// waves per SIMD, not 4).  Every thread of the workgroup calls it (barriers).
__device__ __forceinline__ void leaf_sh_store_basis(const gsr_leaf_grads &L, int P, int idx, bool live, bool vis,
                                                    int ncoef, const float b[16], const float dRGB[3]) {
    __shared__ __attribute__((aligned(16))) float stage[PB_THREADS / 64][32 * 45];
    const bool add = (L.accumulate & 1) != 0;
    auto coef = [&](int k, int c) { return vis && k < ncoef ? b[k] * dRGB[c] : 0.f; };
    if (live)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            float *p = L.dsh_dc + 3 * (size_t)idx + c;
            if (add)
                *p += coef(0, c);
            else
                store_stream<2>(p, coef(0, c));
        }
    const int lane = threadIdx.x & 63;
    float *buf = stage[threadIdx.x >> 6];
    const size_t wave_g0 = (size_t)blockIdx.x * PB_THREADS + (threadIdx.x & ~63u);
    const size_t limit = (size_t)45 * P;  // floats in dsh_rest
#pragma unroll
    for (int h = 0; h < 2; h++) {
        if ((lane >> 5) == h)
#pragma unroll
            for (int k = 1; k < 16; k++)
#pragma unroll
                for (int c = 0; c < 3; c++) buf[(lane & 31) * 45 + 3 * (k - 1) + c] = coef(k, c);
        __syncthreads();
        const size_t f0 = (wave_g0 + 32 * h) * 45;  // the half's first float in dsh_rest
#pragma unroll
        for (int m = 0; m < 6; m++) {
            const int i = lane + 64 * m;  // float4 of the half's 32 x 45 floats
            if (i < 360) {
                const size_t f = f0 + 4 * (size_t)i;
                const float4 v = *reinterpret_cast<const float4 *>(buf + 4 * i);
                if (f + 4 <= limit) {
                    float4 *d = reinterpret_cast<float4 *>(L.dsh_rest + f);
                    if (add) {
                        const float4 o = *d;
                        *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
                    } else {
                        store_stream<1>(d, v);
                    }
                } else {
                    const float vv[4] = {v.x, v.y, v.z, v.w};
                    for (int c = 0; c < 4; c++)
                        if (f + c < limit) L.dsh_rest[f + c] = add ? L.dsh_rest[f + c] + vv[c] : vv[c];
                }
            }
        }
        __syncthreads();
    }
}

// What the SH stage (after the rows reach LDS) needs from the geometry stage.
struct ShStage {
    f3 dmean;      // dL/dmean3D so far
    float dRGB[3];  // clamp-masked colour gradient
    bool vis;
};
__device__ ShStage preprocess_bwd_geom(const PreBwdArgs &a, int idx, const f3 mean, const float gin[7],
                                       const float4 acc0, const float4 acc1, float accb, float opac, float qnorm,
                                       int32_t rad, uint32_t cl, const Mat4 &V, const Mat4 &Pm);

// One workgroup = PB_THREADS consecutive Gaussians.  Each thread loads its own
// inputs first and, at SH degree 3, its own 192-B SH row once the geometry
// backward — cov2D, projection, cov3D — is done (12 x 16 B into registers; issued
// before the geometry, the row's 48 registers were held through it: 122 vs 117
// VGPRs, and 118 vs 114 us at config C on one box), turns the row into dL/dSH in
// place in registers and stores it (row or coefficient-plane layout).  With no
// LDS stage the kernel runs 4 waves per SIMD instead of 3 (112 -> 102 us at config
// C); forcing 5 or 6 spilled (160 us).  Other degrees stage the workgroup's rows
// through LDS and stream them back out coalesced.
// SPLIT: the SH rows come from GaussianModel's two leaves (gsr_inputs.sh_rest).
// LB (degree-3 rows, no dsh output: the leaves, or the exchange's colour gradient
// only): no 48-float row in registers — the Jacobian from the forward's planes (or
// from the row, loaded only to form it), the leaves through leaf_sh_store_basis.
template <int RWC, bool SPLIT, bool LB = false>
__global__ void __launch_bounds__(PB_THREADS) preprocess_bwd_kernel(PreBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sh_lds[];  // [PB_THREADS][3M + 1]
    const gsr_inputs &in = a.in;
    const int g0 = blockIdx.x * PB_THREADS;
    const int n = min(PB_THREADS, in.P - g0);
    const int RW = RWC > 0 ? RWC : 3 * in.M;  // SH row width (floats)
    // the rows are needed for dL/dmean3D's view-direction term even when the
    // exchange takes the colour gradient instead of dsh
    const bool stage = in.sh != nullptr &&
                       (a.o.dsh != nullptr || a.o.drgb != nullptr || a.o.sh_dir || a.o.leaf.dsh_dc != nullptr) &&
                       in.M > 0;
    constexpr bool DIRECT = RWC == 48;  // each thread's own row in registers, no LDS
    const int idx = g0 + (int)threadIdx.x;
    const bool live = idx < in.P;
    const int li = live ? idx : in.P - 1;
    // the forward stored d colour / d direction (a backward was announced): the SH
    // rows are not read at all — dsh needs only the basis, the direction term J
    const bool jac = stage && a.ctrl[CTRL_SHJAC] != 0u;
    // per-Gaussian inputs (issued before the rows: vmcnt counts in issue order)
    const f3 mean = {in.means3D[3 * li], in.means3D[3 * li + 1], in.means3D[3 * li + 2]};
    const Mat4 V = load_mat4(in.viewmatrix);
    const Mat4 Pm = load_mat4(in.projmatrix);
    float gin[7];  // scales + rotation, or the precomputed cov3D
    if (in.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) gin[k] = in.cov3D_precomp[6 * (size_t)li + k];
        gin[6] = 0.f;
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) gin[k] = in.scales[3 * (size_t)li + k];
#pragma unroll
        for (int k = 0; k < 4; k++) gin[3 + k] = in.rotations[4 * (size_t)li + k];
    }
    const float *acc = a.accum + (size_t)li * ACCUM_STRIDE;
    // the row (render_bwd.hip): colour r, g, b, mean2D.x | mean2D.y, conic.x, conic.y, conic.w | opacity
    const float4 row0 = *reinterpret_cast<const float4 *>(acc), row1 = *reinterpret_cast<const float4 *>(acc + 4);
    const float row8 = acc[8];
    const float4 acc0 = make_float4(row0.w, row1.x, row1.y, row1.z);  // mean2D.x, mean2D.y, conic.x, conic.y
    const float4 acc1 = make_float4(row1.w, row8, row0.x, row0.y);    // conic.w, opacity, color r, color g
    const float accb = row0.z;                                        // color b
    // the sums' per-Gaussian opacity factor: the caller's opacities (coalesced), else
    // the forward's splat record (4 B out of every 48)
    const float opac_in = in.opacities ? in.opacities[li] : a.splat_f[12 * (size_t)li + 5];
    const int32_t rad = a.radii[li];
    const uint32_t cl = a.clamped[li];
    static_assert(!LB || RWC == 48, "the basis-staged leaves are built for degree-3 rows");
    float rowv[DIRECT && !LB ? 48 : 1];
    auto load_row = [&](float *rowv) {  // launched only with staged (stage == true) SH rows: 16-B aligned cat rows, or split
        if constexpr (SPLIT) {
            load_sh_row_split(in.sh, in.sh_rest, (size_t)li, rowv);
        } else {
            const float4 *r4 = reinterpret_cast<const float4 *>(in.sh + (size_t)li * 48);
#pragma unroll
            for (int b = 0; b < 12; b++) {
                const float4 v = r4[b];
                rowv[4 * b] = v.x;
                rowv[4 * b + 1] = v.y;
                rowv[4 * b + 2] = v.z;
                rowv[4 * b + 3] = v.w;
            }
        }
    };
    if constexpr (!DIRECT) {
        if (stage && !jac) {
            if constexpr (SPLIT) {
                rows_to_lds_cols<PB_THREADS>(in.sh, g0, n, 3, 0, RW + 1, sh_lds);
                if (RW > 3) rows_to_lds_cols<PB_THREADS>(in.sh_rest, g0, n, RW - 3, 3, RW + 1, sh_lds);
            } else {
                rows_to_lds<PB_THREADS, RWC>(in.sh, g0, n, RW, sh_lds);
            }
        }
    }
    // the stored parameters' activations (gsr_inputs.activations), as the forward
    // applied them; qnorm = the rotation's norm for the normalize backward
    const float opac = (in.activations & GSR_ACT_OPACITY) && in.opacities ? act_sigmoid(opac_in) : opac_in;
    float qnorm = 0.f;
    if (!in.cov3D_precomp) {
        if (in.activations & GSR_ACT_SCALE)
#pragma unroll
            for (int k = 0; k < 3; k++) gin[k] = act_exp(gin[k]);
        if (in.activations & GSR_ACT_ROTATION) qnorm = act_normalize(gin + 3);
    }
    // pin the per-Gaussian loads ahead of the rows (the compiler would otherwise
    // sink them into the branch below, behind the rows, and wait for all of them)
    asm volatile("" ::"v"(acc0.x), "v"(acc0.y), "v"(acc0.z), "v"(acc0.w), "v"(acc1.x), "v"(acc1.y), "v"(acc1.z),
                 "v"(acc1.w), "v"(accb), "v"(opac), "v"(rad), "v"(cl));
    ShStage st{};
    if (live) st = preprocess_bwd_geom(a, idx, mean, gin, acc0, acc1, accb, opac, qnorm, rad, cl, V, Pm);
    float J[9];
    if (jac) {  // after the geometry, like the row (coalesced planes)
        if (live && st.vis)
#pragma unroll
            for (int k = 0; k < 9; k++) J[k] = a.shjac[(size_t)k * in.P + li];
    } else if constexpr (LB) {  // the row only to form J (its registers end here)
        if (live && st.vis) {
            float r[48];
            load_row(r);
            const float ox = mean.x - in.campos[0], oy = mean.y - in.campos[1], oz = mean.z - in.campos[2];
            const float len = sqrtf((ox * ox + oy * oy) + oz * oz);
            sh_dir_jacobian(r, in.D, ox / len, oy / len, oz / len, J);
        }
    } else if constexpr (DIRECT) {  // after the geometry (its registers are not held through it); culled: zeros
        if (live && st.vis) load_row(rowv);
    }
    if (stage && !DIRECT) __syncthreads();
    float b[LB ? 16 : 1];
    if (live) {
        f3 dmean = st.dmean;
        if constexpr (LB) {
            if (stage && st.vis) {
                const float ox = mean.x - in.campos[0], oy = mean.y - in.campos[1], oz = mean.z - in.campos[2];
                if (a.o.leaf.dsh_dc) sh_dir_basis(in.D, ox, oy, oz, b);
                sh_dir_term(J, ox, oy, oz, st.dRGB, dmean);
            }
        } else if (stage) {
            float *row = DIRECT ? rowv : sh_lds + threadIdx.x * (RW + 1);
            const float ox = mean.x - in.campos[0], oy = mean.y - in.campos[1], oz = mean.z - in.campos[2];
            if (!st.vis)
                for (int k = 0; k < RW; k++) row[k] = 0.f;
            else if (jac)
                sh_backward_j(J, row, in.D, DIRECT ? 16 : in.M, ox, oy, oz, st.dRGB, dmean);
            else
                sh_backward(row, row, in.D, DIRECT ? 16 : in.M, ox, oy, oz, st.dRGB, dmean);
        }
        float *dm = a.o.dmeans3D + 3 * (size_t)idx;
        if (a.o.leaf.accumulate & 16) {  // AccumulateGrad of the _xyz leaf: grad += new
            dm[0] += dmean.x;
            dm[1] += dmean.y;
            dm[2] += dmean.z;
        } else {
            store_stream<2>(dm, dmean.x);
            store_stream<2>(dm + 1, dmean.y);
            store_stream<2>(dm + 2, dmean.z);
        }
    }
    if constexpr (LB) {
        if (a.o.leaf.dsh_dc)
            leaf_sh_store_basis(a.o.leaf, in.P, idx, live, live && st.vis, (in.D + 1) * (in.D + 1), b, st.dRGB);
        return;
    } else if constexpr (DIRECT) {
        if (live && a.o.dsh) {
            if (a.o.dsh_planar) {
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (k < in.M)
#pragma unroll
                        for (int c = 0; c < 3; c++) a.o.dsh[(size_t)k * 3 * in.P + 3 * (size_t)idx + c] = rowv[3 * k + c];
            } else {
                float4 *d4 = reinterpret_cast<float4 *>(a.o.dsh + (size_t)idx * 48);
#pragma unroll
                for (int b = 0; b < 12; b++)
                    d4[b] = make_float4(rowv[4 * b], rowv[4 * b + 1], rowv[4 * b + 2], rowv[4 * b + 3]);
            }
        }
        if (a.o.leaf.dsh_dc) leaf_sh_store_direct(a.o.leaf, in.P, idx, live, rowv);
        return;
    }
    if (stage && a.o.dsh) {
        __syncthreads();
        if (a.o.dsh_planar)
            lds_to_planes<PB_THREADS>(sh_lds, g0, n, in.M, (size_t)3 * in.P, a.o.dsh);
        else
            lds_to_rows<PB_THREADS, RWC>(sh_lds, g0, n, RW, a.o.dsh);
    }
    if (stage && a.o.leaf.dsh_dc) {  // the two leaves of the caller's SH cat
        __syncthreads();
        const bool add = (a.o.leaf.accumulate & 1) != 0;
        lds_cols_to_rows<PB_THREADS>(sh_lds, RW + 1, 0, 3, g0, n, a.o.leaf.dsh_dc, add);
        if (RW > 3) lds_cols_to_rows<PB_THREADS>(sh_lds, RW + 1, 3, RW - 3, g0, n, a.o.leaf.dsh_rest, add);
    }
}

// F.normalize's backward as torch's autograd runs it for q = x / clamp_min(||x||,
// eps).expand_as(x) (DivBackward0, ExpandBackward0's sum, ClampMinBackward0,
// LinalgVectorNormBackward0 for ord 2, and the sum of the two paths into x),
// operation for operation: g = dL/dq, n_raw = ||x|| as torch computed it.  Every
// x / n and x / n_raw torch forms is the quotient q it already produced (the same
// division of the same operands; n = n_raw wherever the norm term is not masked),
// so the leaf x itself is not read.  File-wide fp contraction is off, as in
// torch's kernels.
__device__ __forceinline__ void normalize_backward(const float g[4], const float q[4], float n_raw, float eps,
                                                   float dx[4]) {
    const float n = n_raw != n_raw ? n_raw : fmaxf(n_raw, eps);  // clamp_min keeps a NaN
    float og[4];
#pragma unroll
    for (int k = 0; k < 4; k++) og[k] = -g[k] * (q[k] / n);  // -grad * ((self / other) / other)
    const float s = (og[0] + og[1]) + (og[2] + og[3]);  // sum_to_size over the expanded dim (torch's GPU
                                                        // reduction pairs the 4 terms; measured bit for bit)
    const float gm = n_raw >= eps ? s : 0.0f;                        // where(self >= min, grad, 0)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float xn = n_raw == 0.0f ? 0.0f : q[k];  // (self / norm).masked_fill_(norm == 0, 0)
        dx[k] = g[k] / n + gm * xn;
    }
}

// The activation gradients of one Gaussian (zeros for a culled one) go either to
// upstream's outputs or, where the caller asked for them (gsr_leaf_grads), through
// the activation's backward into its leaf's gradient.
// With an activation bit (gsr_inputs.activations) the input is the stored parameter:
// its gradient goes through the activation's backward into the leaf output if
// given, else into the plain one.
__device__ __forceinline__ void write_activation_grads(const PreBwdArgs &a, int idx, float dop, float opac,
                                                       const float ds[3], const float dq[4], const float gin[7],
                                                       float qnorm, bool has_sr) {
    const BwdOutputs &o = a.o;
    const gsr_leaf_grads &L = o.leaf;
    const int act = a.in.activations;
    auto put = [&](float *p, size_t i, float v, int bit) {
        if (L.accumulate & bit)
            p[i] += v;
        else
            store_stream<2>(p + i, v);
    };
    if (L.dopacity || (act & GSR_ACT_OPACITY)) {
        const float sg = opac;  // sigmoid(x): in.opacities[idx], or the activation of the logit
        const float v = (dop * (1.0f - sg)) * sg;  // sigmoid_backward: grad * (1 - y) * y
        if (L.dopacity)
            put(L.dopacity, idx, v, 4);
        else if (o.dopacity)
            o.dopacity[idx] = v;
    } else if (o.dopacity) {
        o.dopacity[idx] = dop;
    }
    if (!has_sr) {  // precomputed cov3D: upstream's zero-initialised dscales / drot
        if (o.dscales)
            for (int k = 0; k < 3; k++) o.dscales[3 * (size_t)idx + k] = 0.f;
        if (o.drot)
            for (int k = 0; k < 4; k++) o.drot[4 * (size_t)idx + k] = 0.f;
        return;
    }
    if (L.dscaling) {
#pragma unroll
        for (int k = 0; k < 3; k++) put(L.dscaling, 3 * (size_t)idx + k, ds[k] * gin[k], 2);  // exp: grad * result
    } else if (o.dscales) {
#pragma unroll
        for (int k = 0; k < 3; k++) o.dscales[3 * (size_t)idx + k] = (act & GSR_ACT_SCALE) ? ds[k] * gin[k] : ds[k];
    }
    if (L.drotation || (act & GSR_ACT_ROTATION)) {
        float dx[4];
        const bool own = (act & GSR_ACT_ROTATION) != 0;  // the norm this kernel computed, else torch's
        normalize_backward(dq, gin + 3, own ? qnorm : L.rotation_norm[idx], own ? ACT_ROTATION_EPS : L.rotation_eps,
                           dx);  // gin[3..6] = q
        float *dst = L.drotation ? L.drotation : o.drot;
        if (dst)
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (L.drotation)
                    put(dst, 4 * (size_t)idx + k, dx[k], 8);
                else
                    dst[4 * (size_t)idx + k] = dx[k];
            }
    } else if (o.drot) {
#pragma unroll
        for (int k = 0; k < 4; k++) o.drot[4 * (size_t)idx + k] = dq[k];
    }
}

__device__ ShStage preprocess_bwd_geom(const PreBwdArgs &a, int idx, const f3 mean, const float gin[7],
                                       const float4 acc0, const float4 acc1, float accb, float opac, float qnorm,
                                       int32_t rad, uint32_t cl, const Mat4 &V, const Mat4 &Pm) {
    const gsr_inputs &in = a.in;
    const BwdOutputs &o = a.o;
    const bool has_sr = in.scales != nullptr;
    ShStage st{};
    st.vis = rad > 0;
    if (!st.vis) {
        for (int k = 0; k < 3; k++) o.dmeans2D[3 * (size_t)idx + k] = 0.f;
        if (o.dcolors)
            for (int k = 0; k < 3; k++) o.dcolors[3 * (size_t)idx + k] = 0.f;
        if (o.drgb)
            for (int k = 0; k < 3; k++) o.drgb[3 * (size_t)idx + k] = 0.f;
        if (o.dcov3D)
            for (int k = 0; k < 6; k++) o.dcov3D[6 * (size_t)idx + k] = 0.f;
        const float zs[3] = {0.f, 0.f, 0.f}, zq[4] = {0.f, 0.f, 0.f, 0.f};
        write_activation_grads(a, idx, 0.f, opac, zs, zq, gin, qnorm, has_sr);
        return st;  // dmeans3D (st.dmean = 0) and the dsh row are written by the caller
    }
    const float dcol[3] = {acc1.z, acc1.w, accb};
    if (o.dcolors) {  // NULL: no precomputed colours to differentiate (the caller discards it)
        o.dcolors[3 * (size_t)idx + 0] = dcol[0];
        o.dcolors[3 * (size_t)idx + 1] = dcol[1];
        o.dcolors[3 * (size_t)idx + 2] = dcol[2];
    }

    // ---- 3D covariance (recomputed exactly as the forward did)
    float c3[6];
    float s[3] = {0, 0, 0}, q[4] = {0, 0, 0, 0};
    if (in.cov3D_precomp) {
        for (int k = 0; k < 6; k++) c3[k] = gin[k];
    } else {
        for (int k = 0; k < 3; k++) s[k] = gin[k];
        for (int k = 0; k < 4; k++) q[k] = gin[3 + k];
        compute_cov3d(s[0], s[1], s[2], in.scale_modifier, q[0], q[1], q[2], q[3], c3);
    }

    // ---- computeCov2DCUDA (backward.cu)
    f3 t = xform_point4x3(mean, V);
    const float h_x = a.focal_x, h_y = a.focal_y;
    const float limx = 1.3f * in.tan_fovx, limy = 1.3f * in.tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0.f : 1.f;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0.f : 1.f;
    const M3 J = m3_cols(h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z, -(h_y * t.y) / (t.z * t.z), 0,
                         0, 0);
    const float *v = V.m;
    const M3 W = m3_cols(v[0], v[4], v[8], v[1], v[5], v[9], v[2], v[6], v[10]);
    const M3 Vk = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    const M3 T = m3_mul(W, J);
    M3 cov2D = m3_mul(m3_mul(m3_transpose(T), m3_transpose(Vk)), T);
    const float ca = cov2D.m[0][0] += 0.3f;
    const float cb = cov2D.m[0][1];
    const float cc = cov2D.m[1][1] += 0.3f;
    // render_bwd.hip accumulates sum g5 (dx, dy) and sum g5 (dx^2, dx dy, dy^2) with
    // g5 = G dL/dalpha per pixel; the per-Gaussian factors — the opacity (W =
    // opacity g5), -conic/2 (the forward's conic, preprocess.hip) and (W, H) of
    // dL/dmean2D — are applied here
    const float sx = opac * acc0.x, sy = opac * acc0.y;
    const float gx = -0.5f * (opac * acc0.z), gy = -0.5f * (opac * acc0.w);  // dL/dconic x, y
    const float gz = -0.5f * (opac * acc1.x);                                // dL/dconic w
    const float denom = ca * cc - cb * cb;
    const float det_inv = 1.f / denom;
    const float kx = cc * det_inv, ky = -cb * det_inv, kz = ca * det_inv;
    const float g2x = -0.5f * (kx * sx + ky * sy) * (float)in.W;
    const float g2y = -0.5f * (ky * sx + kz * sy) * (float)in.H;
    store_stream<2>(o.dmeans2D + 3 * (size_t)idx + 0, g2x);
    store_stream<2>(o.dmeans2D + 3 * (size_t)idx + 1, g2y);
    store_stream<2>(o.dmeans2D + 3 * (size_t)idx + 2, 0.f);
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dc3[6] = {0, 0, 0, 0, 0, 0};
#define TT(i, j) T.m[i][j]
#define VV(i, j) Vk.m[i][j]
    if (denom2inv != 0) {
        dL_da = denom2inv * (-cc * cc * gx + 2 * cb * cc * gy + (denom - ca * cc) * gz);
        dL_dc = denom2inv * (-ca * ca * gz + 2 * ca * cb * gy + (denom - ca * cc) * gx);
        dL_db = denom2inv * 2 * (cb * cc * gx - (denom + 2 * cb * cb) * gy + ca * cb * gz);
        dc3[0] = (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc);
        dc3[3] = (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc);
        dc3[5] = (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc);
        dc3[1] = 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                 2 * TT(1, 0) * TT(1, 1) * dL_dc;
        dc3[2] = 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                 2 * TT(1, 0) * TT(1, 2) * dL_dc;
        dc3[4] = 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                 2 * TT(1, 1) * TT(1, 2) * dL_dc;
    }
    const float dL_dT00 = 2 * (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_da +
                          (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_db;
    const float dL_dT01 = 2 * (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_da +
                          (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_db;
    const float dL_dT02 = 2 * (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_da +
                          (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_db;
    const float dL_dT10 = 2 * (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_dc +
                          (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_db;
    const float dL_dT11 = 2 * (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_dc +
                          (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_db;
    const float dL_dT12 = 2 * (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_dc +
                          (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_db;
#undef TT
#undef VV
    const float dL_dJ00 = W.m[0][0] * dL_dT00 + W.m[0][1] * dL_dT01 + W.m[0][2] * dL_dT02;
    const float dL_dJ02 = W.m[2][0] * dL_dT00 + W.m[2][1] * dL_dT01 + W.m[2][2] * dL_dT02;
    const float dL_dJ11 = W.m[1][0] * dL_dT10 + W.m[1][1] * dL_dT11 + W.m[1][2] * dL_dT12;
    const float dL_dJ12 = W.m[2][0] * dL_dT10 + W.m[2][1] * dL_dT11 + W.m[2][2] * dL_dT12;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dL_dJ12;
    const float dL_dtz = -h_x * tz2 * dL_dJ00 - h_y * tz2 * dL_dJ11 + (2 * h_x * t.x) * tz3 * dL_dJ02 +
                         (2 * h_y * t.y) * tz3 * dL_dJ12;
    f3 dmean = xform_vec4x3_transpose(f3{dL_dtx, dL_dty, dL_dtz}, V);
    if (o.dcov3D)  // NULL: no precomputed cov3D to differentiate
        for (int k = 0; k < 6; k++) o.dcov3D[6 * (size_t)idx + k] = dc3[k];

    // ---- preprocessCUDA (backward.cu): 2D-mean gradient through the projection
    const f4 m_hom = xform_point4x4(mean, Pm);
    const float m_w = 1.0f / (m_hom.w + 0.0000001f);
    const float *pm = Pm.m;
    const float mul1 = (pm[0] * mean.x + pm[4] * mean.y + pm[8] * mean.z + pm[12]) * m_w * m_w;
    const float mul2 = (pm[1] * mean.x + pm[5] * mean.y + pm[9] * mean.z + pm[13]) * m_w * m_w;
    dmean.x += (pm[0] * m_w - pm[3] * mul1) * g2x + (pm[1] * m_w - pm[3] * mul2) * g2y;
    dmean.y += (pm[4] * m_w - pm[7] * mul1) * g2x + (pm[5] * m_w - pm[7] * mul2) * g2y;
    dmean.z += (pm[8] * m_w - pm[11] * mul1) * g2x + (pm[9] * m_w - pm[11] * mul2) * g2y;

    // ---- SH backward (colour gradient masked where the forward clamped): the caller
    // runs it once the row is in LDS, and writes dmeans3D
    {
        st.dRGB[0] = dcol[0] * ((cl & 1) ? 0.f : 1.f);
        st.dRGB[1] = dcol[1] * ((cl & 2) ? 0.f : 1.f);
        st.dRGB[2] = dcol[2] * ((cl & 4) ? 0.f : 1.f);
        if (o.drgb)
            for (int k = 0; k < 3; k++) o.drgb[3 * (size_t)idx + k] = st.dRGB[k];
    }
    st.dmean = dmean;

    // ---- computeCov3D backward: dSigma -> dM = 2 M dSigma -> dscale, drot (q as given)
    float ds[3] = {0.f, 0.f, 0.f}, dq[4] = {0.f, 0.f, 0.f, 0.f};
    if (has_sr) {
        const float qr = q[0], qx = q[1], qy = q[2], qz = q[3];
        const M3 R = quat_to_rot(qr, qx, qy, qz);
        M3 S = m3_cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
        const float sm[3] = {in.scale_modifier * s[0], in.scale_modifier * s[1], in.scale_modifier * s[2]};
        S.m[0][0] = sm[0];
        S.m[1][1] = sm[1];
        S.m[2][2] = sm[2];
        const M3 Mm = m3_mul(S, R);
        const float *d = dc3;
        const M3 dSig = m3_cols(d[0], 0.5f * d[1], 0.5f * d[2], 0.5f * d[1], d[3], 0.5f * d[4], 0.5f * d[2],
                                0.5f * d[4], d[5]);
        M3 twoM;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) twoM.m[i][j] = 2.0f * Mm.m[i][j];
        const M3 dM = m3_mul(twoM, dSig);
        const M3 Rt = m3_transpose(R);
        M3 dMt = m3_transpose(dM);
        for (int k = 0; k < 3; k++)
            ds[k] = (Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1]) + Rt.m[k][2] * dMt.m[k][2];
        for (int k = 0; k < 3; k++)
            for (int j = 0; j < 3; j++) dMt.m[k][j] *= sm[k];
#define D(i, j) dMt.m[i][j]
        dq[0] = 2 * qz * (D(0, 1) - D(1, 0)) + 2 * qy * (D(2, 0) - D(0, 2)) + 2 * qx * (D(1, 2) - D(2, 1));
        dq[1] = 2 * qy * (D(1, 0) + D(0, 1)) + 2 * qz * (D(2, 0) + D(0, 2)) + 2 * qr * (D(1, 2) - D(2, 1)) -
                4 * qx * (D(2, 2) + D(1, 1));
        dq[2] = 2 * qx * (D(1, 0) + D(0, 1)) + 2 * qr * (D(2, 0) - D(0, 2)) + 2 * qz * (D(1, 2) + D(2, 1)) -
                4 * qy * (D(2, 2) + D(0, 0));
        dq[3] = 2 * qr * (D(0, 1) - D(1, 0)) + 2 * qx * (D(2, 0) + D(0, 2)) + 2 * qy * (D(1, 2) + D(2, 1)) -
                4 * qz * (D(1, 1) + D(0, 0));
#undef D
    }
    write_activation_grads(a, idx, acc1.y, opac, ds, dq, gin, qnorm, has_sr);
    return st;
}

hipError_t launch_preprocess_bwd(const gsr_inputs &in, const int32_t *radii, const void *geom, const float *accum,
                                 const BwdOutputs &o, hipStream_t s) {
    const GeomLayout G = geom_layout(in.P, in.W, in.H);
    PreBwdArgs a;
    a.in = in;
    a.focal_y = in.H / (2.0f * in.tan_fovy);
    a.focal_x = in.W / (2.0f * in.tan_fovx);
    a.radii = radii;
    a.clamped = at<uint8_t>(geom, G.off[GSR_GEOM_CLAMPED]);
    a.splat_f = at<float>(geom, G.off[GSR_GEOM_SPLATS]);
    a.accum = accum;
    a.shjac = at<float>(geom, G.shjac);
    a.ctrl = at<uint32_t>(geom, G.off[GSR_GEOM_CTRL]);
    a.o = o;
    const bool stage = in.sh && (o.dsh || o.drgb || o.sh_dir || o.leaf.dsh_dc) && in.M > 0;
    const bool split = in.sh_rest != nullptr;
    const bool direct = stage && 3 * in.M == 48 && (split || ((uintptr_t)in.sh & 15u) == 0) &&
                        (!a.o.dsh || a.o.dsh_planar || ((uintptr_t)a.o.dsh & 15u) == 0) &&
                        (!o.leaf.dsh_dc || ((uintptr_t)o.leaf.dsh_rest & 15u) == 0);
    const size_t lds = stage && !direct ? (size_t)PB_THREADS * (3 * in.M + 1) * sizeof(float) : 0;
    const dim3 grid((in.P + PB_THREADS - 1) / PB_THREADS);
    // see launch_preprocess; the direct-row kernel needs staged rows (cat rows 16-B aligned)
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(PB_THREADS), lds, s, a); };
    if (3 * in.M == 3)  // (M = 1 has no rest coefficients: never split)
        go(preprocess_bwd_kernel<3, false>);
    else if (3 * in.M == 48 && direct && !o.dsh)  // the leaves or the colour gradient: no dsh row
        split ? go(preprocess_bwd_kernel<48, true, true>) : go(preprocess_bwd_kernel<48, false, true>);
    else if (3 * in.M == 48 && direct)
        split ? go(preprocess_bwd_kernel<48, true>) : go(preprocess_bwd_kernel<48, false>);
    else
        split ? go(preprocess_bwd_kernel<0, true>) : go(preprocess_bwd_kernel<0, false>);
    return hipGetLastError();
}

}  // namespace gsr

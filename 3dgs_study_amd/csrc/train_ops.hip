// train_ops.hip — the training-step ops right after the rasterizer (SURVEY.md
// §8f "next" rows 1-2): the fused L1 + D-SSIM loss with its gradient, the Adam
// update of the six parameter groups, and the densification statistics.
//
// Reference: utils/loss_utils.py:17-24 (l1_loss), :59-108 (ssim/_ssim: 11x11
// Gaussian window, sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2, mean over
// C*H*W); train.py:103-105 (loss = (1 - l) L1 + l (1 - SSIM)), :126-141
// (max_radii2D, add_densification_stats, optimizer.step); scene/gaussian_model.py
// :176-213 (Adam, eps 1e-15), :565-581 (densification statistics);
// torch.optim.Adam's update rule (betas 0.9/0.999, bias-corrected).
#include <cmath>

#include "gsr_kernels.hpp"
#include "gsr_l1.hpp"
#include "gsr_wave.hpp"

namespace gsr {

// ------------------------------------------------------------ L1 + D-SSIM
//
// loss = (1 - l)/N sum |x - y| + l (1 - 1/N sum S), N = C*H*W.  The gradient of
// the mean SSIM w.r.t. x needs only constants from the loss (dL/dS = -l/N), so
// ONE pass computes both: per pixel q, with m1 = G*x, m2 = G*y, e11 = G*(x^2),
// e22 = G*(y^2), e12 = G*(xy) (G the separable 11-tap window) and
//   S = A1 A2 / (B1 B2),  A1 = 2 m1 m2 + C1,  A2 = 2 (e12 - m1 m2) + C2,
//                         B1 = m1^2 + m2^2 + C1,  B2 = e11 - m1^2 + e22 - m2^2 + C2,
//   dS/dm1 = S (2 m2/A1 - 2 m2/A2 - 2 m1/B1 + 2 m1/B2),  dS/de11 = -S/B2,
//   dS/de12 = 2 S/A2,
// and dL/dx(p) = (1-l)/N sign(x-y) + G*(dL/dS dS/dm1) + 2 x G*(dL/dS dS/de11)
//              + y G*(dL/dS dS/de12)   (G symmetric: correlation == convolution).
// A workgroup owns a 32x32 output tile of one channel and runs four separable
// passes through LDS, each register-blocked so that a thread reuses the values it
// reads: (1) the horizontal 11-tap sums of the five products (x, y, x^2, y^2, xy)
// over the input rows, 3 map columns per thread; (2) the vertical sums, 7 map rows
// per thread, then the SSIM terms and the three derivative maps; (3) and (4) the
// derivative maps blurred back onto the tile the same way, 4 and 2 outputs per thread,
// with the L1 term and the gradient.  512-thread workgroups: the LDS (65 KB)
// allows two per CU, i.e. 4 waves per SIMD.  3x1080x1920: 134 us (round 1 read
// one LDS operand per tap: 295 us, LDS-bound).
constexpr int SS_T = 32, SS_R = 5;           // tile (square), window radius
constexpr int SS_I = SS_T + 4 * SS_R;        // input region 52 x 52
constexpr int SS_M = SS_T + 2 * SS_R;        // map region 42 x 42
constexpr int SS_TX = SS_T, SS_TY = SS_T;
constexpr int SS_THREADS = 512;  // 8 waves: 2 workgroups (16 waves) per CU within the LDS
// outputs per thread in passes 1-4 (swept at 3x1080x1920: pass 1/2 blocking of
// (6, 6) 158 us, (3, 3) 140, (3, 7) 134, (7, 3) 142, (2, 2) 155)
constexpr int SS_B1 = 3, SS_B2 = 7, SS_B3 = 4, SS_B4 = 2;
static_assert(SS_M % SS_B1 == 0 && SS_M % SS_B2 == 0 && SS_T % SS_B3 == 0 && SS_T % SS_B4 == 0, "blocking");

struct SsimArgs {
    const float *x, *y;
    float *grad;      // [C][H][W]
    float *partials;  // [blocks][2] sum |x - y|, sum S over the tile's pixels
    int C, H, W, tiles_x, tiles_y;
    float lambda, invN;
    float g[11];      // 1-D window (utils/loss_utils.py gaussian(11, 1.5), normalized)
};

__global__ void __launch_bounds__(SS_THREADS) l1_ssim_kernel(SsimArgs a) {
    // xy: the inputs (passes 1), then the derivative maps (passes 2-3);
    // hb: the horizontal sums (passes 1-2), then the blurred-back rows (3-4)
    __shared__ float xy[2 * SS_I * SS_I > 3 * SS_M * SS_M ? 2 * SS_I * SS_I : 3 * SS_M * SS_M];
    __shared__ float hb[5][SS_I][SS_M];
    __shared__ float red[2][SS_THREADS / 64];
    float(*xs)[SS_I] = reinterpret_cast<float(*)[SS_I]>(xy);
    float(*ys)[SS_I] = reinterpret_cast<float(*)[SS_I]>(xy + SS_I * SS_I);
    float(*dm)[SS_M][SS_M] = reinterpret_cast<float(*)[SS_M][SS_M]>(xy);
    const int c = blockIdx.z;
    const int ox = blockIdx.x * SS_T, oy = blockIdx.y * SS_T;
    const size_t plane = (size_t)a.H * a.W;
    const float *X = a.x + c * plane, *Y = a.y + c * plane;
    const int t = threadIdx.x;
    float gw[11];
#pragma unroll
    for (int k = 0; k < 11; k++) gw[k] = a.g[k];
    // inputs over the tile +- 2R, zero outside the image (conv2d zero padding)
    for (int i = t; i < SS_I * SS_I; i += SS_THREADS) {
        const int ry = i / SS_I, rx = i - ry * SS_I;
        const int gy = oy - 2 * SS_R + ry, gx = ox - 2 * SS_R + rx;
        const bool in = gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
        xs[ry][rx] = in ? X[(size_t)gy * a.W + gx] : 0.f;
        ys[ry][rx] = in ? Y[(size_t)gy * a.W + gx] : 0.f;
    }
    __syncthreads();
    // (1) horizontal sums over every input row, map columns [c0, c0 + B1)
    for (int item = t; item < SS_I * (SS_M / SS_B1); item += SS_THREADS) {
        const int row = item / (SS_M / SS_B1), c0 = (item - row * (SS_M / SS_B1)) * SS_B1;
        float xv[SS_B1 + 10], yv[SS_B1 + 10];
#pragma unroll
        for (int k = 0; k < SS_B1 + 10; k++) {
            xv[k] = xs[row][c0 + k];
            yv[k] = ys[row][c0 + k];
        }
#pragma unroll
        for (int o = 0; o < SS_B1; o++) {
            float s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0;
#pragma unroll
            for (int k = 0; k < 11; k++) {
                const float u = xv[o + k], v = yv[o + k], w = gw[k];
                s0 += w * u;
                s1 += w * v;
                s2 += w * (u * u);
                s3 += w * (v * v);
                s4 += w * (u * v);
            }
            hb[0][row][c0 + o] = s0;
            hb[1][row][c0 + o] = s1;
            hb[2][row][c0 + o] = s2;
            hb[3][row][c0 + o] = s3;
            hb[4][row][c0 + o] = s4;
        }
    }
    __syncthreads();
    // (2) vertical sums -> maps over the tile +- R, map rows [r0, r0 + B2) of a
    // column; then the per-pixel SSIM terms and the derivative maps (over xs/ys)
    const float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;
    const float dLdS = -a.lambda * a.invN;
    float ssum = 0.f;
    for (int item = t; item < SS_M * (SS_M / SS_B2); item += SS_THREADS) {
        const int col = item % SS_M, r0 = (item / SS_M) * SS_B2;
        float m[SS_B2][5];
#pragma unroll
        for (int o = 0; o < SS_B2; o++)
#pragma unroll
            for (int q = 0; q < 5; q++) m[o][q] = 0.f;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            float hv[SS_B2 + 10];
#pragma unroll
            for (int k = 0; k < SS_B2 + 10; k++) hv[k] = hb[q][r0 + k][col];
#pragma unroll
            for (int o = 0; o < SS_B2; o++)
#pragma unroll
                for (int k = 0; k < 11; k++) m[o][q] += gw[k] * hv[o + k];
        }
#pragma unroll
        for (int o = 0; o < SS_B2; o++) {
            const int my = r0 + o;
            const int gy = oy - SS_R + my, gx = ox - SS_R + col;
            const bool in = gy >= 0 && gy < a.H && gx >= 0 && gx < a.W;
            const float m1 = m[o][0], m2 = m[o][1];
            const float m1m2 = m1 * m2, m1s = m1 * m1, m2s = m2 * m2;
            const float s1 = m[o][2] - m1s, s2 = m[o][3] - m2s, s12 = m[o][4] - m1m2;
            const float A1 = 2 * m1m2 + C1, A2 = 2 * s12 + C2, B1 = m1s + m2s + C1, B2 = s1 + s2 + C2;
            // four hardware reciprocals (1 ulp) instead of seven IEEE divisions
            const float iA1 = __builtin_amdgcn_rcpf(A1), iA2 = __builtin_amdgcn_rcpf(A2);
            const float iB1 = __builtin_amdgcn_rcpf(B1), iB2 = __builtin_amdgcn_rcpf(B2);
            const float S = (A1 * A2) * (iB1 * iB2);
            const bool own = in && my >= SS_R && my < SS_R + SS_T && col >= SS_R && col < SS_R + SS_T;
            ssum += own ? S : 0.f;
            // derivative maps (zero outside the image: those S do not exist); written
            // after every thread's pass-1 use of xs / ys (the barrier above)
            const float k1 = in ? dLdS * S : 0.f;
            dm[0][my][col] = k1 * (2 * m2 * (iA1 - iA2) + 2 * m1 * (iB2 - iB1));
            dm[1][my][col] = -k1 * iB2;
            dm[2][my][col] = 2 * k1 * iA2;
        }
    }
    __syncthreads();
    // (3) horizontal blur of the derivative maps onto the tile columns [c0, c0 + B3)
    for (int item = t; item < SS_M * (SS_T / SS_B3); item += SS_THREADS) {
        const int row = item / (SS_T / SS_B3), c0 = (item - row * (SS_T / SS_B3)) * SS_B3;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            float dv[SS_B3 + 10];
#pragma unroll
            for (int k = 0; k < SS_B3 + 10; k++) dv[k] = dm[q][row][c0 + k];
#pragma unroll
            for (int o = 0; o < SS_B3; o++) {
                float sacc = 0.f;
#pragma unroll
                for (int k = 0; k < 11; k++) sacc += gw[k] * dv[o + k];
                hb[q][row][c0 + o] = sacc;
            }
        }
    }
    __syncthreads();
    // (4) vertical blur onto the tile rows [r0, r0 + B4) of a column; L1 term; gradient
    float l1sum = 0.f;
    {
        const int col = t % SS_T, r0 = (t / SS_T) * SS_B4;
        float b[SS_B4][3];
#pragma unroll
        for (int q = 0; q < 3; q++) {
            float hv[SS_B4 + 10];
#pragma unroll
            for (int k = 0; k < SS_B4 + 10; k++) hv[k] = hb[q][r0 + k][col];
#pragma unroll
            for (int o = 0; o < SS_B4; o++) {
                float sacc = 0.f;
#pragma unroll
                for (int k = 0; k < 11; k++) sacc += gw[k] * hv[o + k];
                b[o][q] = sacc;
            }
        }
        const float kl1 = (1.f - a.lambda) * a.invN;
        float *G = a.grad + c * plane;
        const int gx = ox + col;
#pragma unroll
        for (int o = 0; o < SS_B4; o++) {
            const int gy = oy + r0 + o;
            if (gy < a.H && gx < a.W) {
                const size_t pix = (size_t)gy * a.W + gx;
                const float xv = X[pix], yv = Y[pix];
                const float d = xv - yv;
                l1sum += fabsf(d);
                const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch.sign
                G[pix] = kl1 * sg + b[o][0] + 2.f * xv * b[o][1] + yv * b[o][2];
            }
        }
    }
    static_assert(SS_T * (SS_T / SS_B4) == SS_THREADS, "pass 4: one item per thread");
    // workgroup partial sums (the loss value itself is finished by l1_ssim_finish)
    const float l1w = wave_sum(l1sum), ssw = wave_sum(ssum);
    if ((t & 63) == 0) {
        red[0][t >> 6] = l1w;
        red[1][t >> 6] = ssw;
    }
    __syncthreads();
    if (t == 0) {
        float s0 = 0, s1 = 0;
        for (int k = 0; k < SS_THREADS / 64; k++) {
            s0 += red[0][k];
            s1 += red[1][k];
        }
        const size_t blk = ((size_t)c * a.tiles_y + blockIdx.y) * a.tiles_x + blockIdx.x;
        a.partials[2 * blk] = s0;
        a.partials[2 * blk + 1] = s1;
    }
}

// loss = (1 - l) * mean|x - y| + l * (1 - mean S), summed in double for a
// deterministic, order-independent-enough total
__global__ void __launch_bounds__(1024) l1_ssim_finish_kernel(const float *partials, int nb, float lambda,
                                                              float invN, float *out) {
    __shared__ double s[2][1024 / 64];
    double l1 = 0, ss = 0;
    for (int i = threadIdx.x; i < nb; i += 1024) {
        l1 += partials[2 * i];
        ss += partials[2 * i + 1];
    }
    for (int o = 32; o >= 1; o >>= 1) {
        l1 += __shfl_xor(l1, o);
        ss += __shfl_xor(ss, o);
    }
    if ((threadIdx.x & 63) == 0) {
        s[0][threadIdx.x >> 6] = l1;
        s[1][threadIdx.x >> 6] = ss;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0, b = 0;
        for (int k = 0; k < 1024 / 64; k++) {
            a += s[0][k];
            b += s[1][k];
        }
        out[0] = (float)((1.0 - lambda) * a * invN + lambda * (1.0 - b * invN));
        out[1] = (float)(a * invN);  // the L1 term alone (train.py logs it)
        out[2] = (float)(b * invN);  // mean SSIM
    }
}

// lambda == 0 (the headline unit's loss, train.py:102 with lambda_dssim = 0): only
// mean |x - y| (l1_kernel, one streaming read of x and y; the window sums of the
// SSIM kernel would cost 10x the time for a zero term), and in the backward its
// gradient (l1_grad_kernel): torch's MeanBackward then AbsBackward, (dloss / N) *
// sign(x - y), bit for bit, with the incoming dloss read on the device — no
// gradient map is written in the forward and scaled again in the backward.
// Per workgroup one partial sum for l1_ssim_finish_kernel.
// (L1_THREADS, L1_BLOCKS, l1_blocks and the block body: gsr_l1.hpp)
__global__ void __launch_bounds__(L1_THREADS) l1_kernel(const float *x, const float *y, size_t n, float *partials) {
    l1_block_partial(x, y, n, blockIdx.x, gridDim.x, partials);
}

__device__ __forceinline__ float sign_f(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }
__global__ void __launch_bounds__(L1_THREADS) l1_grad_kernel(const float *x, const float *y, size_t n, float fN,
                                                             const float *dloss, float *g) {
    const float q = dloss[0] / fN;  // MeanBackward: grad / numel
    const size_t n4 = n >> 2, stride = (size_t)gridDim.x * L1_THREADS;
    const float4 *x4 = reinterpret_cast<const float4 *>(x), *y4 = reinterpret_cast<const float4 *>(y);
    float4 *g4 = reinterpret_cast<float4 *>(g);
    for (size_t i = (size_t)blockIdx.x * L1_THREADS + threadIdx.x; i < n4; i += stride) {
        const float4 a = x4[i], b = y4[i];  // AbsBackward: grad * sgn(self)
        g4[i] = make_float4(q * sign_f(a.x - b.x), q * sign_f(a.y - b.y), q * sign_f(a.z - b.z), q * sign_f(a.w - b.w));
    }
    if (blockIdx.x == 0)
        for (size_t i = (n4 << 2) + threadIdx.x; i < n; i += L1_THREADS) g[i] = q * sign_f(x[i] - y[i]);
}


// The L1 loss from partial sums [nb][2] already in partials (bwd_prepare_kernel's,
// gsr_forward_render_l1), or, with from_xy, from x and y (l1_kernel into partials:
// room for 2 L1_BLOCKS floats).  out: gsr_l1_ssim's [3] (loss, L1 term, 0).
hipError_t launch_l1_finish(const float *x, const float *y, size_t n, float *partials, int nb, bool from_xy,
                            float *out, hipStream_t s) {
    const float invN = 1.0f / (float)(double)n;  // launch_l1_ssim's invN for C H W = n
    if (from_xy) {
        nb = l1_blocks(n);
        hipLaunchKernelGGL(l1_kernel, dim3(nb), dim3(L1_THREADS), 0, s, x, y, n, partials);
    }
    hipLaunchKernelGGL(l1_ssim_finish_kernel, dim3(1), dim3(1024), 0, s, (const float *)partials, nb, 0.0f, invN, out);
    return hipGetLastError();
}

hipError_t launch_l1_grad(const float *x, const float *y, size_t n, const float *dloss, float *grad, hipStream_t s) {
    hipLaunchKernelGGL(l1_grad_kernel, dim3(l1_blocks(n)), dim3(L1_THREADS), 0, s, x, y, n, (float)(double)n, dloss,
                       grad);
    return hipGetLastError();
}

size_t l1_ssim_scratch_floats(int C, int H, int W) {
    const size_t tx = (W + SS_TX - 1) / SS_TX, ty = (H + SS_TY - 1) / SS_TY;
    return 2 * (tx * ty * C > (size_t)L1_BLOCKS ? tx * ty * C : (size_t)L1_BLOCKS);
}

hipError_t launch_l1_ssim(const float *x, const float *y, int C, int H, int W, float lambda, float *grad,
                          float *partials, float *out, hipStream_t s) {
    SsimArgs a;
    a.x = x;
    a.y = y;
    a.grad = grad;
    a.partials = partials;
    a.C = C;
    a.H = H;
    a.W = W;
    a.tiles_x = (W + SS_TX - 1) / SS_TX;
    a.tiles_y = (H + SS_TY - 1) / SS_TY;
    a.lambda = lambda;
    a.invN = 1.0f / (float)((double)C * H * W);  // torch's MeanBackward: grad / numel in float
    if (lambda == 0.0f && grad == nullptr) {  // the loss alone (its gradient: launch_l1_grad)
        const size_t n = (size_t)C * H * W;
        const int nb = l1_blocks(n);
        hipLaunchKernelGGL(l1_kernel, dim3(nb), dim3(L1_THREADS), 0, s, x, y, n, partials);
        hipLaunchKernelGGL(l1_ssim_finish_kernel, dim3(1), dim3(1024), 0, s, (const float *)partials, nb, lambda,
                           a.invN, out);
        return hipGetLastError();
    }
    // gaussian(11, 1.5) as utils/loss_utils.py builds it: float32 taps, normalized in float32
    float sum = 0.f;
    for (int k = 0; k < 11; k++) {
        a.g[k] = (float)std::exp(-(double)((k - 5) * (k - 5)) / (2.0 * 1.5 * 1.5));
        sum += a.g[k];
    }
    for (int k = 0; k < 11; k++) a.g[k] /= sum;
    hipLaunchKernelGGL(l1_ssim_kernel, dim3(a.tiles_x, a.tiles_y, C), dim3(SS_THREADS), 0, s, a);
    const int nb = a.tiles_x * a.tiles_y * C;
    hipLaunchKernelGGL(l1_ssim_finish_kernel, dim3(1), dim3(1024), 0, s, (const float *)partials, nb, lambda, a.invN,
                       out);
    return hipGetLastError();
}

// ------------------------------------------------------------ Adam
//
// torch.optim.Adam (no weight decay, no amsgrad), for up to 8 tensors in one
// launch.  Workgroups are assigned to segments by a prefix table, each thread
// updates 4 consecutive floats (16-B accesses).
constexpr int ADAM_THREADS = 256, ADAM_VEC = 4;
struct AdamArgs {
    int nseg;
    float *p[GSR_ADAM_MAX_SEGS];
    const float *g[GSR_ADAM_MAX_SEGS];
    float *m[GSR_ADAM_MAX_SEGS];
    float *v[GSR_ADAM_MAX_SEGS];
    int64_t n[GSR_ADAM_MAX_SEGS];
    float neg_step[GSR_ADAM_MAX_SEGS];  // -lr / (1 - beta1^t)
    float bc2s[GSR_ADAM_MAX_SEGS];      // sqrt(1 - beta2^t)
    int block0[GSR_ADAM_MAX_SEGS + 1];  // first workgroup of each segment
    float w1, beta2, w2, eps;           // w1 = 1 - beta1, w2 = 1 - beta2
};

// torch's foreach Adam, op for op: exp_avg.lerp_(grad, 1 - beta1) (weight < 0.5
// form), exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2),
// denom = sqrt(exp_avg_sq) / sqrt(bias_correction2) + eps,
// param.addcdiv_(exp_avg, denom, -lr / bias_correction1)
__device__ __forceinline__ void adam_one(float &p, float g, float &m, float &v, float w1, float b2, float w2, float eps,
                                         float neg_step, float bc2s) {
    m = m + w1 * (g - m);
    v = v * b2;
    v = v + w2 * (g * g);
    const float denom = sqrtf(v) / bc2s + eps;
    p = p + neg_step * (m / denom);
}

__global__ void __launch_bounds__(ADAM_THREADS) adam_kernel(AdamArgs a) {
    int s = 0;
    while (s + 1 < a.nseg && (int)blockIdx.x >= a.block0[s + 1]) s++;
    const int64_t i0 = ((int64_t)(blockIdx.x - a.block0[s]) * ADAM_THREADS + threadIdx.x) * ADAM_VEC;
    const int64_t n = a.n[s];
    if (i0 >= n) return;
    float *p = a.p[s], *m = a.m[s], *v = a.v[s];
    const float *g = a.g[s];
    const float w1 = a.w1, b2 = a.beta2, w2 = a.w2, eps = a.eps, ns = a.neg_step[s], bc = a.bc2s[s];
    const bool vec = i0 + ADAM_VEC <= n && ((((uintptr_t)(p + i0)) | ((uintptr_t)(g + i0)) | ((uintptr_t)(m + i0)) |
                                            ((uintptr_t)(v + i0))) & 15u) == 0;
    if (vec) {
        float4 P = *reinterpret_cast<float4 *>(p + i0), G = *reinterpret_cast<const float4 *>(g + i0);
        float4 M = *reinterpret_cast<float4 *>(m + i0), V = *reinterpret_cast<float4 *>(v + i0);
        adam_one(P.x, G.x, M.x, V.x, w1, b2, w2, eps, ns, bc);
        adam_one(P.y, G.y, M.y, V.y, w1, b2, w2, eps, ns, bc);
        adam_one(P.z, G.z, M.z, V.z, w1, b2, w2, eps, ns, bc);
        adam_one(P.w, G.w, M.w, V.w, w1, b2, w2, eps, ns, bc);
        *reinterpret_cast<float4 *>(p + i0) = P;
        *reinterpret_cast<float4 *>(m + i0) = M;
        *reinterpret_cast<float4 *>(v + i0) = V;
    } else {
        for (int64_t i = i0; i < n && i < i0 + ADAM_VEC; i++) adam_one(p[i], g[i], m[i], v[i], w1, b2, w2, eps, ns, bc);
    }
}

hipError_t launch_adam(const gsr_adam_segment *segs, int nseg, int step, double beta1, double beta2, double eps,
                       hipStream_t s) {
    AdamArgs a;
    a.nseg = nseg;
    // Python-side scalars as torch forms them (double math, then float)
    a.w1 = (float)(1.0 - beta1);
    a.beta2 = (float)beta2;
    a.w2 = (float)(1.0 - beta2);
    a.eps = (float)eps;
    const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
    int blocks = 0;
    for (int k = 0; k < nseg; k++) {
        a.p[k] = segs[k].param;
        a.g[k] = segs[k].grad;
        a.m[k] = segs[k].exp_avg;
        a.v[k] = segs[k].exp_avg_sq;
        a.n[k] = segs[k].n;
        a.neg_step[k] = (float)(-(segs[k].lr / bc1));
        a.bc2s[k] = (float)std::sqrt(bc2);
        a.block0[k] = blocks;
        blocks += (int)((segs[k].n + (int64_t)ADAM_THREADS * ADAM_VEC - 1) / ((int64_t)ADAM_THREADS * ADAM_VEC));
    }
    a.block0[nseg] = blocks;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(ADAM_THREADS), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------ densification statistics
// max_radii2D[v] = max(max_radii2D[v], radii[v]); xyz_gradient_accum[v] += |dmean2D[v, :2]|;
// denom[v] += 1, for v with radii > 0 (train.py:126-127, gaussian_model.py:565-581)
__global__ void densify_stats_kernel(int P, const int32_t *radii, const float *vgrad, int vstride, float *max_radii,
                                     float *grad_accum, float *denom) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    max_radii[i] = fmaxf(max_radii[i], (float)r);
    const float gx = vgrad[(size_t)i * vstride], gy = vgrad[(size_t)i * vstride + 1];
    grad_accum[i] += sqrtf(gx * gx + gy * gy);
    denom[i] += 1.f;
}

hipError_t launch_densify_stats(int P, const int32_t *radii, const float *vgrad, int vstride, float *max_radii,
                                float *grad_accum, float *denom, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, vgrad, vstride,
                       max_radii, grad_accum, denom);
    return hipGetLastError();
}

}  // namespace gsr

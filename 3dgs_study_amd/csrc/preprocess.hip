// preprocess.hip — forward per-Gaussian stage and the tile-count scan.
//
// Replaces upstream FORWARD::preprocessCUDA (forward.cu) and the
// cub::DeviceScan::InclusiveSum of Rasterizer::forward (rasterizer_impl.cu),
// SURVEY.md §8a rows a9/a10 and Appendix A.2-A.4.  One thread per Gaussian;
// the per-block sums of tiles_touched are produced in the same pass so the
// scan costs one extra small launch (block prefixes) plus a down-sweep.
//
// No floating-point contraction in this file: radii and tile rects must match
// the oracle (oracle/gsr_oracle.c, built with -ffp-contract=off) bit for bit.
#pragma clang fp contract(off)

#include "gsr_blend.hpp"
#include "gsr_colour.hpp"
#include "gsr_kernels.hpp"
#include "gsr_math.hpp"
#include "gsr_publish.hpp"
#include "gsr_rows.hpp"
#include "gsr_spans.hpp"
#include "gsr_wave.hpp"

namespace gsr {

struct PreArgs {
    gsr_inputs in;
    float focal_x, focal_y;
    int gx, gy;
    float *depths;
    float2 *means2D;
    float4 *splats;  // [P][3]
    uint8_t *clamped;
    uint32_t *tiles_touched;
    uint4 *rects;  // tile rect {x0 | x1 << 16, y0 | y1 << 16} + 64-bit tile mask per Gaussian (binning.hip)
    uint32_t *rwords;  // instead (the row-span binning of the rect footprint): the rect as one word (gsr_spans.hpp)
    uint2 *ranges;           // [T] zeroed here (empty tiles keep (0, 0); binning.hip fills the rest)
    int tiles;
    uint4 *block_sums;       // [pre_blocks(P)] {instances | prefiltered error << 31, smallest, largest candidate depth key, 0}
    int32_t *radii;
    uint32_t *order_cnt;
    uint32_t *sup0;   // the grouped first depth pass's group counts (binning.hip), zeroed here, or NULL
    int sup0_n;
    float *shjac;     // [9][P] the SH direction Jacobian, when a backward will follow (else NULL)
    uint32_t *ctrl;   // geom control words (CTRL_SHJAC)
};

// SPLIT: the SH rows come from GaussianModel's two leaves (gsr_inputs.sh_rest)
// instead of their cat.  GEOM: everything but the colour (no SH rows read; the
// splat records' colour words left 0, clamped and the Jacobian unwritten) —
// preprocess_colour_kernel fills those on a side stream while the binning runs.
template <int RWC, bool SPLIT, bool GEOM = false>
__global__ void __launch_bounds__(PRE_THREADS) preprocess_fwd_kernel(PreArgs a) {
    __shared__ uint32_t wsum[PRE_THREADS / 64];
    extern __shared__ __attribute__((aligned(16))) float sh_lds[];  // [PRE_THREADS][3M + 1]
    const gsr_inputs &in = a.in;
    const int g0 = blockIdx.x * PRE_THREADS;
    const int idx = g0 + threadIdx.x;
    const int RW = RWC > 0 ? RWC : 3 * in.M;  // SH row width (floats)
    const bool use_sh = !GEOM && in.sh != nullptr && in.colors_precomp == nullptr;
    const int n = min(PRE_THREADS, in.P - g0);
    // This Gaussian's own inputs are loaded first and its SH row after them: at
    // degree 3 each thread loads its own 192-B row as 12 x 16 B straight into
    // registers, in flight behind the geometry below (vmcnt counts in issue
    // order).  Per instruction the lanes touch 64 different 128-B lines (stride
    // 192 B) but the 12 loads cover the wave's 12 KB exactly, so L2 serves the
    // re-touches; without an LDS stage the kernel is no longer LDS-limited to 3
    // waves per SIMD (preprocess 68 -> 66 us at C, 334 -> 317 us at E).  Other
    // degrees stage the workgroup's rows through LDS (coalesced, odd row stride).
    constexpr bool DIRECT = RWC == 48 && !GEOM;  // each thread's own row in registers, no LDS
    const bool live = idx < in.P;
    const int li = live ? idx : in.P - 1;
    const f3 p = {in.means3D[3 * li], in.means3D[3 * li + 1], in.means3D[3 * li + 2]};
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
    const float opac_in = in.opacities[li];
    float4 rowv[DIRECT ? 12 : 1];
    if constexpr (DIRECT && SPLIT) {  // _features_dc + _features_rest rows
        float r[48];
        load_sh_row_split(in.sh, in.sh_rest, (size_t)li, r);
#pragma unroll
        for (int b = 0; b < 12; b++) rowv[b] = make_float4(r[4 * b], r[4 * b + 1], r[4 * b + 2], r[4 * b + 3]);
    } else if constexpr (DIRECT) {  // launched only with SH rows (16-B aligned)
        const float4 *r4 = reinterpret_cast<const float4 *>(in.sh + (size_t)li * 48);
#pragma unroll
        for (int b = 0; b < 12; b++) rowv[b] = r4[b];
    } else if (use_sh) {
        if constexpr (SPLIT) {
            rows_to_lds_cols<PRE_THREADS>(in.sh, g0, n, 3, 0, RW + 1, sh_lds);
            if (RW > 3) rows_to_lds_cols<PRE_THREADS>(in.sh_rest, g0, n, RW - 3, 3, RW + 1, sh_lds);
        } else {
            rows_to_lds<PRE_THREADS, RWC>(in.sh, g0, n, RW, sh_lds);
        }
    }
    // the stored parameters' activations (gsr_inputs.activations), as torch computes them
    const float opac = (in.activations & GSR_ACT_OPACITY) ? act_sigmoid(opac_in) : opac_in;
    if (!in.cov3D_precomp) {
        if (in.activations & GSR_ACT_SCALE)
#pragma unroll
            for (int k = 0; k < 3; k++) gin[k] = act_exp(gin[k]);
        if (in.activations & GSR_ACT_ROTATION) (void)act_normalize(gin + 3);
    }
    uint32_t touched = 0;
    bool perr = false;
    // the depth sort's candidate key range (gsr_publish.hpp): depth_keys_kernel keys
    // a Gaussian in front of the near plane by its view depth's bits — the same
    // xform_point4x3 as here, so the same bits
    uint32_t kmin = 0xffffffffu, kmax = 0u;
    // what the colour stage (after the barrier) needs
    bool emit = false;
    float px = 0.f, py = 0.f, conic_x = 0.f, conic_y = 0.f, conic_z = 0.f, qmax = 0.f, depth = 0.f;
    if (live) {
        int radius_out = 0;
        uint4 rect_out = make_uint4(0u, 0u, 0u, 0u);
        const f4 p_hom = xform_point4x4(p, Pm);
        const float p_w = 1.0f / (p_hom.w + 0.0000001f);
        const f3 p_proj = {p_hom.x * p_w, p_hom.y * p_w, p_hom.z * p_w};
        const f3 p_view = xform_point4x3(p, V);
        if (p_view.z > 0.2f) kmin = kmax = __float_as_uint(p_view.z);
        bool ok = true;
        if (p_view.z <= 0.2f) {
            ok = false;
            perr = in.prefiltered != 0;
        }
        float c3[6];
        if (ok) {
            if (in.cov3D_precomp) {
#pragma unroll
                for (int k = 0; k < 6; k++) c3[k] = gin[k];
            } else {
                compute_cov3d(gin[0], gin[1], gin[2], in.scale_modifier, gin[3], gin[4], gin[5], gin[6], c3);
            }
        }
        f3 cov = {0, 0, 0};
        float det = 0.f;
        if (ok) {
            cov = compute_cov2d(p, a.focal_x, a.focal_y, in.tan_fovx, in.tan_fovy, c3, V);
            det = (cov.x * cov.z - cov.y * cov.y);
            if (det == 0.0f) ok = false;
        }
        if (ok) {
            const float det_inv = 1.f / det;
            conic_x = cov.z * det_inv;
            conic_y = -cov.y * det_inv;
            conic_z = cov.x * det_inv;
            const float mid = 0.5f * (cov.x + cov.z);
            const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
            const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
            const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
            px = ndc2pix(p_proj.x, in.W);
            py = ndc2pix(p_proj.y, in.H);
            const int r = f2i_sat(my_radius);
            const TileRect rc = get_rect(px, py, r, a.gx, a.gy);
            const uint32_t area = (rc.x1 - rc.x0) * (rc.y1 - rc.y0);
            if (area != 0) {
                // Cull bound for the blend kernels: alpha = o*exp(-q/2) >= 1/255 needs
                // q = d^T conic d <= 2 ln(255 o).  Stored widened (0.1% + 0.002) so a
                // wave may skip a Gaussian only when every pixel would reject it.
                qmax = 2.0f * logf(255.0f * opac) * 1.001f + 0.002f;
                emit = true;
                depth = p_view.z;
                radius_out = r;
                // Tile mask of the rect (row-major bit per tile); all ones = every
                // tile of the rect, whatever its area (upstream's getRect
                // footprint, GSR_FOOTPRINT_RECT).
                // Tight footprint (GSR_FOOTPRINT_TIGHT): of the bounding rect's
                // tiles keep those whose 16x16 pixel box meets the alpha >= 1/255
                // ellipse q(d) <= qmax (qmax already widened, above).  Per tile row
                // the ellipse's x-extent over the row's band of pixel centres is
                // exact: the leftmost / rightmost points of the ellipse clamped into
                // the band (the boundary's x is convex / concave in y).  Dropped
                // tiles hold only pixels that every blend would skip, so images and
                // gradients are unchanged while ~40% fewer instances are binned
                // (config C).  Rects of more than 64 tiles, and NaN bounds, keep
                // every tile.
                uint64_t m = ~0ull;
                touched = area;
                if (in.footprint == GSR_FOOTPRINT_TIGHT && area <= 64 && !(qmax != qmax)) {
                    m = 0;
                    const float ka = conic_x, kb = conic_y, kc = conic_z;
                    const float kdet = ka * kc - kb * kb;
                    const float tq = fmaxf(qmax, 0.0f);  // qmax < 0: opacity < 1/255, no pixel blends
                    const float yext = sqrtf(tq * ka / kdet);                    // |dy| reach
                    const float yl = kb / kc * sqrtf(tq * kc / kdet);            // dy of the leftmost point
                    const float ia = 1.0f / ka;
                    const int w = rc.x1 - rc.x0;
                    for (int ty = rc.y0; ty < rc.y1 && qmax >= 0.0f; ty++) {
                        const float b0 = fmaxf((float)(ty * TILE_Y) - py, -yext);
                        const float b1 = fminf((float)(ty * TILE_Y + TILE_Y - 1) - py, yext);
                        if (!(b0 <= b1)) continue;
                        const float y1 = fminf(fmaxf(yl, b0), b1), y2 = fminf(fmaxf(-yl, b0), b1);
                        const float xmin = (-kb * y1 - sqrtf(fmaxf(ka * tq - kdet * y1 * y1, 0.0f))) * ia;
                        const float xmax = (-kb * y2 + sqrtf(fmaxf(ka * tq - kdet * y2 * y2, 0.0f))) * ia;
                        // pixel-centre x range, widened by a rounding allowance
                        const float lo = px + xmin - 1e-3f - 1e-5f * fabsf(xmin);
                        const float hi = px + xmax + 1e-3f + 1e-5f * fabsf(xmax);
                        const int ta = max(rc.x0, (int)ceilf((lo - (float)(TILE_X - 1)) / (float)TILE_X));
                        const int tb = min(rc.x1 - 1, (int)floorf(hi / (float)TILE_X));
                        if (ta > tb) continue;
                        const int n = tb - ta + 1, sh = (ty - rc.y0) * w + (ta - rc.x0);
                        m |= (n >= 64 ? ~0ull : ((1ull << n) - 1ull)) << sh;
                    }
                    touched = m == ~0ull ? area : (uint32_t)__builtin_popcountll(m);
                }
                rect_out = make_uint4(rc.x0 | (rc.x1 << 16), rc.y0 | (rc.y1 << 16), (uint32_t)m, (uint32_t)(m >> 32));
            }
        }
        // depths of invisible Gaussians: +inf (the depth sort keys its candidates
        // itself, binning.hip depth_keys_kernel)
        if (!radius_out) a.depths[idx] = __uint_as_float(0x7f800000u);
        a.radii[idx] = radius_out;
        a.tiles_touched[idx] = touched;
        if (a.rwords)
            a.rwords[idx] = rect_word(rect_out);
        else
            a.rects[idx] = rect_out;
    }
    // (stores are counted by vmcnt too: issued here, after the geometry, they do not
    // hold up its waits for the per-Gaussian loads)
    for (int t = idx; t < a.tiles; t += gridDim.x * PRE_THREADS) a.ranges[t] = make_uint2(0u, 0u);
    for (int t = idx; t < a.sup0_n; t += gridDim.x * PRE_THREADS) a.sup0[t] = 0u;
    if (idx < 8 * ORDER_NBUCKET) a.order_cnt[idx] = 0u;  // the backward wave-order buckets (render_bwd.hip)
    if (idx == 0) {  // and the flag words (one block may be all there is)
        a.order_cnt[ORDER_FILED] = 0u;
        a.order_cnt[ORDER_FRESH] = 0u;
        a.ctrl[CTRL_SHJAC] = a.shjac != nullptr && (use_sh || GEOM) ? 1u : 0u;  // this call's Jacobian, or none
    }
    // colour stage: the SH rows land in LDS now, after the geometry
    if (use_sh && !DIRECT) __syncthreads();
    if (emit) {
        float rgb[3] = {0.f, 0.f, 0.f};
        uint8_t clampbits = 0;
        if (GEOM) {
            // the colour words and clamp bits: preprocess_colour_kernel
        } else if (in.colors_precomp) {
            rgb[0] = in.colors_precomp[3 * (size_t)idx];
            rgb[1] = in.colors_precomp[3 * (size_t)idx + 1];
            rgb[2] = in.colors_precomp[3 * (size_t)idx + 2];
        } else {
            const float dx = p.x - in.campos[0], dy = p.y - in.campos[1], dz = p.z - in.campos[2];
            const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
            const float x = dx / len, y = dy / len, z = dz / len;
            const float *sh = DIRECT ? reinterpret_cast<const float *>(rowv) : sh_lds + threadIdx.x * (RW + 1);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float v = sh_channel(sh, c, in.D, x, y, z);
                clampbits |= (v < 0) ? (uint8_t)(1u << c) : (uint8_t)0;
                rgb[c] = fmaxf(v, 0.0f);
            }
            if (a.shjac) {
                // a backward follows: its view-direction term needs d colour / d dir,
                // 36 B here (coalesced planes) instead of the 192-B SH row there
                float J[9];
                sh_dir_jacobian(sh, in.D, x, y, z, J);
#pragma unroll
                for (int k = 0; k < 9; k++) store_jac(a.shjac + (size_t)k * in.P + idx, J[k]);
            }
        }
        // (depths and means2D: introspection only — no kernel of the step reads them)
        store_stream<1>(a.depths + idx, depth);
        store_stream<1>(&a.means2D[idx].x, px);
        store_stream<1>(&a.means2D[idx].y, py);
        // conic and bound stored times -1/2 (exact): the blend kernels then
        // evaluate upstream's power -0.5 * d^T conic d as d^T conic' d, bit for
        // bit, one multiply fewer per (pixel, Gaussian).  The record also carries
        // the Gaussian's index (the backward's atomic target).
        const float ca = -0.5f * conic_x, cb = -0.5f * conic_y, cc = -0.5f * conic_z, qm = -0.5f * qmax;
        float4 *sp = a.splats + 3 * (size_t)idx;
        sp[0] = make_float4(px, py, ca, cb);
        sp[1] = make_float4(cc, opac, rgb[0], rgb[1]);
        sp[2] = make_float4(rgb[2], __uint_as_float((uint32_t)idx), qm, 0.0f);
        if (!GEOM) a.clamped[idx] = clampbits;
    }
    // num_rendered is only a total (emit works in depth order, binning.hip): each
    // workgroup stores its sum (bit 31 flags a prefiltered violation)
    const uint32_t tot = block_sum<PRE_THREADS>(touched, wsum);
    const int berr = __syncthreads_or(perr);
    __shared__ uint32_t wmin[PRE_THREADS / 64], wmax[PRE_THREADS / 64];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    if ((threadIdx.x & 63) == 0) {
        wmin[threadIdx.x >> 6] = kmin;
        wmax[threadIdx.x >> 6] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < PRE_THREADS / 64; k++) {
            kmin = min(kmin, wmin[k]);
            kmax = max(kmax, wmax[k]);
        }
        a.block_sums[blockIdx.x] = make_uint4(tot | (berr ? 0x80000000u : 0u), kmin, kmax, 0u);
    }
}

// The colour half's inputs and outputs (gsr_colour.hpp), from the preprocess arguments.
__host__ __device__ inline ColourRide colour_ride(const gsr_inputs &in, const PreArgs &a) {
    ColourRide c{};
    c.sh = in.sh;
    c.sh_rest = in.sh_rest;
    c.means3D = in.means3D;
    c.campos = in.campos;
    c.radii = a.radii;
    c.shjac = a.shjac;
    c.splats = a.splats;
    c.clamped = a.clamped;
    c.P = in.P;
    c.D = in.D;
    c.b0 = 0;
    c.nb = 0;
    return c;
}

// The colour half of preprocess for the Gaussians the geometry half kept (radii >
// 0; launched after it on a side stream, beside the depth sort and the binning,
// which are bound by their launches' latency and leave the CUs mostly idle):
// forward.cu computeColorFromSH -> the splat record's colour words, the clamp bits
// and, when a backward follows, the SH direction Jacobian — the same operations
// as the fused kernel's colour stage, so the same bits.
template <int RWC, bool SPLIT>
__global__ void __launch_bounds__(PRE_THREADS) preprocess_colour_kernel(PreArgs a) {
    constexpr bool DIRECT = RWC == 48;
    if constexpr (DIRECT) {  // each thread's own row in registers (gsr_colour.hpp)
        colour_rows48<SPLIT>(colour_ride(a.in, a), (int)blockIdx.x);
        return;
    } else {
        extern __shared__ __attribute__((aligned(16))) float sh_lds[];  // [PRE_THREADS][3M + 1]
        const gsr_inputs &in = a.in;
        const int g0 = blockIdx.x * PRE_THREADS;
        const int idx = g0 + threadIdx.x;
        const int RW = RWC > 0 ? RWC : 3 * in.M;
        const int n = min(PRE_THREADS, in.P - g0);
        const bool emit = idx < in.P && a.radii[idx] > 0;
        // the workgroup's rows through LDS (coalesced), every thread takes part
        if constexpr (SPLIT) {
            rows_to_lds_cols<PRE_THREADS>(in.sh, g0, n, 3, 0, RW + 1, sh_lds);
            if (RW > 3) rows_to_lds_cols<PRE_THREADS>(in.sh_rest, g0, n, RW - 3, 3, RW + 1, sh_lds);
        } else {
            rows_to_lds<PRE_THREADS, RWC>(in.sh, g0, n, RW, sh_lds);
        }
        __syncthreads();
        if (!emit) return;
        const f3 p = {in.means3D[3 * idx], in.means3D[3 * idx + 1], in.means3D[3 * idx + 2]};
        const float dx = p.x - in.campos[0], dy = p.y - in.campos[1], dz = p.z - in.campos[2];
        const float len = sqrtf((dx * dx + dy * dy) + dz * dz);
        const float x = dx / len, y = dy / len, z = dz / len;
        const float *sh = sh_lds + threadIdx.x * (RW + 1);
        float rgb[3];
        uint8_t clampbits = 0;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float v = sh_channel(sh, c, in.D, x, y, z);
            clampbits |= (v < 0) ? (uint8_t)(1u << c) : (uint8_t)0;
            rgb[c] = fmaxf(v, 0.0f);
        }
        if (a.shjac) {
            float J[9];
            sh_dir_jacobian(sh, in.D, x, y, z, J);
#pragma unroll
            for (int k = 0; k < 9; k++) store_jac(a.shjac + (size_t)k * in.P + idx, J[k]);
        }
        // the record's colour words: floats 6, 7 ({cc, opacity, r, g}) and 8 ({b, ...})
        float *rec = reinterpret_cast<float *>(a.splats + 3 * (size_t)idx);
        *reinterpret_cast<float2 *>(rec + 6) = make_float2(rgb[0], rgb[1]);
        rec[8] = rgb[2];
        a.clamped[idx] = clampbits;
    }
}

// auxiliary.h in_frustum via checkFrustum (markVisible).
__global__ void mark_visible_kernel(int P, const float *means3D, const float *viewmatrix, uint8_t *present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const Mat4 V = load_mat4(viewmatrix);
    const f3 p = {means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]};
    const f3 pv = xform_point4x3(p, V);
    present[idx] = !(pv.z <= 0.2f);
}

static PreArgs pre_args(const gsr_inputs &in, void *geom, int32_t *radii, bool rwords) {
    const GeomLayout L = geom_layout(in.P, in.W, in.H);
    const GridDims g = grid_dims(in.W, in.H);
    PreArgs a;
    a.in = in;
    a.focal_y = in.H / (2.0f * in.tan_fovy);  // rasterizer_impl.cu: height / (2.0f * tan_fovy)
    a.focal_x = in.W / (2.0f * in.tan_fovx);
    a.gx = g.gx;
    a.gy = g.gy;
    a.depths = at<float>(geom, L.off[GSR_GEOM_DEPTHS]);
    a.means2D = at<float2>(geom, L.off[GSR_GEOM_MEANS2D]);
    a.splats = at<float4>(geom, L.off[GSR_GEOM_SPLATS]);
    a.clamped = at<uint8_t>(geom, L.off[GSR_GEOM_CLAMPED]);
    a.tiles_touched = at<uint32_t>(geom, L.off[GSR_GEOM_TILES_TOUCHED]);
    a.rects = at<uint4>(geom, L.rects);
    a.rwords = rwords ? at<uint32_t>(geom, L.rs_words) + 3 * (size_t)in.P : nullptr;
    a.ranges = at<uint2>(geom, L.off[GSR_GEOM_RANGES]);
    a.tiles = g.tiles;
    a.block_sums = at<uint4>(geom, L.block_sums);
    a.radii = radii;
    a.order_cnt = at<uint32_t>(geom, L.order_cnt);
    a.ctrl = at<uint32_t>(geom, L.off[GSR_GEOM_CTRL]);
    a.sup0 = dsort_grouped1(in.P) ? at<uint32_t>(geom, L.dsort_sup0) : nullptr;
    a.sup0_n = dsort_grouped1(in.P) ? dsort_nsup(in.P) * RADIX : 0;
    a.shjac = (in.flags & GSR_FLAG_PREPARE_BACKWARD) && in.sh && !in.colors_precomp ? at<float>(geom, L.shjac) : nullptr;
    return a;
}

// the register prefetch of cat rows reads them as float4: 16-B aligned only
static bool direct_rows(const gsr_inputs &in) {
    return in.sh && !in.colors_precomp && 3 * in.M == 48 && (in.sh_rest != nullptr || ((uintptr_t)in.sh & 15u) == 0);
}

bool colour_ride_plan(const gsr_inputs &in, void *geom, int32_t *radii, ColourRide *ride) {
    if (!direct_rows(in) || in.P <= 0) return false;
    const PreArgs a = pre_args(in, geom, radii, false);
    *ride = colour_ride(in, a);
    ride->nb = pre_blocks(in.P);
    return true;
}

hipError_t launch_preprocess(const gsr_inputs &in, void *geom, int32_t *radii, bool rwords, hipStream_t s,
                             int phase) {
    const PreArgs a = pre_args(in, geom, radii, rwords);
    const int nb = pre_blocks(in.P);
    const bool split = in.sh_rest != nullptr;
    const bool direct = direct_rows(in);
    const size_t lds = (in.sh && !in.colors_precomp && !direct) ? (size_t)PRE_THREADS * (3 * in.M + 1) * sizeof(float) : 0;
    // SH row width as a compile-time constant for the common degrees (cheap LDS
    // row indexing); any other width takes the run-time path
    const int width = in.sh && !in.colors_precomp ? 3 * in.M : 0;
    auto go = [&](auto kern, size_t shm) { hipLaunchKernelGGL(kern, dim3(nb), dim3(PRE_THREADS), shm, s, a); };
    if (phase == PRE_PHASE_GEOM) {  // (SH inputs only: launch_preprocess_apart)
        go(preprocess_fwd_kernel<0, false, true>, 0);
    } else if (phase == PRE_PHASE_COLOUR) {
        if (width == 3)
            go(preprocess_colour_kernel<3, false>, lds);
        else if (width == 48 && direct)
            split ? go(preprocess_colour_kernel<48, true>, 0) : go(preprocess_colour_kernel<48, false>, 0);
        else
            split ? go(preprocess_colour_kernel<0, true>, lds) : go(preprocess_colour_kernel<0, false>, lds);
    } else if (width == 3) {  // (M = 1 has no rest coefficients: never split)
        go(preprocess_fwd_kernel<3, false>, lds);
    } else if (width == 48 && direct) {
        split ? go(preprocess_fwd_kernel<48, true>, lds) : go(preprocess_fwd_kernel<48, false>, lds);
    } else {
        split ? go(preprocess_fwd_kernel<0, true>, lds) : go(preprocess_fwd_kernel<0, false>, lds);
    }
    // num_rendered: the depth sort's first digit scan publishes it (binning.hip)
    return hipGetLastError();
}

hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present, hipStream_t s) {
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, viewmatrix, present);
    return hipGetLastError();
}

}  // namespace gsr

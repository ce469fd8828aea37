/*
 * gsr.h — C ABI of the MI355X (gfx950) differentiable Gaussian rasterizer.
 *
 * This is the drop-in boundary beneath the Python package
 * `diff_gaussian_rasterization` (3dgs_study_amd/diff_gaussian_rasterization),
 * which the reference imports at gaussian_renderer/__init__.py:14 and calls at
 * gaussian_renderer/__init__.py:98-106.  Upstream, the same boundary is the
 * pybind11 module `_C` with three entry points ([UPSTREAM-SPEC]):
 *
 *   _C.rasterize_gaussians(bg, means3D, colors, opacity, scales, rotations,
 *       scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tanfovx,
 *       tanfovy, image_height, image_width, sh, sh_degree, campos,
 *       prefiltered, debug)
 *       -> (num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer)
 *   _C.rasterize_gaussians_backward(bg, means3D, radii, colors, scales,
 *       rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
 *       tanfovx, tanfovy, dL_dout_color, sh, sh_degree, campos, geomBuffer,
 *       num_rendered, binningBuffer, imgBuffer, debug)
 *       -> (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drot)
 *   _C.mark_visible(means3D, viewmatrix, projmatrix) -> present
 *
 * Here the same work is split into C functions with plain pointers and sizes
 * (no torch types).  The caller owns every buffer: the library never
 * allocates device memory.  All pointers are device pointers unless noted;
 * `stream` is a hipStream_t.  Optional inputs use NULL = absent (upstream's
 * empty-tensor convention).  Every function returns 0 on success or a
 * nonzero gsr_status; gsr_last_error() then describes the failure
 * (thread-local string).
 *
 * The binning buffer's size depends on num_rendered, which needs one
 * device->host read (upstream does the same cudaMemcpy inside
 * Rasterizer::forward).  Two ways to run the forward:
 *   - gsr_forward (one call): the caller passes a binning buffer of a guessed
 *     capacity (e.g. the last num_rendered of this scene plus a margin); the
 *     whole forward is queued before the host waits for the count, so the
 *     device never idles on the read-back.  If the count exceeds the capacity
 *     it returns GSR_NEED_BINNING with *num_rendered set, and the caller
 *     finishes with gsr_forward_render on a buffer of that size;
 *   - gsr_forward_preprocess -> *num_rendered (synchronises `stream` once), the
 *     caller allocates gsr_binning_bytes(num_rendered, W, H) bytes, then
 *     gsr_forward_render: bucket by tile, per-tile depth sort, blend.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 12

enum gsr_status {
    GSR_OK = 0,
    GSR_ERR_ARGS = 1,        /* bad sizes / pointer combination (upstream AT_ERROR / Exception) */
    GSR_ERR_HIP = 2,         /* HIP runtime error (launch failure, fault) */
    GSR_ERR_PREFILTERED = 3, /* a point was culled although prefiltered=1 (upstream __trap) */
    GSR_ERR_CAPACITY = 4,    /* image/tile count beyond the supported range */
    GSR_NEED_BINNING = 5     /* gsr_forward: num_rendered exceeds the binning buffer's capacity (not an error:
                                preprocess is done, finish with gsr_forward_render on a bigger buffer) */
};

/* Tile footprint of a Gaussian (which of its bounding-rect tiles get a list
 * entry).  Not an upstream argument: RECT (0, the struct's zero value) is upstream's
 * getRect footprint — every tile of the 3-sigma bounding rect, so num_rendered,
 * tiles_touched, the sorted (tile << 32 | depth) keys, point_list, ranges and
 * n_contrib are upstream's (rasterizer_impl.cu duplicateWithKeys /
 * identifyTileRanges).  TIGHT (1) keeps only the rect tiles whose 16x16 box the
 * Gaussian's alpha >= 1/255 ellipse reaches: the dropped entries are ones every
 * pixel of their tile skips, so image, radii, final_T and every gradient are
 * the same, with ~40 % fewer instances to sort and stream (config C: 8.0M ->
 * 4.9M); num_rendered, the lists and n_contrib then index the shorter lists.
 * Forward and backward of one render must use the same footprint.  The Python
 * package defaults to RECT (upstream's); TIGHT changes only num_rendered and the
 * lists among upstream's outputs. */
enum gsr_footprint { GSR_FOOTPRINT_RECT = 0, GSR_FOOTPRINT_TIGHT = 1 };

/* gsr_inputs.flags.  GSR_FLAG_PREPARE_BACKWARD (forward calls; not upstream):
 * a backward will follow, so the blend kernel also zeroes the backward's
 * gradient accumulator (inside the geom buffer) and a small launch after it files
 * the quadrants for the backward's wave order — work the backward then skips
 * (its accum argument NULL: the geom buffer's accumulator; a second backward of
 * the same forward zeroes it again itself).  Only a speed hint: every backward
 * is correct with or without it, and any number of forward renders may follow
 * one preprocess (each files its own quadrants afresh). */
enum gsr_flags { GSR_FLAG_PREPARE_BACKWARD = 1, GSR_FLAG_L1_SEED = 2, GSR_FLAG_NO_WAIT = 4 };

/* GSR_FLAG_NO_WAIT (gsr_forward only; not upstream): for stream capture (HIP
 * graphs, torch.cuda.graph).  gsr_forward queues the whole forward into the
 * capacity-sized binning buffer and returns without reading anything back (the
 * depth sort with gsr_depth_passes_hint() passes), with *num_rendered = capacity.
 * Each binning kernel still checks the count and pass count the device publishes
 * and does nothing unless both fit, so after the queued (or replayed) work has run
 * the caller checks them with gsr_forward_status.  Needs capacity > 0 and debug
 * off. */

/* GSR_FLAG_L1_SEED (backward calls; not upstream): the image's gradient is that of
 * the L1 loss mean|image - gt| (utils/loss_utils.py l1_loss, train.py:102 with
 * lambda_dssim = 0), and the backward's dL_dout_color argument points to this
 * struct instead of a [3,H,W] map.  The render backward forms each pixel's
 * dL/dpixel = (dloss / n) * sign(image - gt) itself — gsr_l1_grad's values bit
 * for bit — so no gradient map is written or read.  image is the forward's
 * out_color, gt a [3,H,W] float32 image, dloss one float on the device, n = 3 H W. */
typedef struct gsr_l1_seed {
    const float *image;
    const float *gt;
    const float *dloss;
    int64_t n;
} gsr_l1_seed;

/* gsr_inputs.activations (not upstream; 0 = upstream's inputs, used as given).
 * The reference hands the rasterizer activations of GaussianModel's stored
 * parameters (scene/gaussian_model.py:107-126, gaussian_renderer/__init__.py:
 * 81-96): opacities = sigmoid(_opacity), scales = exp(_scaling), rotations =
 * F.normalize(_rotation).  With a bit set the input IS the stored parameter and
 * the library applies that activation itself, with torch's GPU operations in
 * torch's order, so the values equal torch's bit for bit (sigmoid: 1 / (1 +
 * exp(-x)); exp; normalize: x / max(sqrt((x0^2 + x1^2) + (x2^2 + x3^2)), 1e-12),
 * tools/act_probe.py measured that order), and every backward output for that
 * input — the plain one (dopacity / dscales / drot) or the leaf one — is the
 * gradient of the stored parameter (through the activation's backward, as
 * gsr_leaf_grads describes; rotation_norm is not needed). */
enum gsr_activations {
    GSR_ACT_OPACITY = 1,  /* opacities are logits (_opacity) */
    GSR_ACT_SCALE = 2,    /* scales are logarithms (_scaling) */
    GSR_ACT_ROTATION = 4  /* rotations are unnormalised quaternions (_rotation) */
};

/* Inputs shared by forward and backward.  Mirrors the argument list of
 * _C.rasterize_gaussians (rasterize_points.cu RasterizeGaussiansCUDA); the
 * fields after campos are not upstream (zero = upstream's behaviour). */
typedef struct gsr_inputs {
    int32_t P;                  /* number of Gaussians (means3D.size(0)) */
    int32_t D;                  /* active SH degree (sh_degree) */
    int32_t M;                  /* SH coefficients per channel = sh.size(1), 0 if sh == NULL */
    int32_t W, H;               /* image_width, image_height */
    float tan_fovx, tan_fovy;   /* tanfovx, tanfovy */
    float scale_modifier;
    int32_t prefiltered;        /* bool */
    int32_t debug;              /* bool: synchronise + check after every kernel */
    int32_t footprint;          /* enum gsr_footprint: which (tile, Gaussian) pairs are binned */
    int32_t flags;              /* gsr_flags bits (0 = none) */
    const float *bg;            /* [3]   background colour */
    const float *means3D;       /* [P,3] */
    const float *colors_precomp;/* [P,3] or NULL */
    const float *opacities;     /* [P,1] */
    const float *scales;        /* [P,3] or NULL */
    const float *rotations;     /* [P,4] or NULL (quaternion r,x,y,z, used as given) */
    const float *cov3D_precomp; /* [P,6] or NULL */
    const float *viewmatrix;    /* [4,4] row-major storage of W2C^T (scene/cameras.py:103) */
    const float *projmatrix;    /* [4,4] full_proj_transform (scene/cameras.py:114-118) */
    const float *sh;            /* [P,M,3] or NULL */
    const float *campos;        /* [3]   camera_center (scene/cameras.py:121) */
    /* GaussianModel's SH storage without the cat (scene/gaussian_model.py:
     * get_features): with sh_rest non-NULL, sh is _features_dc [P,1,3] and sh_rest
     * _features_rest [P,M-1,3] (both 4-byte aligned rows); M counts both. */
    const float *sh_rest;
    int32_t activations;        /* gsr_activations bits */
    int32_t reserved;           /* 0 */
} gsr_inputs;

/* Scratch sizes in bytes (all buffers 256-byte aligned internally).
 * geom:    per-Gaussian state + per-tile counting scratch (upstream GeometryState),
 *          and the backward's gradient accumulator (64 B per Gaussian)
 * binning: per-instance keys and the sorted point list (upstream BinningState),
 *          for a capacity of num_rendered instances or more; the point list sits
 *          at offset 0 whatever the capacity (the backward needs only the pointer)
 * img:     per-pixel final T / contributor counts (ImageState)
 * accum:   a separate backward accumulator (64 B per Gaussian), for callers that
 *          pass one to a backward instead of NULL (the geom buffer's) */
size_t gsr_geom_bytes(int32_t P, int32_t W, int32_t H);
size_t gsr_binning_bytes(int64_t num_rendered, int32_t W, int32_t H);
size_t gsr_img_bytes(int32_t W, int32_t H);
size_t gsr_accum_bytes(int32_t P);

/* Replaces the first half of RasterizeGaussiansCUDA -> Rasterizer::forward
 * (preprocess + InclusiveSum + the num_rendered cudaMemcpy).  The device also
 * sorts the P Gaussians by depth (the first half of the binning, see
 * 3dgs_study_amd/csrc/binning.hip), in line on `stream` after preprocess.
 * Writes radii [P] int32 and *num_rendered (host pointer). */
int gsr_forward_preprocess(const gsr_inputs *in, void *geom, int32_t *radii, int64_t *num_rendered, void *stream);

/* Replaces the second half of Rasterizer::forward (duplicateWithKeys,
 * SortPairs, identifyTileRanges, FORWARD::render).  out_color is [3,H,W];
 * radii as written by gsr_forward_preprocess. */
int gsr_forward_render(const gsr_inputs *in, void *geom, void *binning, void *img, int64_t num_rendered,
                       const int32_t *radii, float *out_color, void *stream);

/* gsr_forward_render plus the L1 loss mean|out_color - gt| (utils/loss_utils.py
 * l1_loss, train.py:102; not upstream) into loss_out [3] = {loss, loss, 0}
 * (gsr_l1_ssim's layout with lambda 0, the same bits).  With
 * GSR_FLAG_PREPARE_BACKWARD the loss's partial sums are computed in the same
 * launch as the backward's preparation, and so, when visible_out is not NULL, is
 * visible_out [P] bytes = radii > 0 (render()'s visibility_filter,
 * gaussian_renderer/__init__.py; visible_out requires the flag).  gt is [3,H,W]
 * float32; img is required.  The backward's GSR_FLAG_L1_SEED (above) is its
 * gradient. */
int gsr_forward_render_l1(const gsr_inputs *in, void *geom, void *binning, void *img, int64_t num_rendered,
                          const int32_t *radii, float *out_color, const float *gt, float *loss_out,
                          uint8_t *visible_out, void *stream);

/* The whole of Rasterizer::forward in one call (not an upstream entry point; the
 * Python binding's _C.rasterize_gaussians uses it once it knows a capacity for the
 * scene): gsr_forward_preprocess + gsr_forward_render(_l1), with emit, the tile
 * sort, the blend (and with gt the L1 loss, as gsr_forward_render_l1; gt NULL: no
 * loss, loss_out / visible_out unused) queued BEFORE the host waits for
 * num_rendered, into `binning`, a buffer of gsr_binning_bytes(capacity, W, H) bytes.
 * Each binning kernel reads the published count on the device and does nothing
 * unless it fits.  Returns GSR_OK (*num_rendered <= capacity: every output is
 * written, as by the two-call form) or GSR_NEED_BINNING (*num_rendered >
 * capacity: radii and the geom buffer are complete, the rest is not — the caller
 * allocates gsr_binning_bytes(*num_rendered, W, H) and calls gsr_forward_render /
 * gsr_forward_render_l1 with it).  Debug mode runs the two-call sequence inside
 * the call.  Results are bit-identical to the two-call form. */
int gsr_forward(const gsr_inputs *in, void *geom, int32_t *radii, void *binning, int64_t capacity, void *img,
                float *out_color, const float *gt, float *loss_out, uint8_t *visible_out, int64_t *num_rendered,
                void *stream);

/* Replaces RasterizeGaussiansBackwardCUDA -> Rasterizer::backward.
 * accum: NULL = the accumulator inside geom (zeroed by a forward called with
 * GSR_FLAG_PREPARE_BACKWARD, else here), or a caller buffer of gsr_accum_bytes(P).
 * Every output is fully written (no pre-zeroing needed); dsh may be NULL when
 * in->sh is NULL, dscales/drot may be NULL when in->scales is NULL, dcolors
 * when in->colors_precomp is NULL and dcov3D when in->cov3D_precomp is NULL
 * (upstream returns zeros there, which its autograd wrapper discards).
 * Shapes: dmeans2D [P,3], dcolors [P,3], dopacity [P,1], dmeans3D [P,3],
 * dcov3D [P,6], dsh [P,M,3], dscales [P,3], drot [P,4]. */
int gsr_backward(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning, const void *img,
                 int64_t num_rendered, const float *dL_dout_color, void *accum, float *dmeans2D, float *dcolors,
                 float *dopacity, float *dmeans3D, float *dcov3D, float *dsh, float *dscales, float *drot,
                 void *stream);

/* gsr_backward_planar: gsr_backward with dsh written as M coefficient planes
 * [M][P][3] (plane k at dsh + 3 P k), i.e. the [P,M,3] tensor with strides
 * (3, 3P, 1).  Not an upstream layout: the autograd wrapper returns that strided
 * view, so the f_dc slice the reference's SH `cat` backward hands to
 * AccumulateGrad is already laid out like _features_dc (no copy; scene/
 * gaussian_model.py:106-110 get_features).  Values are gsr_backward's. */
int gsr_backward_planar(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                        float *dscales, float *drot, void *stream);

/* Leaf gradients of the caller's activations, written by the per-Gaussian
 * backward itself (not upstream).  The reference feeds the rasterizer
 * activations of GaussianModel's leaf parameters (scene/gaussian_model.py:
 * 106-126): shs = cat(_features_dc, _features_rest, dim=1), scales =
 * exp(_scaling), opacities = sigmoid(_opacity), rotations =
 * F.normalize(_rotation) (norm clamped at rotation_eps).  Upstream returns
 * dsh / dscales / dopacity / drot and torch's autograd then runs the cat slice
 * copies, exp / sigmoid / normalize backwards and AccumulateGrad; with a
 * non-NULL output here the library writes the leaf's gradient directly, with
 * torch's operation order (exp: d * scales; sigmoid: (d * (1 - o)) * o;
 * normalize: the Div / Expand / ClampMin / LinalgVectorNorm backwards), and
 * the corresponding activation gradient is not written (that output pointer
 * may be NULL).  accumulate bit k adds into output k (AccumulateGrad's
 * `grad += new`) instead of overwriting: bit 0 dsh_dc + dsh_rest, bit 1
 * dscaling, bit 2 dopacity, bit 3 drotation, bit 4 the backward's own dmeans3D
 * output (means3D is itself the leaf GaussianModel._xyz, scene/gaussian_model.py:
 * 114-116: a caller may point dmeans3D at that leaf's .grad).  Inputs by output:
 *   dsh_dc [P,1,3], dsh_rest [P,M-1,3] (NULL when M == 1): in->sh required;
 *   dscaling [P,3]: in->scales (= exp(_scaling)) required;
 *   dopacity [P,1]: in->opacities (= sigmoid(_opacity)) required;
 *   drotation [P,4]: in->rotations (= F.normalize(_rotation), the quotient
 *                    torch computed) and rotation_norm [P] (the row norms
 *                    torch computed, LinalgVectorNormBackward0's result) required,
 *                    or in->rotations = _rotation itself with GSR_ACT_ROTATION.
 * (The backward reads in->opacities whenever it is given; without it the
 * opacity comes from the forward's geom buffer.) */
typedef struct gsr_leaf_grads {
    float *dsh_dc;
    float *dsh_rest;
    float *dscaling;
    float *dopacity;
    float *drotation;
    const float *rotation_norm;
    float rotation_eps;
    int32_t accumulate;
    int32_t dsh_planar;  /* a (non-leaf) dsh output is written as gsr_backward_planar's planes */
    int32_t reserved;
} gsr_leaf_grads;

/* gsr_backward with the leaf outputs above (leaf may be NULL = gsr_backward). */
int gsr_backward_leaves(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                        float *dscales, float *drot, const gsr_leaf_grads *leaf, void *stream);

/* The general backward, every output form at once (not upstream; the entry points
 * above and below are special cases of it).  phases: 1 = accumulator zeroing +
 * render backward (+ drgb, below), 2 = the per-Gaussian backward, 3 = both; a
 * caller splitting them issues 1 then 2 with the same arguments on the same
 * stream, and may start exchanging drgb in between.  GSR_PHASE_COLOURS_APART (4)
 * takes drgb out of the render half: 1 | 4 = the render half without it, 4 alone =
 * drgb only (after the render half; the caller may issue it on another stream,
 * ordered after the render half, beside the per-Gaussian half).  drgb (instead of dsh, and
 * instead of leaf dsh_dc / dsh_rest): the clamp-masked colour gradient of the
 * view-parallel SH exchange (gsr_backward_colors); leaf: as gsr_backward_leaves
 * (NULL = none) — so one backward can hand the SH gradient to the exchange and
 * write the scaling / opacity / rotation leaf gradients and dmeans3D straight into
 * the caller's all-reduce bucket (3dgs_study_amd/multiview.py). */
#define GSR_PHASE_COLOURS_APART 4
int gsr_backward_phase(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                       const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                       float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                       float *drgb, float *dscales, float *drot, const gsr_leaf_grads *leaf, int32_t phases,
                       void *stream);

/* View-parallel exchange of the SH gradient (3dgs_study_amd/multiview.py;
 * SURVEY.md §8e).  Upstream has no multi-GPU path; these two calls split
 * backward.cu computeColorFromSH's dL/dsh = basis(dir) (x) dL/dRGB so that
 * ranks exchange the 12-byte colour gradient per Gaussian and view instead of
 * all-reducing the 12·M-byte dsh.
 *
 * gsr_backward_colors: gsr_backward, except that instead of dsh it writes drgb
 * [P,3], the clamp-masked colour gradient (zero for culled Gaussians); dmeans3D
 * still includes the view-direction term of the SH backward (sh is read).
 * sh_degree must be <= 3.
 *
 * gsr_sh_record_floats(P): floats per view record = 4 + 3P rounded up to a
 * multiple of 4.  A record is [campos.x, campos.y, campos.z, (float)sh_degree,
 * drgb [P][3], padding]; drgb starts 16 B into the record.
 *
 * gsr_sh_grad_from_colors: dsh_dc [P,1,3] and dsh_rest [P,M-1,3] (the leaf
 * gradients of GaussianModel._features_dc / _features_rest) = the sum over the
 * nviews consecutive records of basis_v(normalize(mean - campos_v)) (x) drgb_v,
 * added in record order with preprocess_bwd's exact products (M in {1,4,9,16};
 * dsh_rest may be NULL when M = 1).  Outputs are overwritten. */
int gsr_backward_colors(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *drgb,
                        float *dscales, float *drot, void *stream);
/* The two halves of gsr_backward_colors, so the caller can start exchanging
 * drgb while the per-Gaussian backward runs: _render = accumulator memset,
 * render backward and drgb; _finish = the per-Gaussian backward (same
 * arguments, on the same stream, in that order). */
int gsr_backward_colors_render(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                               const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                               float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D,
                               float *drgb, float *dscales, float *drot, void *stream);
int gsr_backward_colors_finish(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                               const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                               float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D,
                               float *drgb, float *dscales, float *drot, void *stream);
int64_t gsr_sh_record_floats(int32_t P);
int gsr_sh_grad_from_colors(int32_t P, int32_t M, int32_t nviews, const float *means3D, const float *records,
                            float *dsh_dc, float *dsh_rest, void *stream);

/* Replaces markVisible (rasterize_points.cu) / checkFrustum:
 * present[i] = (viewmatrix * means3D[i]).z > 0.2.  present is [P] bytes. */
int gsr_mark_visible(int32_t P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream);

/* Introspection for parity tests: byte offsets of the named sub-arrays inside
 * the scratch buffers.  Returns the number of entries written (<= cap). */
enum gsr_geom_field {
    GSR_GEOM_DEPTHS = 0,     /* float  [P] */
    GSR_GEOM_MEANS2D,        /* float2 [P]  pixel-space centre */
    GSR_GEOM_SPLATS,         /* float4 [P][3] {x,y,c.x,c.y},{c.z,opacity,r,g},{b,id bits,qmax,0}, c = -conic/2, qmax = -bound/2 */
    GSR_GEOM_CLAMPED,        /* uint8  [P]  bit c set = channel c clamped in SH->RGB */
    GSR_GEOM_TILES_TOUCHED,  /* uint32 [P] */
    GSR_GEOM_RANGES,         /* uint2  [T]  [start,end) of each tile in point_list */
    GSR_GEOM_CTRL,           /* uint32 [16] num_rendered, status flags */
    GSR_GEOM_DEPTH_ORDER,    /* uint32 [P]  Gaussian ids in (depth_bits, id) order */
    GSR_GEOM_DSORT_CTRL,     /* uint32 [16] the depth sort's key base (low byte clear) and pass count (3 or 4) */
    GSR_GEOM_NFIELDS
};
enum gsr_binning_field {
    GSR_BIN_KEYS = 0,        /* uint32 [cap] tile-sort scratch */
    GSR_BIN_POINT_LIST,      /* uint32 [I]  Gaussian ids in (tile, depth, id) order: offset 0 */
    GSR_BIN_ROWSPAN,         /* uint32 [2][257] row-span binning (gsr_binning_mode 0): per tile row the first pass-B
                                block and first span; [256] = pass-B blocks, [513] = spans of the forward */
    GSR_BIN_NFIELDS
};
enum gsr_img_field {
    GSR_IMG_FINAL_T = 0,     /* float  [H*W] */
    GSR_IMG_N_CONTRIB,       /* uint32 [H*W] */
    GSR_IMG_NFIELDS
};
/* upstream's sorted keys (BinningState point_list_keys): keys[i] =
 * (tile of entry i) << 32 | float bits of its Gaussian's view depth, for the
 * num_rendered entries of a forward's binning buffer (keys: device, u64). */
int gsr_point_list_keys(int32_t P, int32_t W, int32_t H, const void *geom, const void *binning,
                        int64_t num_rendered, uint64_t *keys, void *stream);
/* Binning form (not upstream; ABI 11).  0 (the default): the row-span binning —
 * every footprint's per-row spans sorted stably by tile row, then their tiles by
 * column — for tile grids of at most 256 x 256 tiles (3840 x 3840 px at 16 x 16),
 * the LSD sort by tile index beyond; 1: the LSD sort by tile index everywhere.
 * Both produce upstream's point_list and ranges bit for bit.  Takes effect at the
 * next preprocess; -1 queries.  Returns the previous mode, or -1 for any other
 * argument (gsr_last_error says why; the mode is unchanged). */
int gsr_binning_mode(int mode);
/* Split replay (not upstream; ABI 12).  The backward replays a tile's list serially
 * per 8x8 pixel quadrant; a list far longer than the average load of a wave slot
 * (config B's centre tiles) then sets the kernel's time.  With split replay the
 * forward (GSR_FLAG_PREPARE_BACKWARD) stores each pixel's transmittance and colour
 * at every SEG-th entry of a list longer than SEG, and the backward replays each
 * SEG-entry segment in a wave of its own from that state.  Gradients agree with the
 * unsplit replay to float rounding (the segment's start state is the forward's T and
 * (C_final - C) / T instead of upstream's divided-down T and running accum_rec).
 * mode -1 (default): SEG from the binning capacity (4 cap / 6144 wave slots, raised
 * to a power of two >= 128; no split when above 1024); 0: off; > 0: that SEG (raised
 * to a power of two the buffer allows).  Takes effect at the next forward; -2
 * queries.  Returns the previous mode, or -3 for an invalid argument. */
int gsr_split_mode(int mode);
/* The depth-sort passes (3 or 4) the next forward on this host thread queues up
 * front: 4 once a forward's keys spanned more than 2^24 steps. */
int gsr_depth_passes_hint(void);
/* After a GSR_FLAG_NO_WAIT forward (or a replay of its capture) has run on the
 * device: *num_rendered = the count its preprocess published to this host
 * thread's pinned words; GSR_OK when it fits `capacity` and the keys needed no
 * more than the `passes` that forward queued (gsr_depth_passes_hint at its call),
 * GSR_NEED_BINNING when not (that forward's lists, image and the backward that
 * followed are incomplete), GSR_ERR_PREFILTERED for upstream's prefiltered error. */
int gsr_forward_status(int64_t capacity, int passes, int64_t *num_rendered);
/* Colour apart (not upstream; ABI 12; opt-in): 1 — gsr_forward runs preprocess as
 * its geometry half on the caller's stream and its colour half (SH -> RGB, the clamp
 * bits, the SH direction Jacobian) on a low-priority side stream forked after it,
 * beside the depth sort and the binning, joined before the blend; 0 (default) — one
 * fused preprocess kernel (the side queue measured slower: DESIGN.md §9); 2 — the
 * geometry half in line and the colour half as extra workgroups of the depth sort's
 * first three downsweeps (one queue; degree-3 SH rows only, else the fused kernel;
 * both forward forms, debug mode too).  Mode 1: SH inputs only, never in debug mode
 * or the two-call form.  The same bits in every mode.  -2 queries; returns the
 * previous mode, or -3 for an invalid argument. */
int gsr_colour_mode(int mode);
/* Microseconds the host has spent in the forward's one wait (the num_rendered
 * read-back) since the last reset, summed over threads; reset != 0 also zeroes it.
 * For benchmarks: a step's host time minus this is the host's own work. */
double gsr_host_wait_us(int reset);
int gsr_geom_layout(int32_t P, int32_t W, int32_t H, size_t *offsets, int cap);
int gsr_binning_layout(int64_t capacity, int32_t W, int32_t H, size_t *offsets, int cap);
int gsr_img_layout(int32_t W, int32_t H, size_t *offsets, int cap);

/* Per-stage device timing (HIP events on the launch stream), for benchmarks.
 * gsr_timing_enable(mask) resets the accumulators and starts recording the
 * stages whose bit (1 << stage) is set in mask (-1: all; 0: off);
 * gsr_timing_read() waits for the recorded events and returns, per stage,
 * the summed milliseconds and the launch count (returns the number of stages,
 * negative on error).  A stage is one launch_* group of kernels. */
enum gsr_stage {
    GSR_STAGE_PREPROCESS = 0, /* FORWARD::preprocessCUDA */
    GSR_STAGE_SCAN,           /* InclusiveSum of tiles_touched: the rects in depth order + emission offsets */
    GSR_STAGE_DEPTH_SORT,     /* stable sort of the P depths */
    GSR_STAGE_DUPLICATE,      /* duplicateWithKeys in depth order (row-span binning: the spans sorted by tile row) */
    GSR_STAGE_TILE_SORT,      /* stable sort by tile (SortPairs) + identifyTileRanges (row spans: tiles by column) */
    GSR_STAGE_RENDER_FWD,     /* FORWARD::renderCUDA */
    GSR_STAGE_RENDER_BWD,     /* BACKWARD::renderCUDA */
    GSR_STAGE_PREPROCESS_BWD, /* BACKWARD::computeCov2DCUDA + preprocessCUDA */
    GSR_STAGE_BWD_PREPARE,    /* accumulator zeroing + the render backward's wave order (no upstream kernel) */
    GSR_STAGE_EXCHANGE_WAIT,  /* caller-marked (gsr_timing_begin/end): the view-parallel exchange's wait for its collectives */
    GSR_STAGE_SH_REBUILD,     /* caller-marked: the SH gradients rebuilt from the gathered colour records */
    GSR_STAGE_COLOUR,         /* preprocess's colour half on the side stream (gsr_colour_mode 1), beside the binning */
    GSR_STAGE_COUNT
};
int gsr_timing_enable(int mask);
int gsr_timing_read(double *total_ms, int64_t *launches, int cap);
/* Record the library's stage events on every `every`-th launch of a stage only
 * (1 = every launch, the default; reset counts restart at gsr_timing_enable): each
 * event pair is a marker packet that leaves the device idle ~4 us, so a benchmark
 * that times a stage inside its timed region samples it.  Caller-marked regions
 * (gsr_timing_begin/end) are always recorded. */
int gsr_timing_sample(int every);
const char *gsr_stage_name(int stage);
/* A caller-marked region of `stage` on `stream` (the same fence-free events as the
 * library's own stages; nothing is recorded unless the stage's bit is enabled):
 * begin and end pair up per stage; each pair counts one launch. */
int gsr_timing_begin(int stage, void *stream);
int gsr_timing_end(int stage, void *stream);

/* ---- Training-step ops after the rasterizer (SURVEY.md §8f "next" rows 1-2) ----
 *
 * gsr_l1_ssim: loss = (1 - lambda) L1(img, gt) + lambda (1 - SSIM(img, gt)) for
 * [C,H,W] float images (utils/loss_utils.py l1_loss + ssim, train.py:103-105),
 * AND its gradient dloss/dimg in the same pass.  loss_out (device, 3 floats):
 * loss, L1 term, mean SSIM.  scratch: gsr_l1_ssim_scratch_bytes.  With
 * lambda_dssim == 0 grad_img may be NULL: the L1 loss alone, whose gradient
 * gsr_l1_grad computes in the backward. */
size_t gsr_l1_ssim_scratch_bytes(int32_t C, int32_t H, int32_t W);
int gsr_l1_ssim(const float *img, const float *gt, int32_t C, int32_t H, int32_t W, float lambda_dssim,
                float *grad_img, void *scratch, float *loss_out, void *stream);
/* The L1 loss's backward for n floats: grad_img = (*dloss / n) * sign(img - gt)
 * (torch's MeanBackward then AbsBackward, bit for bit); dloss is the incoming
 * gradient of the loss, a device scalar. */
int gsr_l1_grad(const float *img, const float *gt, int64_t n, const float *dloss, float *grad_img, void *stream);

/* gsr_adam_step: torch.optim.Adam's update (no weight decay, no amsgrad) on up
 * to GSR_ADAM_MAX_SEGS tensors in one launch; step = the 1-based step count
 * after the increment (scene/gaussian_model.py:176-205: six groups, eps 1e-15).
 * betas/eps/lr are doubles, as the Python-side scalars torch derives its
 * per-step constants from. */
#define GSR_ADAM_MAX_SEGS 8
typedef struct {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;
    double lr;
} gsr_adam_segment;
int gsr_adam_step(const gsr_adam_segment *segs, int32_t nseg, int32_t step, double beta1, double beta2, double eps,
                  void *stream);

/* gsr_densify_stats: for radii[i] > 0: max_radii2D[i] = max(max_radii2D[i], radii[i]),
 * xyz_gradient_accum[i] += |viewspace_grad[i, 0:2]|, denom[i] += 1
 * (train.py:126-127, scene/gaussian_model.py:565-581).  viewspace_grad rows
 * are grad_stride floats apart (3 for the [P,3] means2D gradient). */
int gsr_densify_stats(int32_t P, const int32_t *radii, const float *viewspace_grad, int32_t grad_stride,
                      float *max_radii2D, float *xyz_gradient_accum, float *denom, void *stream);

/* gsr_knn_mean_dist2 (distCUDA2 of the absent simple-knn submodule, used at
 * scene/gaussian_model.py:153-155): dist2[i] = mean of the squared distances
 * from points[i] to its 3 nearest other points (exact; FLT_MAX for missing
 * neighbours).  points [P,3] float; synchronises the stream once (the grid
 * shape depends on the bounding box).  scratch: gsr_knn_scratch_bytes(P). */
size_t gsr_knn_scratch_bytes(int32_t P);
int gsr_knn_mean_dist2(int32_t P, const float *points, float *dist2, void *scratch, void *stream);

const char *gsr_last_error(void);
int gsr_abi_version(void);
/* SHA-256 (hex) of the sources the library was built from (tools/build_id.py):
 * build provenance for tests and benchmark records.  Not upstream. */
const char *gsr_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */

// gsr_kernels.hpp — host-side launchers of the gfx950 kernels (internal).
#pragma once

#include <hip/hip_runtime.h>

#include "gsr_common.hpp"

namespace gsr {

// preprocess.hip (num_rendered is published by the depth sort's first digit scan)
// rwords: write each rect as one word into the depth sort's carried-word input
// (the row-span binning of the rect footprint) instead of the 16-B rect records
// phase: PRE_PHASE_FUSED (one kernel), or the geometry half (PRE_PHASE_GEOM: no SH
// rows read, colour words 0) and the colour half (PRE_PHASE_COLOUR, SH inputs only:
// the records' colour words, clamp bits and Jacobian of the Gaussians the geometry
// half kept) — abi.hip runs the colour half on a side stream beside the binning
enum PrePhase { PRE_PHASE_FUSED = 0, PRE_PHASE_GEOM = 1, PRE_PHASE_COLOUR = 2 };
hipError_t launch_preprocess(const gsr_inputs &in, void *geom, int32_t *radii, bool rwords, hipStream_t s,
                             int phase = PRE_PHASE_FUSED);
// The colour half's arguments as depth-sort riders (gsr_colour.hpp): false when the
// inputs do not take the degree-3 register path (the fused kernel then runs)
bool colour_ride_plan(const gsr_inputs &in, void *geom, int32_t *radii, ColourRide *ride);
hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present,
                               hipStream_t s);

// binning.hip
// passes: 3 (the host launches the fourth after its sync when the published pass
// count says so) or 4 (queued up front; returns at once when three suffice).
// host_ctrl: the caller's pinned words, which the first digit scan fills with the
// pass count and num_rendered (after preprocess, in stream order).
// carry: the rect footprint's words travel with the ids (the row-span binning of the
// rect footprint; gsr_spans.hpp rect_word)
// ride: the colour half of preprocess as extra workgroups of the downsweeps
// (colour_ride_plan; preprocess then ran PRE_PHASE_GEOM), or NULL
hipError_t launch_depth_sort(int P, int W, int H, const float *means3D, const float *viewmatrix, void *geom,
                             int passes, uint32_t *host_ctrl, bool carry, hipStream_t s,
                             const ColourRide *ride = nullptr);
hipError_t launch_depth_sort_fourth(int P, int W, int H, void *geom, bool carry, hipStream_t s);
// rowspan: the row-span binning follows (pass A's row counts and their scan)
hipError_t launch_rank_gather(int P, int W, int H, void *geom, bool require3, bool rowspan, bool carry,
                              hipStream_t s);
hipError_t launch_count_scan(uint32_t *hist, int NB, const uint32_t *nb_dev, uint32_t *totals, int digits,
                             const SpecGuard &g, hipStream_t s);
// cap: the binning buffer's instance capacity (its layout); g: speculative guard
// (gsr_common.hpp SpecGuard; ctrl NULL = the count is exact, cap == num_rendered
// or larger)
hipError_t launch_emit(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                       hipStream_t s);
hipError_t launch_tile_sort(int P, int W, int H, void *geom, void *binning, int64_t n, int64_t cap,
                            const SpecGuard &g, hipStream_t s);
// rowspan.hip: the row-span binning (grids of at most 256 x 256 tiles), after
// launch_rank_gather(..., rowspan = true): pass A (spans by tile row), pass B
// (tiles by column into point_list, and the tile ranges)
hipError_t launch_rowspan_a(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                            bool carry, hipStream_t s);
hipError_t launch_rowspan_b(int P, int W, int H, void *geom, void *binning, int64_t cap, const SpecGuard &g,
                            hipStream_t s);
hipError_t launch_point_list_keys(int P, int W, int H, const void *geom, const void *binning, int64_t I,
                                  uint64_t *keys, hipStream_t s);

// render_fwd.hip
// (binning: point_list at offset 0, whatever the buffer's capacity)
// qmask_cap > 0: record each chunk's cull mask for render_bwd in the binning
// buffer's qmask region (binning_layout(qmask_cap): the buffer's capacity), and with
// seg > 0 the split replay's checkpoints of the lists longer than seg (gsr_common.hpp)
hipError_t launch_render_fwd(const gsr_inputs &in, void *geom, const void *binning, void *img, float *out_color,
                             float *acc_zero, size_t acc_bytes, hipStream_t s, int64_t qmask_cap = 0, int seg = 0);

// render_bwd.hip
// l1 (forward only, or NULL): the L1 loss mean|l1_x - l1_y| (n = 3 W H) into
// l1_out [3], its partial sums and finish (gsr_l1.hpp) in the same launch; needs
// render_fwd_kernel before it (the finish ticket).  visible (forward only, or
// NULL): visible[i] = radii[i] > 0 in the same launch.
hipError_t launch_bwd_prepare(const gsr_inputs &in, void *geom, const void *img, float *accum, bool file,
                              bool internal, bool forward, hipStream_t s, const float *l1_x = nullptr,
                              const float *l1_y = nullptr, float *l1_out = nullptr, const int32_t *radii = nullptr,
                              uint8_t *visible = nullptr);
// qmask_cap > 0: the forward recorded its chunk masks in this binning buffer of that
// capacity (launch_render_fwd); the replay then skips the cull
hipError_t launch_render_bwd(const gsr_inputs &in, const void *geom, const void *binning, const void *img,
                             const float *dL_dpix, const gsr_l1_seed *l1, float *accum, hipStream_t s,
                             int64_t qmask_cap = 0, bool l1_signs = false, int seg = 0);

// preprocess_bwd.hip
struct BwdOutputs {
    float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *dsh, *dscales, *drot;
    float *drgb;  // instead of dsh: the clamp-masked colour gradient [P,3] (view-parallel exchange)
    int dsh_planar;  // dsh laid out [M][P][3] (coefficient planes) instead of [P][M][3]
    int sh_dir;      // read the SH rows for dL/dmean3D's direction term although dsh and drgb are NULL
    gsr_leaf_grads leaf;  // leaf gradients of the caller's activations (NULL outputs: not requested)
};
hipError_t launch_preprocess_bwd(const gsr_inputs &in, const int32_t *radii, const void *geom, const float *accum,
                                 const BwdOutputs &o, hipStream_t s);

// sh_exchange.hip
hipError_t launch_colors_from_accum(int P, const int32_t *radii, const uint8_t *clamped, const float *accum,
                                    float *drgb, hipStream_t s);
hipError_t launch_sh_grad_from_colors(int P, int M, int nviews, int64_t view_stride, const float *means3D,
                                      const float *records, float *dsh_dc, float *dsh_rest, hipStream_t s);

// train_ops.hip
size_t l1_ssim_scratch_floats(int C, int H, int W);
hipError_t launch_l1_ssim(const float *x, const float *y, int C, int H, int W, float lambda, float *grad,
                          float *partials, float *out, hipStream_t s);
hipError_t launch_l1_grad(const float *x, const float *y, size_t n, const float *dloss, float *grad, hipStream_t s);
hipError_t launch_l1_finish(const float *x, const float *y, size_t n, float *partials, int nb, bool from_xy,
                            float *out, hipStream_t s);
hipError_t launch_adam(const gsr_adam_segment *segs, int nseg, int step, double beta1, double beta2, double eps,
                       hipStream_t s);
hipError_t launch_densify_stats(int P, const int32_t *radii, const float *vgrad, int vstride, float *max_radii,
                                float *grad_accum, float *denom, hipStream_t s);

// knn.hip
size_t knn_scratch_bytes(int P);
hipError_t launch_knn(int P, const float *pts, float *dist2, void *scratch, uint32_t *pinned6, hipStream_t s);

}  // namespace gsr

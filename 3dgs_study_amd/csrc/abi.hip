// abi.hip — the C ABI (include/gsr.h): argument checks, orchestration of the
// kernel launches on the caller's stream, error reporting.
//
// Mirrors upstream rasterize_points.cu (RasterizeGaussiansCUDA,
// RasterizeGaussiansBackwardCUDA, markVisible) and Rasterizer::forward /
// Rasterizer::backward (rasterizer_impl.cu).  No device allocation happens
// here: every buffer belongs to the caller (torch's caching allocator on the
// Python side).  The only host synchronisation is the num_rendered read-back
// in gsr_forward_preprocess, as upstream.
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "gsr_kernels.hpp"

using namespace gsr;

namespace {

thread_local std::string g_err;
// Per host thread: pinned words the preprocess launch publishes num_rendered into
// (the call waits for that launch's event before returning, so calls from one
// thread never share them in flight).
thread_local uint32_t *g_pinned = nullptr;

// geom buffers whose last forward prepared the backward (GSR_FLAG_PREPARE_BACKWARD:
// accumulator zeroed, quadrants filed) and that no backward has used since: the
// first backward then skips its bwd_prepare launch (the kernel would only read the
// flag words and return).  Host-side, in call order; a forward_preprocess on the
// buffer forgets it.  Shared by all threads (autograd runs the backward on its own
// thread).  Anything not in the set takes the launch, so the set is only a hint.
std::mutex g_prep_mu;
std::unordered_set<const void *> g_prepared;
void prepared_set(const void *geom, bool on) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    if (!on) {
        g_prepared.erase(geom);
        return;
    }
    if (g_prepared.size() > 4096) g_prepared.clear();  // forwards whose backward never came
    g_prepared.insert(geom);
}
bool prepared_take(const void *geom) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    return g_prepared.erase(geom) != 0;
}
// binning buffers whose last forward recorded its chunk cull masks for the backward
// (render_fwd with GSR_FLAG_PREPARE_BACKWARD), with the buffer's capacity (the
// masks' place in it): every forward into a buffer records or forgets it, and a
// backward finds the masks only for the buffer its forward wrote.  Without a
// record the backward culls itself (same entries, same pairs).
// The record also holds the split replay's SEG of that forward (0: no checkpoints).
std::unordered_map<const void *, std::pair<int64_t, int>> g_qmask;
void qmask_set(const void *binning, int64_t cap, int seg) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    if (cap <= 0) {
        g_qmask.erase(binning);
        return;
    }
    if (g_qmask.size() > 4096) g_qmask.clear();
    g_qmask[binning] = {cap, seg};
}
int64_t qmask_get(const void *binning) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    const auto it = g_qmask.find(binning);
    return it == g_qmask.end() ? 0 : it->second.first;
}
int split_get(const void *binning) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    const auto it = g_qmask.find(binning);
    return it == g_qmask.end() ? 0 : it->second.second;
}
// Split replay (gsr_split_mode; gsr_common.hpp): -1 automatic SEG, 0 off, > 0 that SEG
std::atomic<int> g_split_mode{-1};
// Colour apart (gsr_colour_mode, opt-in): preprocess's colour half on a side stream of
// this host thread and device, forked after the geometry half and joined before the
// blend.  Measured slower, so off by default: the side queue's kernels and the
// cross-queue waits opened ~35-40 us gaps in the binning chain (config B graph
// replays 4,786 -> 2,000-2,380 it/s, C 1,472 -> 1,016-1,026).
std::atomic<int> g_colour_mode{0};
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
thread_local SideStream g_side[64];
static SideStream *side_stream() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    SideStream &ss = g_side[dev];
    if (!ss.s) {
        int least = 0, greatest = 0;  // the side stream at the lowest priority: the binning chain's
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);  // kernels take the CUs first
        if (hipStreamCreateWithPriority(&ss.s, hipStreamNonBlocking, least) != hipSuccess ||
            hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&ss.join, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
            ss.s = nullptr;
            return nullptr;
        }
    }
    return &ss;
}
// the host's time inside the forward's num_rendered wait (gsr_host_wait_us: the
// benchmark separates the host's own work per step from its waiting on the device)
std::atomic<int64_t> g_wait_ns{0};
// img buffers whose last forward wrote sign(image - gt) beside the L1 loss's partial
// sums (gsr_forward_render_l1 with GSR_FLAG_PREPARE_BACKWARD), with the image and
// target it compared: an L1-seeded backward of that pair reads the signs (3 B per
// pixel) instead of both images (24 B).
std::unordered_map<const void *, std::pair<const float *, const float *>> g_l1sign;
void l1sign_set(const void *img, const float *image, const float *gt) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    if (!image) {
        g_l1sign.erase(img);
        return;
    }
    if (g_l1sign.size() > 4096) g_l1sign.clear();
    g_l1sign[img] = {image, gt};
}
bool l1sign_has(const void *img, const float *image, const float *gt) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    const auto it = g_l1sign.find(img);
    return it != g_l1sign.end() && it->second.first == image && it->second.second == gt;
}
// Binning form (gsr_binning_mode): 0 = the row-span binning (rowspan.hip) wherever
// the tile grid allows it (at most 256 x 256 tiles), 1 = the LSD tile sort of
// binning.hip everywhere.  The form of each geom buffer's last preprocess is
// recorded, so its render uses the rank gather's matching outputs.
// With the rect footprint the row-span binning also has the depth sort carry each
// Gaussian's rect word beside its id (RS_CARRY; binning.hip), so nothing gathers the
// rects in rank order.
enum BinForm { BIN_LSD = 0, BIN_ROWSPAN = 1, BIN_ROWSPAN_CARRY = 2 };
std::atomic<int> g_binning_mode{0};
std::unordered_map<const void *, int> g_rowspan;
#ifndef GSR_RS_CARRY
#define GSR_RS_CARRY 1  // (0: a timing build whose rect footprint gathers the rects like the tight one)
#endif
int binform_wanted(const gsr_inputs *in) {
    if (g_binning_mode.load() != 0 || !rowspan_grid(in->W, in->H)) return BIN_LSD;
    return in->footprint == GSR_FOOTPRINT_RECT && GSR_RS_CARRY ? BIN_ROWSPAN_CARRY : BIN_ROWSPAN;
}
void binform_set(const void *geom, int form) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    if (g_rowspan.size() > 4096) g_rowspan.clear();
    g_rowspan[geom] = form;
}
int binform_get(const void *geom, const gsr_inputs *in) {
    std::lock_guard<std::mutex> lk(g_prep_mu);
    const auto it = g_rowspan.find(geom);
    return it == g_rowspan.end() ? binform_wanted(in) : it->second;
}
// the num_rendered read-back's event (per host thread, like g_pinned): timing off
// and no system-scope fence — the pinned words are written with system-scope stores
// already, and a fenced event's cache writeback / invalidate opened a ~6 us idle gap
// before the next kernel (round 4 profile, before rank_gather_kernel)
thread_local hipEvent_t g_ctrl_ready = nullptr;
// the last forward's depth-sort pass count (per host thread): 4 queues the fourth
// pass up front (it returns at once when three suffice), so a scene whose depths
// span more than 2^24 key steps keeps gsr_forward's speculation
thread_local bool g_four_hint = false;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int check_hip(hipError_t e, const char *what) {
    if (e != hipSuccess) return fail(GSR_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return GSR_OK;
}

// Optional per-stage timing with HIP events recorded on the launch stream
// (bench.py reads it to price the dominant kernel against the HBM roofline).
struct StageTimer {
    int mask = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    std::vector<int> stage;  // stage of each used pair
    size_t used = 0;
    double total_ms[GSR_STAGE_COUNT] = {};
    int64_t launches[GSR_STAGE_COUNT] = {};
    // gsr_timing_sample: events on every `every`-th launch of a stage only (each
    // event pair is a marker packet with a ~4 us idle gap behind it)
    int every = 1;
    int64_t seen[GSR_STAGE_COUNT] = {};
    bool sampled[GSR_STAGE_COUNT] = {};
};
StageTimer g_timer;  // the ABI is driven from one host thread per process
size_t g_open[GSR_STAGE_COUNT];  // gsr_timing_begin: the pool slot whose end event is pending, + 1

const char *kStageNames[GSR_STAGE_COUNT] = {"preprocess", "scan",           "depth_sort",  "duplicate",
                                            "tile_sort",  "render_fwd",     "render_bwd",  "preprocess_bwd",
                                            "bwd_prepare", "exchange_wait", "sh_rebuild",  "colour"};

// st | TIMED_MORE: more work of a stage already counted once in this step (its
// time is added, its launch count is not)
constexpr int TIMED_MORE = 0x100;
// The next pool pair for stage st (created on first use).  Timing-only events: no
// system-scope fence on record (a default event's cache writeback / invalidate
// opened a ~6 us idle gap before the next kernel and cooled its caches); the
// elapsed time is read after a stream sync.
hipError_t take_pair(int st, std::pair<hipEvent_t, hipEvent_t> **out) {
    if (g_timer.used == g_timer.pool.size()) {
        hipEvent_t a, b;
        hipError_t e = hipEventCreateWithFlags(&a, hipEventDisableSystemFence);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b, hipEventDisableSystemFence);
        if (e != hipSuccess) return e;
        g_timer.pool.emplace_back(a, b);
        g_timer.stage.push_back(st);
    }
    *out = &g_timer.pool[g_timer.used];
    g_timer.stage[g_timer.used] = st;
    g_timer.used++;
    return hipSuccess;
}

template <typename F>
hipError_t timed(int st, hipStream_t s, F &&launch) {
    if (!(g_timer.mask & (1 << (st & 0xff)))) return launch();
    const int k = st & 0xff;
    if (!(st & TIMED_MORE)) g_timer.sampled[k] = g_timer.seen[k]++ % g_timer.every == 0;
    if (!g_timer.sampled[k]) return launch();  // (more work of an unsampled launch: unsampled too)
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    hipError_t e = take_pair(st, &ev);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ev->first, s);
    if (e != hipSuccess) return e;
    e = launch();
    if (e != hipSuccess) return e;
    return hipEventRecord(ev->second, s);
}

// upstream debug mode: synchronise and check after every kernel
int step(hipError_t e, const char *what, bool debug, hipStream_t s) {
    int rc = check_hip(e, what);
    if (rc || !debug) return rc;
    return check_hip(hipStreamSynchronize(s), what);
}

int validate(const gsr_inputs *in, bool forward) {
    if (!in) return fail(GSR_ERR_ARGS, "inputs is NULL");
    if (in->P < 0) return fail(GSR_ERR_ARGS, "means3D must have dimensions (num_points, 3)");
    if (in->W <= 0 || in->H <= 0) return fail(GSR_ERR_ARGS, "image size must be positive (got %dx%d)", in->W, in->H);
    if ((int64_t)in->W * in->H > (int64_t)1 << 30 || in->W > 65535 * TILE_X || in->H > 65535 * TILE_Y)
        return fail(GSR_ERR_CAPACITY, "image too large");
    if (in->footprint != GSR_FOOTPRINT_RECT && in->footprint != GSR_FOOTPRINT_TIGHT)
        return fail(GSR_ERR_ARGS, "footprint must be GSR_FOOTPRINT_RECT or GSR_FOOTPRINT_TIGHT (got %d)", in->footprint);
    if (in->flags & ~(GSR_FLAG_PREPARE_BACKWARD | GSR_FLAG_L1_SEED | GSR_FLAG_NO_WAIT)) return fail(GSR_ERR_ARGS, "unknown flags 0x%x", in->flags);
    if (forward && (in->flags & GSR_FLAG_L1_SEED)) return fail(GSR_ERR_ARGS, "GSR_FLAG_L1_SEED is a backward flag");
    if (in->activations & ~(GSR_ACT_OPACITY | GSR_ACT_SCALE | GSR_ACT_ROTATION))
        return fail(GSR_ERR_ARGS, "unknown activations 0x%x", in->activations);
    if (in->P == 0) return GSR_OK;
    if (!in->means3D || !in->viewmatrix || !in->projmatrix || !in->bg || (forward && !in->opacities))
        return fail(GSR_ERR_ARGS, "missing required input (means3D/opacities/viewmatrix/projmatrix/bg)");
    if ((in->sh == nullptr) == (in->colors_precomp == nullptr))
        return fail(GSR_ERR_ARGS, "Please provide excatly one of either SHs or precomputed colors!");
    const bool have_sr = in->scales && in->rotations;
    if (have_sr == (in->cov3D_precomp != nullptr))
        return fail(GSR_ERR_ARGS,
                    "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (in->sh) {
        if (!in->campos) return fail(GSR_ERR_ARGS, "campos required with SH colours");
        if (in->D < 0 || in->D > 3) return fail(GSR_ERR_ARGS, "sh_degree must be in [0, 3] (got %d)", in->D);
        if (in->M < (in->D + 1) * (in->D + 1))
            return fail(GSR_ERR_ARGS, "sh has %d coefficients per channel, degree %d needs %d", in->M, in->D,
                        (in->D + 1) * (in->D + 1));
    }
    if (in->sh_rest && (!in->sh || in->M < 2))
        return fail(GSR_ERR_ARGS, "sh_rest needs sh (the DC coefficients) and M >= 2");
    return GSR_OK;
}

}  // namespace

extern "C" {

size_t gsr_geom_bytes(int32_t P, int32_t W, int32_t H) { return geom_layout(P, W, H).bytes; }
size_t gsr_binning_bytes(int64_t num_rendered, int32_t W, int32_t H) {
    return binning_layout(num_rendered, W, H).bytes;
}
size_t gsr_img_bytes(int32_t W, int32_t H) { return img_layout(W, H).bytes; }
size_t gsr_accum_bytes(int32_t P) { return (size_t)(P > 0 ? P : 1) * ACCUM_STRIDE * sizeof(float); }

int gsr_geom_layout(int32_t P, int32_t W, int32_t H, size_t *offsets, int cap) {
    const GeomLayout L = geom_layout(P, W, H);
    int n = 0;
    for (; n < cap && n < GSR_GEOM_NFIELDS; n++) offsets[n] = L.off[n];
    return n;
}
int gsr_binning_layout(int64_t num_rendered, int32_t W, int32_t H, size_t *offsets, int cap) {
    const BinningLayout L = binning_layout(num_rendered, W, H);
    int n = 0;
    for (; n < cap && n < GSR_BIN_NFIELDS; n++) offsets[n] = L.off[n];
    return n;
}
int gsr_img_layout(int32_t W, int32_t H, size_t *offsets, int cap) {
    const ImgLayout L = img_layout(W, H);
    int n = 0;
    for (; n < cap && n < GSR_IMG_NFIELDS; n++) offsets[n] = L.off[n];
    return n;
}

int gsr_point_list_keys(int32_t P, int32_t W, int32_t H, const void *geom, const void *binning,
                        int64_t num_rendered, uint64_t *keys, void *stream) {
    if (P < 0 || W <= 0 || H <= 0 || num_rendered < 0) return fail(GSR_ERR_ARGS, "point_list_keys: bad sizes");
    if (num_rendered == 0) return GSR_OK;
    if (!geom || !binning || !keys) return fail(GSR_ERR_ARGS, "point_list_keys: NULL buffer");
    return check_hip(launch_point_list_keys(P, W, H, geom, binning, num_rendered, keys, (hipStream_t)stream),
                     "point_list_keys");
}

int gsr_binning_mode(int mode) {
    if (mode < -1 || mode > 1) {
        fail(GSR_ERR_ARGS, "binning mode %d: 0 (row spans where possible), 1 (LSD tile sort) or -1 (query)", mode);
        return -1;
    }
    return mode < 0 ? g_binning_mode.load() : g_binning_mode.exchange(mode);
}

double gsr_host_wait_us(int reset) {
    const int64_t ns = reset ? g_wait_ns.exchange(0) : g_wait_ns.load();
    return (double)ns * 1e-3;
}

int gsr_colour_mode(int mode) {
    if (mode == -2) return g_colour_mode.load();
    if (mode != 0 && mode != 1 && mode != 2) {
        fail(GSR_ERR_ARGS,
             "colour mode %d: 2 (colour half riding the depth sort), 1 (on a side stream), 0 (fused) or -2 (query)",
             mode);
        return -3;
    }
    return g_colour_mode.exchange(mode);
}

int gsr_split_mode(int mode) {
    if (mode == -2) return g_split_mode.load();
    if (mode < -1 || mode > 65536) {
        fail(GSR_ERR_ARGS, "split mode %d: -1 (automatic), 0 (off), a segment length in list entries, or -2 (query)",
             mode);
        return -3;
    }
    return g_split_mode.exchange(mode);
}

const char *gsr_last_error(void) { return g_err.c_str(); }
int gsr_abi_version(void) { return GSR_ABI_VERSION; }

#ifndef GSR_BUILD_ID
#define GSR_BUILD_ID "unknown"
#endif
const char *gsr_build_id(void) { return GSR_BUILD_ID; }

static int ensure_pinned() {
    if (g_pinned) return GSR_OK;
    // coherent: the kernel's system-scope stores land in host memory directly
    if (int rc = check_hip(hipHostMalloc((void **)&g_pinned, CTRL_WORDS * 4, hipHostMallocCoherent), "hipHostMalloc"))
        return rc;
    return check_hip(hipEventCreateWithFlags(&g_ctrl_ready, hipEventDisableTiming | hipEventDisableSystemFence),
                     "hipEventCreate");
}

// Preprocess, the depth sort (its first digit scan publishes num_rendered and the
// pass count into the pinned words), the read-back event and the rank-order gather:
// queued, not waited for.  passes: the depth passes queued (3, or 4 up front).
static int queue_preprocess(const gsr_inputs *in, void *geom, int32_t *radii, int passes, hipStream_t s, bool dbg,
                            bool wait_event = true, hipEvent_t *colour_join = nullptr) {
    prepared_set(geom, false);  // preprocess resets the device's flag words too
    const int form = binform_wanted(in);
    binform_set(geom, form);
    const bool rowspan = form != BIN_LSD, carry = form == BIN_ROWSPAN_CARRY;
    if (int rc = ensure_pinned()) return rc;
    g_pinned[CTRL_NUM_RENDERED_LO] = g_pinned[CTRL_NUM_RENDERED_HI] = g_pinned[CTRL_PREFILTER_ERR] = 0;
    g_pinned[CTRL_DSORT_PASSES] = 0;
    // colour apart: the geometry half here, the colour half on the side stream (its
    // join event goes back to the caller, who waits on it before the blend)
    SideStream *side = nullptr;
    if (colour_join && !dbg && g_colour_mode.load() == 1 && in->sh && !in->colors_precomp) side = side_stream();
    if (colour_join) *colour_join = nullptr;
    // colour riding: the colour half runs as extra workgroups of the depth sort's
    // downsweeps (binning.hip), in stream order — no second queue
    ColourRide ride{};
    const bool riding = !side && g_colour_mode.load() == 2 && colour_ride_plan(*in, geom, radii, &ride);
    if (int rc = step(timed(GSR_STAGE_PREPROCESS, s,
                            [&] {
                                return launch_preprocess(*in, geom, radii, carry, s,
                                                         side || riding ? PRE_PHASE_GEOM : PRE_PHASE_FUSED);
                            }),
                      "preprocess", dbg, s))
        return rc;
    if (side) {
        if (int rc = check_hip(hipEventRecord(side->fork, s), "colour fork")) return rc;
        if (int rc = check_hip(hipStreamWaitEvent(side->s, side->fork, 0), "colour fork")) return rc;
        if (int rc = check_hip(timed(GSR_STAGE_COLOUR, side->s,
                                     [&] { return launch_preprocess(*in, geom, radii, carry, side->s, PRE_PHASE_COLOUR); }),
                               "preprocess colour"))
            return rc;
        if (int rc = check_hip(hipEventRecord(side->join, side->s), "colour join")) return rc;
        *colour_join = side->join;
    }
    // the sort needs only the view depths; after preprocess, so that its first digit
    // scan can also publish num_rendered (one launch fewer than a publish kernel)
    if (int rc = step(timed(GSR_STAGE_DEPTH_SORT, s,
                            [&] {
                                return launch_depth_sort(in->P, in->W, in->H, in->means3D, in->viewmatrix, geom,
                                                         passes, g_pinned, carry, s, riding ? &ride : nullptr);
                            }),
                      "depth sort", dbg, s))
        return rc;
    if (wait_event)
        if (int rc = check_hip(hipEventRecord(g_ctrl_ready, s), "num_rendered read-back")) return rc;
    // the rects in rank order and the emission offsets (upstream's InclusiveSum of
    // tiles_touched, in depth order), queued before the host waits: the device stays
    // busy (with three passes queued it returns at once if the keys need four)
    return step(timed(GSR_STAGE_SCAN, s,
                      [&] { return launch_rank_gather(in->P, in->W, in->H, geom, passes == 3, rowspan, carry, s); }),
                "rank gather", dbg, s);
}

// The host's one wait: num_rendered and the pass count.  When only three depth
// passes were queued and the keys need four, the fourth pass and the rank gather
// are queued now (*late).
static int finish_preprocess(const gsr_inputs *in, void *geom, int passes, hipStream_t s, bool dbg, int64_t *I,
                             bool *late) {
    const auto w0 = std::chrono::steady_clock::now();
    const hipError_t we = hipEventSynchronize(g_ctrl_ready);
    g_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
    if (int rc = check_hip(we, "num_rendered read-back")) return rc;
    if (g_pinned[CTRL_PREFILTER_ERR])
        return fail(GSR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    const bool four = g_pinned[CTRL_DSORT_PASSES] != 3u;
    g_four_hint = four;
    *late = four && passes == 3;
    if (*late) {
        // the keys span more than 2^24: the fourth pass, then the rank gather the
        // queued one skipped (rank_gather_kernel returns at once on a four-pass sort)
        if (int rc = step(timed(GSR_STAGE_DEPTH_SORT | TIMED_MORE, s,
                                [&] {
                                    return launch_depth_sort_fourth(in->P, in->W, in->H, geom,
                                                                    binform_get(geom, in) == BIN_ROWSPAN_CARRY, s);
                                }),
                          "depth sort (fourth pass)", dbg, s))
            return rc;
        if (int rc = step(timed(GSR_STAGE_SCAN | TIMED_MORE, s,
                                [&] {
                                    const int f = binform_get(geom, in);
                                    return launch_rank_gather(in->P, in->W, in->H, geom, false, f != BIN_LSD,
                                                              f == BIN_ROWSPAN_CARRY, s);
                                }),
                          "rank gather", dbg, s))
            return rc;
    }
    *I = (int64_t)g_pinned[CTRL_NUM_RENDERED_LO] | ((int64_t)g_pinned[CTRL_NUM_RENDERED_HI] << 32);
    if (*I > 0xFFFFFFFFll) return fail(GSR_ERR_CAPACITY, "num_rendered %lld exceeds 32-bit list indexing", (long long)*I);
    return GSR_OK;
}

int gsr_forward_preprocess(const gsr_inputs *in, void *geom, int32_t *radii, int64_t *num_rendered, void *stream) {
    if (int rc = validate(in, true)) return rc;
    if (!num_rendered) return fail(GSR_ERR_ARGS, "num_rendered is NULL");
    *num_rendered = 0;
    if (in->P == 0) return GSR_OK;
    if (!geom || !radii) return fail(GSR_ERR_ARGS, "geom/radii buffers are NULL");
    hipStream_t s = (hipStream_t)stream;
    const bool dbg = in->debug != 0;
    const int passes = g_four_hint ? 4 : 3;
    if (int rc = queue_preprocess(in, geom, radii, passes, s, dbg)) return rc;
    bool late = false;
    return finish_preprocess(in, geom, passes, s, dbg, num_rendered, &late);
}

// P == 0: upstream returns the zero-initialised image untouched
static int render_empty(const gsr_inputs *in, void *img, float *out_color, const float *gt, float *loss_out,
                        hipStream_t s) {
    const size_t npix = (size_t)3 * in->W * in->H;
    if (int rc = check_hip(hipMemsetAsync(out_color, 0, npix * sizeof(float), s), "memset")) return rc;
    if (!gt) return GSR_OK;
    float *l1_part = at<float>(img, img_layout(in->W, in->H).l1_part);
    return step(launch_l1_finish(out_color, gt, npix, l1_part, 0, true, loss_out, s), "l1 loss", in->debug != 0, s);
}

// Emit and the tile sort of n instances into a binning buffer of capacity cap (g:
// speculative, then n = cap and the kernels take the published count), then the
// blend, the backward's preparation and the L1 loss.
static int queue_render(const gsr_inputs *in, void *geom, void *binning, int64_t n, int64_t cap, const SpecGuard &g,
                        void *img, const int32_t *radii, float *out_color, const float *gt, float *loss_out,
                        uint8_t *visible_out, hipStream_t s, bool dbg, hipEvent_t colour_join = nullptr) {
    const size_t npix = (size_t)3 * in->W * in->H;
    float *l1_part = gt ? at<float>(img, img_layout(in->W, in->H).l1_part) : nullptr;
    const int form = binform_get(geom, in);
    if (n > 0 && form != BIN_LSD) {
        // row-span binning: pass A (spans by tile row), pass B (tiles by column)
        if (int rc = step(timed(GSR_STAGE_DUPLICATE, s,
                                [&] {
                                    return launch_rowspan_a(in->P, in->W, in->H, geom, binning, cap, g,
                                                            form == BIN_ROWSPAN_CARRY, s);
                                }),
                          "row spans", dbg, s))
            return rc;
        if (int rc = step(timed(GSR_STAGE_TILE_SORT, s,
                                [&] { return launch_rowspan_b(in->P, in->W, in->H, geom, binning, cap, g, s); }),
                          "tile columns", dbg, s))
            return rc;
    } else if (n > 0) {
        if (int rc = step(timed(GSR_STAGE_DUPLICATE, s,
                                [&] { return launch_emit(in->P, in->W, in->H, geom, binning, cap, g, s); }),
                          "duplicateWithKeys", dbg, s))
            return rc;
        if (int rc = step(timed(GSR_STAGE_TILE_SORT, s,
                                [&] { return launch_tile_sort(in->P, in->W, in->H, geom, binning, n, cap, g, s); }),
                          "tile sort", dbg, s))
            return rc;
    }  // else every range stays (0, 0) as preprocess left it
    // GSR_FLAG_PREPARE_BACKWARD: render_fwd zeroes the backward's accumulator beside
    // its blend, and the quadrants are filed after it, so the backward starts with
    // render_bwd
    const bool prep = (in->flags & GSR_FLAG_PREPARE_BACKWARD) != 0;
    const GeomLayout G = geom_layout(in->P, in->W, in->H);
    void *acc = at<void>(geom, G.accum);
    const size_t acc_bytes = (size_t)in->P * ACCUM_STRIDE * sizeof(float);
    // the split replay's SEG (0: none), for the lists this forward bins into cap
    const int seg = prep && n > 0 ? split_seg(cap, g_split_mode.load()) : 0;
    // the colour half (side stream) lands before the blend reads the records
    if (colour_join)
        if (int rc = check_hip(hipStreamWaitEvent(s, colour_join, 0), "colour join")) return rc;
    if (int rc = step(timed(GSR_STAGE_RENDER_FWD, s,
                            [&] {
                                return launch_render_fwd(*in, geom, n > 0 ? binning : nullptr, img, out_color,
                                                         prep ? (float *)acc : nullptr, acc_bytes, s,
                                                         prep && n > 0 ? cap : 0, seg);
                            }),
                      "render", dbg, s))
        return rc;
    if (binning) qmask_set(binning, prep && n > 0 ? cap : 0, seg);
    l1sign_set(img, prep && gt ? out_color : nullptr, gt);
    if (!prep) {  // the L1 loss, if asked for, on its own
        prepared_set(geom, false);
        return gt ? step(launch_l1_finish(out_color, gt, npix, l1_part, 0, true, loss_out, s), "l1 loss", dbg, s)
                  : GSR_OK;
    }
    // the L1 loss (partial sums and finish) rides in the same launch as the quadrant filing
    if (int rc = step(launch_bwd_prepare(*in, geom, img, (float *)acc, n > 0, true, true, s, gt ? out_color : nullptr,
                                         gt, loss_out, radii, visible_out),
                      "backward prepare", dbg, s))
        return rc;
    prepared_set(geom, true);
    return GSR_OK;
}

static int check_render_args(const gsr_inputs *in, void *img, const int32_t *radii, float *out_color, const float *gt,
                             float *loss_out, uint8_t *visible_out) {
    if (!out_color) return fail(GSR_ERR_ARGS, "out_color is NULL");
    if (gt && (!loss_out || !img)) return fail(GSR_ERR_ARGS, "l1: loss_out and img required");
    if (visible_out && !gt) return fail(GSR_ERR_ARGS, "visible_out needs gt (the L1 form)");
    if (visible_out && !(in->flags & GSR_FLAG_PREPARE_BACKWARD))
        return fail(GSR_ERR_ARGS, "visible_out needs GSR_FLAG_PREPARE_BACKWARD");
    if (visible_out && !radii && in->P > 0) return fail(GSR_ERR_ARGS, "visible_out needs radii");
    return GSR_OK;
}

static int forward_render_impl(const gsr_inputs *in, void *geom, void *binning, void *img, int64_t num_rendered,
                               const int32_t *radii, float *out_color, const float *gt, float *loss_out,
                               uint8_t *visible_out, void *stream) {
    if (int rc = validate(in, true)) return rc;
    if (int rc = check_render_args(in, img, radii, out_color, gt, loss_out, visible_out)) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (in->P == 0) return render_empty(in, img, out_color, gt, loss_out, s);
    if (!geom || !img || (num_rendered > 0 && !binning)) return fail(GSR_ERR_ARGS, "scratch buffers are NULL");
    if (num_rendered < 0 || num_rendered > 0xFFFFFFFFll) return fail(GSR_ERR_ARGS, "num_rendered out of range");
    return queue_render(in, geom, binning, num_rendered, num_rendered, SpecGuard{}, img, radii, out_color, gt,
                        loss_out, visible_out, s, in->debug != 0);
}

int gsr_forward_render(const gsr_inputs *in, void *geom, void *binning, void *img, int64_t num_rendered,
                       const int32_t *radii, float *out_color, void *stream) {
    return forward_render_impl(in, geom, binning, img, num_rendered, radii, out_color, nullptr, nullptr, nullptr,
                               stream);
}

int gsr_forward_render_l1(const gsr_inputs *in, void *geom, void *binning, void *img, int64_t num_rendered,
                          const int32_t *radii, float *out_color, const float *gt, float *loss_out,
                          uint8_t *visible_out, void *stream) {
    if (!gt) return fail(GSR_ERR_ARGS, "gt is NULL");
    return forward_render_impl(in, geom, binning, img, num_rendered, radii, out_color, gt, loss_out, visible_out,
                               stream);
}

int gsr_forward(const gsr_inputs *in, void *geom, int32_t *radii, void *binning, int64_t capacity, void *img,
                float *out_color, const float *gt, float *loss_out, uint8_t *visible_out, int64_t *num_rendered,
                void *stream) {
    if (int rc = validate(in, true)) return rc;
    if (!num_rendered) return fail(GSR_ERR_ARGS, "num_rendered is NULL");
    *num_rendered = 0;
    if (int rc = check_render_args(in, img, radii, out_color, gt, loss_out, visible_out)) return rc;
    if (capacity < 0 || capacity > 0xFFFFFFFFll) return fail(GSR_ERR_ARGS, "binning capacity out of range");
    hipStream_t s = (hipStream_t)stream;
    if (in->P == 0) return render_empty(in, img, out_color, gt, loss_out, s);
    if (!geom || !radii || !img || (capacity > 0 && !binning)) return fail(GSR_ERR_ARGS, "scratch buffers are NULL");
    const bool dbg = in->debug != 0;
    // GSR_FLAG_NO_WAIT (stream capture): the depth passes the last forward needed
    // (gsr_depth_passes_hint), nothing read back; gsr_forward_status checks the
    // device's count and pass count once the work has run
    const bool nowait = (in->flags & GSR_FLAG_NO_WAIT) != 0;
    if (nowait && (dbg || capacity <= 0))
        return fail(GSR_ERR_ARGS, "GSR_FLAG_NO_WAIT needs a binning capacity and debug off");
    const int passes = g_four_hint ? 4 : 3;
    hipEvent_t join = nullptr;  // the colour half's (gsr_colour_mode), until a blend waits on it
    if (int rc = queue_preprocess(in, geom, radii, passes, s, dbg, !nowait, &join)) return rc;
    // every path out of here leaves the caller's stream after the colour half
    auto joined = [&](int rc) {
        if (join) {
            if (int e = check_hip(hipStreamWaitEvent(s, join, 0), "colour join")) return rc ? rc : e;
            join = nullptr;
        }
        return rc;
    };
    // Speculative: everything after the depth sort is queued before the host reads
    // num_rendered, into the caller's buffer of `capacity` instances; each binning
    // kernel checks the published count on the device and does nothing unless it
    // fits (SpecGuard).  Debug mode checks every kernel in turn instead.
    const bool spec = !dbg && capacity > 0;
    if (spec) {
        const GeomLayout G = geom_layout(in->P, in->W, in->H);
        const SpecGuard g{at<const uint32_t>(geom, G.off[GSR_GEOM_CTRL]), at<const uint32_t>(geom, G.dsort_ctrl),
                          (uint32_t)capacity, passes == 3 ? 1 : 0};
        if (int rc = queue_render(in, geom, binning, capacity, capacity, g, img, radii, out_color, gt, loss_out,
                                  visible_out, s, dbg, join))
            return rc;
        join = nullptr;  // the blend waited on it
    }
    if (nowait) {
        *num_rendered = capacity;
        return joined(GSR_OK);
    }
    int64_t I = 0;
    bool late = false;
    if (int rc = finish_preprocess(in, geom, passes, s, dbg, &I, &late)) return joined(rc);
    *num_rendered = I;
    if (I > capacity) {
        fail(GSR_NEED_BINNING, "binning capacity %lld < num_rendered %lld: call gsr_forward_render with a buffer of "
             "gsr_binning_bytes(num_rendered)", (long long)capacity, (long long)I);
        return joined(GSR_NEED_BINNING);
    }
    if (spec && !late) return GSR_OK;
    // debug mode, or the fourth depth pass queued only now: the rest, exactly
    const hipEvent_t j = join;
    join = nullptr;
    return queue_render(in, geom, binning, I, capacity, SpecGuard{}, img, radii, out_color, gt, loss_out, visible_out,
                        s, dbg, j);
}

int gsr_depth_passes_hint(void) { return g_four_hint ? 4 : 3; }

int gsr_forward_status(int64_t capacity, int passes, int64_t *num_rendered) {
    if (!num_rendered) return fail(GSR_ERR_ARGS, "num_rendered is NULL");
    if (int rc = ensure_pinned()) return rc;
    const int64_t I = (int64_t)g_pinned[CTRL_NUM_RENDERED_LO] | ((int64_t)g_pinned[CTRL_NUM_RENDERED_HI] << 32);
    *num_rendered = I;
    if (g_pinned[CTRL_PREFILTER_ERR])
        return fail(GSR_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (passes == 3 && g_pinned[CTRL_DSORT_PASSES] == 4u)
        return fail(GSR_NEED_BINNING, "the depth keys need four sort passes, three were queued: the forward's lists "
                    "are incomplete (an eager forward sets the hint; capture again)");
    if (I > capacity)
        return fail(GSR_NEED_BINNING, "binning capacity %lld < num_rendered %lld: the forward's lists are incomplete",
                    (long long)capacity, (long long)I);
    return GSR_OK;
}

static int backward_impl(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                         const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                         float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                         float *drgb, float *dscales, float *drot, void *stream, int dsh_planar = 0,
                         int phases = 3, const gsr_leaf_grads *leaf = nullptr) {
    // phases: bit 0 = accumulator zeroing + render_bwd (+ the colour gradient into
    // drgb), bit 1 = preprocess_bwd, bit 2 = the colour gradient apart (below).  The
    // view-parallel exchange runs them as separate calls and starts its all-gather of
    // drgb in between.
    if (int rc = validate(in, false)) return rc;
    if (in->P == 0) return GSR_OK;
    if (!radii || !geom || !img || !dL_dout_color || (num_rendered > 0 && !binning))
        return fail(GSR_ERR_ARGS, "backward scratch/inputs are NULL");
    const gsr_leaf_grads L = leaf ? *leaf : gsr_leaf_grads{};
    if (L.dsh_dc && (!in->sh || in->M <= 0 || (in->M > 1 && !L.dsh_rest)))
        return fail(GSR_ERR_ARGS, "leaf dsh: needs sh and dsh_rest (M > 1)");
    if ((L.dscaling || L.drotation) && !in->scales) return fail(GSR_ERR_ARGS, "leaf dscaling/drotation: needs scales");
    if (L.drotation && (!in->rotations || (!L.rotation_norm && !(in->activations & GSR_ACT_ROTATION))))
        return fail(GSR_ERR_ARGS, "leaf drotation: needs rotations and rotation_norm (or GSR_ACT_ROTATION)");
    if (L.dopacity && !in->opacities) return fail(GSR_ERR_ARGS, "leaf dopacity: needs opacities");
    if (drgb && (dsh || L.dsh_dc)) return fail(GSR_ERR_ARGS, "drgb replaces dsh: dsh / leaf dsh must be NULL with it");
    const bool internal = accum == nullptr;  // geom's accumulator (GSR_FLAG_PREPARE_BACKWARD may have zeroed it)
    if (internal) accum = at<void>(const_cast<void *>(geom), geom_layout(in->P, in->W, in->H).accum);
    if (!dmeans2D || (!dcolors && in->colors_precomp) || (!dopacity && !L.dopacity) || !dmeans3D ||
        (!dcov3D && in->cov3D_precomp))
        return fail(GSR_ERR_ARGS, "backward outputs are NULL");
    if (in->sh && in->M > 0 && !dsh && !drgb && !L.dsh_dc) return fail(GSR_ERR_ARGS, "dsh is NULL");
    if (in->scales && ((!dscales && !L.dscaling) || (!drot && !L.drotation)))
        return fail(GSR_ERR_ARGS, "dscales/drot are NULL");
    hipStream_t s = (hipStream_t)stream;
    const bool dbg = in->debug != 0;
    float *acc = (float *)accum;
    const bool colors = drgb && in->sh && in->M > 0;
    // GSR_FLAG_L1_SEED: dL_dout_color is a gsr_l1_seed (the render backward forms
    // the L1 loss's pixel gradient itself)
    const gsr_l1_seed *seed = (in->flags & GSR_FLAG_L1_SEED) ? reinterpret_cast<const gsr_l1_seed *>(dL_dout_color) : nullptr;
    if (seed && (!seed->image || !seed->gt || !seed->dloss || seed->n != (int64_t)3 * in->W * in->H))
        return fail(GSR_ERR_ARGS, "l1 seed: image, gt and dloss required, n must be 3 W H = %lld (got %lld)",
                    (long long)3 * in->W * in->H, (long long)seed->n);
    if (phases & 1) {
        // zeroes the accumulator and files the quadrants for render_bwd's wave order,
        // unless this forward's prepare did both and no backward has run since
        if (!(internal && prepared_take(geom)))
            if (int rc = step(timed(GSR_STAGE_BWD_PREPARE, s, [&] { return launch_bwd_prepare(*in, const_cast<void *>(geom), img, acc, num_rendered > 0, internal, false, s); }),
                              "backward prepare", dbg, s))
                return rc;
        if (num_rendered > 0) {
            if (int rc = step(timed(GSR_STAGE_RENDER_BWD, s, [&] {
                                  return launch_render_bwd(*in, geom, binning, img, seed ? nullptr : dL_dout_color,
                                                           seed, acc, s, qmask_get(binning),
                                                           seed && l1sign_has(img, seed->image, seed->gt),
                                                           split_get(binning));
                              }),
                              "render backward", dbg, s))
                return rc;
        }
    }
    // the colour gradient: with the render half, unless GSR_PHASE_COLOURS_APART asks
    // for it in a call of its own (on the caller's exchange stream, beside the
    // per-Gaussian half); that bit without the render half is that call
    if (colors && ((phases & 1) != 0) == ((phases & 4) == 0)) {
        const GeomLayout G = geom_layout(in->P, in->W, in->H);
        if (int rc = step(launch_colors_from_accum(in->P, radii, at<uint8_t>(const_cast<void *>(geom), G.off[GSR_GEOM_CLAMPED]),
                                                   acc, drgb, s),
                          "colour gradient", dbg, s))
            return rc;
    }
    if (!(phases & 2)) return GSR_OK;
    // with the colour gradient taken by the exchange, preprocess_bwd still reads the
    // SH rows for dL/dmean3D's view-direction term but writes no dsh
    BwdOutputs o{dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, colors ? nullptr : dsh, dscales, drot, nullptr,
                 dsh_planar, colors ? 1 : 0, L};
    if (L.dsh_dc) o.dsh = nullptr;
    if (L.dscaling) o.dscales = nullptr;
    if (L.drotation) o.drot = nullptr;
    if (L.dopacity) o.dopacity = nullptr;
    return step(timed(GSR_STAGE_PREPROCESS_BWD, s, [&] { return launch_preprocess_bwd(*in, radii, geom, acc, o, s); }), "preprocess backward", dbg, s);
}

int gsr_backward(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning, const void *img,
                 int64_t num_rendered, const float *dL_dout_color, void *accum, float *dmeans2D, float *dcolors,
                 float *dopacity, float *dmeans3D, float *dcov3D, float *dsh, float *dscales, float *drot,
                 void *stream) {
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, dsh, nullptr, dscales, drot, stream);
}

int gsr_backward_leaves(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                        float *dscales, float *drot, const gsr_leaf_grads *leaf, void *stream) {
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, dsh, nullptr, dscales, drot, stream, leaf ? leaf->dsh_planar : 0, 3, leaf);
}

int gsr_backward_planar(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                        float *dscales, float *drot, void *stream) {
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, dsh, nullptr, dscales, drot, stream, 1);
}

int gsr_backward_colors(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *drgb,
                        float *dscales, float *drot, void *stream) {
    if (in && in->P > 0 && in->sh && in->M > 0 && !drgb) return fail(GSR_ERR_ARGS, "drgb is NULL");
    if (in && in->sh && in->D > 3) return fail(GSR_ERR_ARGS, "sh_degree > 3 is not supported");
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, nullptr, drgb, dscales, drot, stream);
}

int gsr_backward_phase(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                       const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                       float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *dsh,
                       float *drgb, float *dscales, float *drot, const gsr_leaf_grads *leaf, int32_t phases,
                       void *stream) {
    if (phases < 1 || phases > 7) return fail(GSR_ERR_ARGS, "phases must be 1 .. 7 (got %d)", phases);
    if (in && in->P > 0 && drgb && in->sh && in->D > 3) return fail(GSR_ERR_ARGS, "sh_degree > 3 is not supported");
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, dsh, drgb, dscales, drot, stream, leaf ? leaf->dsh_planar : 0,
                         phases, leaf);
}

static int colors_phase(int phases, const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                        const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                        float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D, float *drgb,
                        float *dscales, float *drot, void *stream) {
    if (in && in->P > 0 && in->sh && in->M > 0 && !drgb) return fail(GSR_ERR_ARGS, "drgb is NULL");
    if (in && in->sh && in->D > 3) return fail(GSR_ERR_ARGS, "sh_degree > 3 is not supported");
    return backward_impl(in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                         dopacity, dmeans3D, dcov3D, nullptr, drgb, dscales, drot, stream, 0, phases);
}

int gsr_backward_colors_render(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                               const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                               float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D,
                               float *drgb, float *dscales, float *drot, void *stream) {
    return colors_phase(1, in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                        dopacity, dmeans3D, dcov3D, drgb, dscales, drot, stream);
}

int gsr_backward_colors_finish(const gsr_inputs *in, const int32_t *radii, const void *geom, const void *binning,
                               const void *img, int64_t num_rendered, const float *dL_dout_color, void *accum,
                               float *dmeans2D, float *dcolors, float *dopacity, float *dmeans3D, float *dcov3D,
                               float *drgb, float *dscales, float *drot, void *stream) {
    return colors_phase(2, in, radii, geom, binning, img, num_rendered, dL_dout_color, accum, dmeans2D, dcolors,
                        dopacity, dmeans3D, dcov3D, drgb, dscales, drot, stream);
}

int64_t gsr_sh_record_floats(int32_t P) { return P < 0 ? -1 : 4 + (((int64_t)3 * P + 3) / 4) * 4; }

int gsr_sh_grad_from_colors(int32_t P, int32_t M, int32_t nviews, const float *means3D, const float *records,
                            float *dsh_dc, float *dsh_rest, void *stream) {
    if (P < 0 || nviews < 0) return fail(GSR_ERR_ARGS, "sh_grad_from_colors: negative size");
    if (M != 1 && M != 4 && M != 9 && M != 16) return fail(GSR_ERR_ARGS, "sh_grad_from_colors: M must be 1, 4, 9 or 16");
    if (P == 0) return GSR_OK;
    if (!means3D || !dsh_dc || (M > 1 && !dsh_rest) || (nviews > 0 && !records))
        return fail(GSR_ERR_ARGS, "sh_grad_from_colors: NULL pointer");
    hipStream_t s = (hipStream_t)stream;
    return check_hip(launch_sh_grad_from_colors(P, M, nviews, gsr_sh_record_floats(P), means3D, records, dsh_dc,
                                                dsh_rest, s),
                     "sh_grad_from_colors");
}

int gsr_mark_visible(int32_t P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_ARGS, "means3D must have dimensions (num_points, 3)");
    if (P == 0) return GSR_OK;
    if (!means3D || !viewmatrix || !present) return fail(GSR_ERR_ARGS, "mark_visible: NULL input");
    hipStream_t s = (hipStream_t)stream;
    return check_hip(launch_mark_visible(P, means3D, viewmatrix, present, s), "mark_visible");
}

size_t gsr_l1_ssim_scratch_bytes(int32_t C, int32_t H, int32_t W) {
    if (C <= 0 || H <= 0 || W <= 0) return 0;
    return l1_ssim_scratch_floats(C, H, W) * sizeof(float);
}

int gsr_l1_ssim(const float *img, const float *gt, int32_t C, int32_t H, int32_t W, float lambda_dssim,
                float *grad_img, void *scratch, float *loss_out, void *stream) {
    if (C <= 0 || H <= 0 || W <= 0) return fail(GSR_ERR_ARGS, "l1_ssim: empty image (%d x %d x %d)", C, H, W);
    if (!img || !gt || (!grad_img && lambda_dssim != 0.0f) || !scratch || !loss_out)
        return fail(GSR_ERR_ARGS, "l1_ssim: NULL buffer");
    return check_hip(launch_l1_ssim(img, gt, C, H, W, lambda_dssim, grad_img, (float *)scratch, loss_out,
                                    (hipStream_t)stream),
                     "l1_ssim");
}

int gsr_l1_grad(const float *img, const float *gt, int64_t n, const float *dloss, float *grad_img, void *stream) {
    if (n < 0) return fail(GSR_ERR_ARGS, "l1_grad: negative size");
    if (n == 0) return GSR_OK;
    if (!img || !gt || !dloss || !grad_img) return fail(GSR_ERR_ARGS, "l1_grad: NULL buffer");
    return check_hip(launch_l1_grad(img, gt, (size_t)n, dloss, grad_img, (hipStream_t)stream), "l1_grad");
}

int gsr_adam_step(const gsr_adam_segment *segs, int32_t nseg, int32_t step, double beta1, double beta2, double eps,
                  void *stream) {
    if (nseg < 0 || nseg > GSR_ADAM_MAX_SEGS) return fail(GSR_ERR_ARGS, "adam: %d segments (max %d)", nseg, GSR_ADAM_MAX_SEGS);
    if (step < 1) return fail(GSR_ERR_ARGS, "adam: step must be >= 1 (got %d)", step);
    for (int k = 0; k < nseg; k++)
        if (segs[k].n > 0 && (!segs[k].param || !segs[k].grad || !segs[k].exp_avg || !segs[k].exp_avg_sq))
            return fail(GSR_ERR_ARGS, "adam: NULL buffer in segment %d", k);
    return check_hip(launch_adam(segs, nseg, step, beta1, beta2, eps, (hipStream_t)stream), "adam");
}

int gsr_densify_stats(int32_t P, const int32_t *radii, const float *viewspace_grad, int32_t grad_stride,
                      float *max_radii2D, float *xyz_gradient_accum, float *denom, void *stream) {
    if (P < 0 || grad_stride < 2) return fail(GSR_ERR_ARGS, "densify_stats: bad P %d / stride %d", P, grad_stride);
    if (P > 0 && (!radii || !viewspace_grad || !max_radii2D || !xyz_gradient_accum || !denom))
        return fail(GSR_ERR_ARGS, "densify_stats: NULL buffer");
    return check_hip(launch_densify_stats(P, radii, viewspace_grad, grad_stride, max_radii2D, xyz_gradient_accum,
                                          denom, (hipStream_t)stream),
                     "densify_stats");
}

size_t gsr_knn_scratch_bytes(int32_t P) { return P > 0 ? knn_scratch_bytes(P) : 0; }

int gsr_knn_mean_dist2(int32_t P, const float *points, float *dist2, void *scratch, void *stream) {
    if (P < 0) return fail(GSR_ERR_ARGS, "knn: P must be >= 0 (got %d)", P);
    if (P == 0) return GSR_OK;
    if (!points || !dist2 || !scratch) return fail(GSR_ERR_ARGS, "knn: NULL buffer");
    if (int rc = ensure_pinned()) return rc;
    return check_hip(launch_knn(P, points, dist2, scratch, g_pinned, (hipStream_t)stream), "knn");
}

int gsr_timing_sample(int every) {
    if (every < 1) return fail(GSR_ERR_ARGS, "timing sample period must be >= 1 (got %d)", every);
    g_timer.every = every;
    for (auto &n : g_timer.seen) n = 0;
    return GSR_OK;
}

int gsr_timing_enable(int mask) {
    g_timer.mask = mask;
    g_timer.used = 0;
    for (auto &n : g_timer.seen) n = 0;
    for (auto &o : g_open) o = 0;
    for (int k = 0; k < GSR_STAGE_COUNT; k++) {
        g_timer.total_ms[k] = 0;
        g_timer.launches[k] = 0;
    }
    return GSR_OK;
}

int gsr_timing_read(double *total_ms, int64_t *launches, int cap) {
    for (size_t i = 0; i < g_timer.used; i++) {
        auto &ev = g_timer.pool[i];
        if (int rc = check_hip(hipEventSynchronize(ev.second), "timing event")) return -rc;
        float ms = 0.f;
        if (int rc = check_hip(hipEventElapsedTime(&ms, ev.first, ev.second), "timing event")) return -rc;
        g_timer.total_ms[g_timer.stage[i] & 0xff] += ms;
        g_timer.launches[g_timer.stage[i] & 0xff] += (g_timer.stage[i] & TIMED_MORE) ? 0 : 1;
    }
    g_timer.used = 0;
    for (auto &o : g_open) o = 0;
    int n = 0;
    for (; n < cap && n < GSR_STAGE_COUNT; n++) {
        if (total_ms) total_ms[n] = g_timer.total_ms[n];
        if (launches) launches[n] = g_timer.launches[n];
    }
    return n;
}

const char *gsr_stage_name(int stage) { return (stage >= 0 && stage < GSR_STAGE_COUNT) ? kStageNames[stage] : ""; }

int gsr_timing_begin(int stage, void *stream) {
    if (stage < 0 || stage >= GSR_STAGE_COUNT) return fail(GSR_ERR_ARGS, "timing stage %d out of range", stage);
    if (!(g_timer.mask & (1 << stage))) return GSR_OK;
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    if (int rc = check_hip(take_pair(stage, &ev), "timing begin")) return rc;
    g_open[stage] = g_timer.used;  // the pair's slot + 1
    hipStream_t s = (hipStream_t)stream;
    // the end event is recorded here too (a read before gsr_timing_end then sees an
    // empty region, not an unrecorded event) and again by gsr_timing_end
    if (int rc = check_hip(hipEventRecord(ev->first, s), "timing begin")) return rc;
    return check_hip(hipEventRecord(ev->second, s), "timing begin");
}

int gsr_timing_end(int stage, void *stream) {
    if (stage < 0 || stage >= GSR_STAGE_COUNT) return fail(GSR_ERR_ARGS, "timing stage %d out of range", stage);
    if (!(g_timer.mask & (1 << stage)) || g_open[stage] == 0) return GSR_OK;
    auto &ev = g_timer.pool[g_open[stage] - 1];
    g_open[stage] = 0;
    return check_hip(hipEventRecord(ev.second, (hipStream_t)stream), "timing end");
}

}  // extern "C"

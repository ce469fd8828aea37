// binning.hip — tile bucketing and per-tile depth sort.
//
// Replaces upstream duplicateWithKeys + cub::DeviceRadixSort::SortPairs +
// identifyTileRanges (rasterizer_impl.cu).
// Upstream emits one (tile<<32 | depth_bits, id) pair per touched tile and
// radix-sorts all I pairs over 32+log2(T) bits (~6 passes of 24 B/pair).
// Here the same order is produced with one pass over the instances:
//
//  1. bin_count   — workgroup b owns a contiguous slice of Gaussians and counts
//                   its instances per tile in LDS -> counts[b][t] (no global
//                   atomics; the rect is recomputed exactly as preprocess did).
//  2. bin_colscan — per tile, exclusive scan over b -> counts[b][t] becomes the
//                   slice's write offset inside the tile's bucket.
//  3. bin_tilescan— exclusive scan over tiles -> ranges[t] (identifyTileRanges'
//                   output, available before any key exists) and max tile length.
//  4. bin_scatter — each workgroup re-walks its slice and drops the 64-bit key
//                   (depth_bits << 32 | id) into the tile bucket via LDS cursors.
//  5. tile sort   — one workgroup per tile sorts its bucket in LDS.  Ascending
//                   (depth_bits, id) is exactly the stable radix order upstream
//                   gets (equal depth bits keep emission = index order), so
//                   point_list and ranges match upstream bit for bit.
//
// Steps 1-3 run before the num_rendered host read-back, overlapping it.
#pragma clang fp contract(off)

#include "gsr_kernels.hpp"
#include "gsr_math.hpp"
#include "gsr_wave.hpp"

namespace gsr {

struct BinArgs {
    int P, gpb, gx, gy, T;
    const float2 *means2D;
    const int32_t *radii;
    const float *depths;
    uint32_t *counts;  // [NB][T]
    const uint2 *ranges;
    uint64_t *keys;
};

__global__ void __launch_bounds__(BIN_THREADS) bin_count_kernel(BinArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int b = blockIdx.x;
    const int c0 = blockIdx.y * BIN_TILE_CHUNK;
    const int clen = min(BIN_TILE_CHUNK, a.T - c0);
    for (int j = threadIdx.x; j < clen; j += BIN_THREADS) hist[j] = 0;
    __syncthreads();
    const int g0 = b * a.gpb, g1 = min(a.P, g0 + a.gpb);
    for (int i = g0 + threadIdx.x; i < g1; i += BIN_THREADS) {
        const int r = a.radii[i];
        if (r <= 0) continue;
        const float2 m = a.means2D[i];
        const TileRect rc = get_rect(m.x, m.y, r, a.gx, a.gy);
        for (unsigned y = rc.y0; y < rc.y1; y++) {
            const int row = (int)(y * a.gx);
            const int t0 = max(row + (int)rc.x0, c0), t1 = min(row + (int)rc.x1, c0 + clen);
            for (int t = t0; t < t1; t++) atomicAdd(&hist[t - c0], 1u);
        }
    }
    __syncthreads();
    uint32_t *dst = a.counts + (size_t)b * a.T + c0;
    for (int j = threadIdx.x; j < clen; j += BIN_THREADS) dst[j] = hist[j];
}

__global__ void __launch_bounds__(256) bin_colscan_kernel(uint32_t *counts, int NB, int T, uint32_t *tile_total) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    uint32_t run = 0;
    int b = 0;
    for (; b + 8 <= NB; b += 8) {
        uint32_t c[8];
#pragma unroll
        for (int k = 0; k < 8; k++) c[k] = counts[(size_t)(b + k) * T + t];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            counts[(size_t)(b + k) * T + t] = run;
            run += c[k];
        }
    }
    for (; b < NB; b++) {
        const uint32_t c = counts[(size_t)b * T + t];
        counts[(size_t)b * T + t] = run;
        run += c;
    }
    tile_total[t] = run;
}

constexpr int TS_THREADS = 1024;
__global__ void __launch_bounds__(TS_THREADS)
    bin_tilescan_kernel(const uint32_t *tile_total, int T, uint2 *ranges, uint32_t *ctrl) {
    __shared__ uint32_t wsum[TS_THREADS / 64];
    __shared__ uint32_t smax;
    if (threadIdx.x == 0) smax = 0;
    __syncthreads();
    uint32_t carry = 0, mx = 0;
    for (int base = 0; base < T; base += TS_THREADS) {
        const int t = base + threadIdx.x;
        const uint32_t v = t < T ? tile_total[t] : 0u;
        uint32_t tot;
        const uint32_t inc = block_inclusive_scan<TS_THREADS>(v, wsum, &tot);
        // identifyTileRanges leaves empty tiles at the memset value (0, 0)
        if (t < T) ranges[t] = v ? make_uint2(carry + inc - v, carry + inc) : make_uint2(0u, 0u);
        carry += tot;
        mx = max(mx, v);
    }
    atomicMax(&smax, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
        ctrl[CTRL_MAX_TILE] = smax;
        ctrl[CTRL_TILE_TOTAL_LO] = carry;
    }
}

__global__ void __launch_bounds__(BIN_THREADS) bin_scatter_kernel(BinArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    const int b = blockIdx.x;
    const int c0 = blockIdx.y * BIN_TILE_CHUNK;
    const int clen = min(BIN_TILE_CHUNK, a.T - c0);
    const uint32_t *offs = a.counts + (size_t)b * a.T + c0;
    for (int j = threadIdx.x; j < clen; j += BIN_THREADS) cur[j] = a.ranges[c0 + j].x + offs[j];
    __syncthreads();
    const int g0 = b * a.gpb, g1 = min(a.P, g0 + a.gpb);
    for (int i = g0 + threadIdx.x; i < g1; i += BIN_THREADS) {
        const int r = a.radii[i];
        if (r <= 0) continue;
        const float2 m = a.means2D[i];
        const TileRect rc = get_rect(m.x, m.y, r, a.gx, a.gy);
        const uint64_t key = ((uint64_t)__float_as_uint(a.depths[i]) << 32) | (uint32_t)i;
        for (unsigned y = rc.y0; y < rc.y1; y++) {
            const int row = (int)(y * a.gx);
            const int t0 = max(row + (int)rc.x0, c0), t1 = min(row + (int)rc.x1, c0 + clen);
            for (int t = t0; t < t1; t++) {
                const uint32_t slot = atomicAdd(&cur[t - c0], 1u);
                a.keys[slot] = key;
            }
        }
    }
}

// ---------------------------------------------------------------- tile sort
__device__ __forceinline__ int next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// Bitonic sort of s[0, np) in LDS (np a power of two).  The participating waves
// each own a contiguous region of R = np / nw elements; every stage whose stride
// j is below R pairs elements inside one region, so that wave runs it on its
// own: a wave's LDS operations execute in issue order, so only a compiler fence
// separates such stages.  Only the log2(nw) * (log2(nw) + 1) / 2 stages with
// j >= R need a workgroup barrier (6 of 78 for np = 4096 on 8 waves).
template <int THREADS>
__device__ __forceinline__ void bitonic_lds(uint64_t *s, int np) {
    constexpr int NW = THREADS / 64;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int nw = np >> 7;  // keep >= 128 elements (64 pairs) per wave
    nw = nw < 1 ? 1 : (nw > NW ? NW : nw);
    const int R = np / nw, half = R >> 1;
    bool synced = true;  // all waves' previous writes are visible
    for (int k = 2; k <= np; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= R) {
                if (!synced) __syncthreads();
                for (int i = threadIdx.x; i < (np >> 1); i += THREADS) {
                    const int lo = 2 * i - (i & (j - 1));
                    const int hi = lo + j;
                    const bool asc = (lo & k) == 0;
                    const uint64_t x = s[lo], y = s[hi];
                    if ((x > y) == asc) {
                        s[lo] = y;
                        s[hi] = x;
                    }
                }
                __syncthreads();
                synced = true;
            } else {
                if (w < nw) {
                    for (int q = lane; q < half; q += 64) {
                        const int i = w * half + q;
                        const int lo = 2 * i - (i & (j - 1));
                        const int hi = lo + j;
                        const bool asc = (lo & k) == 0;
                        const uint64_t x = s[lo], y = s[hi];
                        if ((x > y) == asc) {
                            s[lo] = y;
                            s[hi] = x;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
                synced = false;
            }
        }
    }
    if (!synced) __syncthreads();
}

template <int CAP, int THREADS>
__global__ void __launch_bounds__(THREADS)
    sort_tiles_lds_kernel(const uint2 *ranges, uint64_t *keys, uint32_t *point_list) {
    __shared__ uint64_t s[CAP];
    const uint2 r = ranges[blockIdx.x];
    const int n = (int)(r.y - r.x);
    if (n <= 0 || n > CAP) return;
    if (n == 1) {
        if (threadIdx.x == 0) point_list[r.x] = (uint32_t)keys[r.x];
        return;
    }
    const int np = next_pow2(n);
    for (int i = threadIdx.x; i < np; i += THREADS) s[i] = i < n ? keys[r.x + i] : ~0ull;
    __syncthreads();
    bitonic_lds<THREADS>(s, np);
    for (int i = threadIdx.x; i < n; i += THREADS) {
        const uint64_t k = s[i];
        keys[r.x + i] = k;
        point_list[r.x + i] = (uint32_t)k;
    }
}

// Tiles longer than SORT_MAX_LDS: sort LDS-sized chunks, then merge runs
// pairwise in global memory (merge path, ping-pong with tmp).
constexpr int BIG_THREADS = 1024;
__device__ inline int merge_corank(int d, const uint64_t *A, int na, const uint64_t *B, int nb) {
    int lo = max(0, d - nb), hi = min(d, na);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A[mid] < B[d - mid - 1])
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(BIG_THREADS)
    sort_tiles_big_kernel(const uint2 *ranges, uint64_t *keys, uint64_t *tmp, uint32_t *point_list) {
    __shared__ uint64_t s[SORT_MAX_LDS];
    const uint2 r = ranges[blockIdx.x];
    const int n = (int)(r.y - r.x);
    if (n <= SORT_MAX_LDS) return;
    uint64_t *src = keys + r.x, *dst = tmp + r.x;
    for (int c = 0; c < n; c += SORT_MAX_LDS) {
        const int m = min(SORT_MAX_LDS, n - c);
        const int np = next_pow2(m);
        for (int i = threadIdx.x; i < np; i += BIG_THREADS) s[i] = i < m ? src[c + i] : ~0ull;
        __syncthreads();
        bitonic_lds<BIG_THREADS>(s, np);
        for (int i = threadIdx.x; i < m; i += BIG_THREADS) src[c + i] = s[i];
        __syncthreads();
    }
    for (int w = SORT_MAX_LDS; w < n; w <<= 1) {
        for (int s0 = 0; s0 < n; s0 += 2 * w) {
            const int na = min(w, n - s0);
            const int nb = max(0, min(w, n - s0 - na));
            const uint64_t *A = src + s0, *B = src + s0 + na;
            uint64_t *out = dst + s0;
            const int total = na + nb;
            const int per = (total + BIG_THREADS - 1) / BIG_THREADS;
            const int d0 = threadIdx.x * per;
            if (d0 < total) {
                const int d1 = min(d0 + per, total);
                int i = merge_corank(d0, A, na, B, nb);
                int j = d0 - i;
                for (int d = d0; d < d1; d++) {
                    const bool takeA = (j >= nb) || (i < na && A[i] <= B[j]);
                    out[d] = takeA ? A[i++] : B[j++];
                }
            }
        }
        __syncthreads();
        uint64_t *t = src;
        src = dst;
        dst = t;
    }
    for (int i = threadIdx.x; i < n; i += BIG_THREADS) {
        const uint64_t k = src[i];
        if (src != keys + r.x) keys[r.x + i] = k;
        point_list[r.x + i] = (uint32_t)k;
    }
}

// ---------------------------------------------------------------- launchers
static BinArgs make_args(int P, int W, int H, void *geom, const int32_t *radii) {
    const GeomLayout L = geom_layout(P, W, H);
    const GridDims g = grid_dims(W, H);
    BinArgs a;
    a.P = P;
    a.gpb = bin_gpb(P);
    a.gx = g.gx;
    a.gy = g.gy;
    a.T = g.tiles;
    a.means2D = at<float2>(geom, L.off[GSR_GEOM_MEANS2D]);
    a.radii = radii;
    a.depths = at<float>(geom, L.off[GSR_GEOM_DEPTHS]);
    a.counts = at<uint32_t>(geom, L.bin_counts);
    a.ranges = at<uint2>(geom, L.off[GSR_GEOM_RANGES]);
    a.keys = nullptr;
    return a;
}

static int nchunks(int T) { return (T + BIN_TILE_CHUNK - 1) / BIN_TILE_CHUNK; }
static size_t chunk_lds(int T) { return (size_t)min(T, BIN_TILE_CHUNK) * 4; }

hipError_t launch_bin_count(int P, int W, int H, void *geom, const int32_t *radii, hipStream_t s) {
    const BinArgs a = make_args(P, W, H, geom, radii);
    const GeomLayout L = geom_layout(P, W, H);
    const int NB = bin_blocks(P);
    uint32_t *tile_total = at<uint32_t>(geom, L.tile_total);
    hipLaunchKernelGGL(bin_count_kernel, dim3(NB, nchunks(a.T)), dim3(BIN_THREADS), chunk_lds(a.T), s, a);
    hipLaunchKernelGGL(bin_colscan_kernel, dim3((a.T + 255) / 256), dim3(256), 0, s, a.counts, NB, a.T, tile_total);
    hipLaunchKernelGGL(bin_tilescan_kernel, dim3(1), dim3(TS_THREADS), 0, s, (const uint32_t *)tile_total, a.T,
                       at<uint2>(geom, L.off[GSR_GEOM_RANGES]), at<uint32_t>(geom, L.off[GSR_GEOM_CTRL]));
    return hipGetLastError();
}

hipError_t launch_bin_scatter(int P, int W, int H, void *geom, const int32_t *radii, void *binning, int64_t I,
                              hipStream_t s) {
    BinArgs a = make_args(P, W, H, geom, radii);
    a.keys = at<uint64_t>(binning, binning_layout(I, W, H).off[GSR_BIN_KEYS]);
    const int NB = bin_blocks(P);
    hipLaunchKernelGGL(bin_scatter_kernel, dim3(NB, nchunks(a.T)), dim3(BIN_THREADS), chunk_lds(a.T), s, a);
    return hipGetLastError();
}

hipError_t launch_tile_sort(int P, int W, int H, void *geom, void *binning, int64_t I, uint32_t max_tile,
                            hipStream_t s) {
    const GridDims g = grid_dims(W, H);
    const BinningLayout B = binning_layout(I, W, H);
    const uint2 *ranges = at<uint2>(geom, geom_layout(P, W, H).off[GSR_GEOM_RANGES]);
    uint64_t *keys = at<uint64_t>(binning, B.off[GSR_BIN_KEYS]);
    uint32_t *pl = at<uint32_t>(binning, B.off[GSR_BIN_POINT_LIST]);
    const dim3 grid(g.tiles);
    const uint32_t m = max_tile < (uint32_t)SORT_MAX_LDS ? max_tile : (uint32_t)SORT_MAX_LDS;
    if (m <= 256)
        hipLaunchKernelGGL((sort_tiles_lds_kernel<256, 128>), grid, dim3(128), 0, s, ranges, keys, pl);
    else if (m <= 1024)
        hipLaunchKernelGGL((sort_tiles_lds_kernel<1024, 256>), grid, dim3(256), 0, s, ranges, keys, pl);
    else if (m <= 2048)
        hipLaunchKernelGGL((sort_tiles_lds_kernel<2048, 256>), grid, dim3(256), 0, s, ranges, keys, pl);
    else if (m <= 4096)
        hipLaunchKernelGGL((sort_tiles_lds_kernel<4096, 512>), grid, dim3(512), 0, s, ranges, keys, pl);
    else
        hipLaunchKernelGGL((sort_tiles_lds_kernel<SORT_MAX_LDS, 1024>), grid, dim3(1024), 0, s, ranges, keys, pl);
    if (max_tile > (uint32_t)SORT_MAX_LDS)
        hipLaunchKernelGGL(sort_tiles_big_kernel, grid, dim3(BIG_THREADS), 0, s, ranges, keys,
                           at<uint64_t>(binning, B.tmp_keys), pl);
    return hipGetLastError();
}

}  // namespace gsr

// knn.hip — distCUDA2: mean squared distance to the 3 nearest neighbours
// (SURVEY.md §8f "next" row 4).
//
// The reference initialises every Gaussian's scale from
//   dist2 = clamp_min(distCUDA2(points), 1e-7); scales = log(sqrt(dist2)) x3
// (scene/gaussian_model.py:20,153-155).  distCUDA2 lives in the absent
// simple-knn submodule; its published contract is the exact mean of the squared
// distances to the 3 nearest OTHER points (missing neighbours count as FLT_MAX).
//
// Here: a uniform grid with ~2 points per cubic cell.  Points are counting-sorted
// into cells; each point then visits cells in growing Chebyshev shells around its
// own and stops once its third-best squared distance is within (r h)^2 of shell
// r — every point in a farther shell is at least r h away, so the result is
// exact.  Queries run in cell order, so neighbouring threads scan the same cells.
#include <cfloat>
#include <cmath>
#include <cstring>

#include "gsr_kernels.hpp"
#include "gsr_wave.hpp"

namespace gsr {

constexpr int KNN_THREADS = 256;
constexpr uint32_t KNN_MAX_CELLS = 1u << 22;

struct KnnGrid {
    float ox, oy, oz, inv_h, h;
    int gx, gy, gz;
};

__device__ __forceinline__ uint32_t ord_f(float f) {  // order-preserving float -> uint
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(KNN_THREADS) knn_bbox_kernel(int P, const float *pts, uint32_t *bb) {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * KNN_THREADS + threadIdx.x; i < P; i += gridDim.x * KNN_THREADS)
        for (int k = 0; k < 3; k++) {
            const float v = pts[3 * (size_t)i + k];
            lo[k] = fminf(lo[k], v);
            hi[k] = fmaxf(hi[k], v);
        }
    for (int k = 0; k < 3; k++) {
        for (int o = 32; o >= 1; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&bb[k], ord_f(lo[k]));
            atomicMax(&bb[3 + k], ord_f(hi[k]));
        }
    }
}

__device__ __forceinline__ int knn_cell(const KnnGrid &g, float x, float y, float z, int &cx, int &cy, int &cz) {
    cx = min(max((int)((x - g.ox) * g.inv_h), 0), g.gx - 1);
    cy = min(max((int)((y - g.oy) * g.inv_h), 0), g.gy - 1);
    cz = min(max((int)((z - g.oz) * g.inv_h), 0), g.gz - 1);
    return (cz * g.gy + cy) * g.gx + cx;
}

__global__ void knn_count_kernel(int P, const float *pts, KnnGrid g, uint32_t *cell_of, uint32_t *count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    int cx, cy, cz;
    const int c = knn_cell(g, pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2], cx, cy, cz);
    cell_of[i] = (uint32_t)c;
    atomicAdd(&count[c], 1u);
}

// exclusive scan of count[0, n) into start[0, n] in two levels (block sums, one-block carry)
__global__ void __launch_bounds__(KNN_THREADS) knn_scan_blocks_kernel(const uint32_t *count, int n, uint32_t *start,
                                                                      uint32_t *bsum) {
    __shared__ uint32_t wsum[KNN_THREADS / 64];
    const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
    const uint32_t v = i < n ? count[i] : 0u;
    uint32_t tot;
    const uint32_t inc = block_inclusive_scan<KNN_THREADS>(v, wsum, &tot);
    if (i < n) start[i] = inc - v;
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(1024) knn_scan_carry_kernel(uint32_t *bsum, int nb) {
    __shared__ uint32_t wsum[1024 / 64];
    uint32_t carry = 0;
    for (int b = 0; b < nb; b += 1024) {
        const int i = b + threadIdx.x;
        const uint32_t v = i < nb ? bsum[i] : 0u;
        uint32_t tot;
        const uint32_t inc = block_inclusive_scan<1024>(v, wsum, &tot);
        if (i < nb) bsum[i] = carry + inc - v;
        carry += tot;
    }
}
__global__ void knn_scan_add_kernel(uint32_t *start, int n, const uint32_t *bsum, uint32_t *cursor) {
    const int i = blockIdx.x * KNN_THREADS + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = start[i] + bsum[blockIdx.x];
    start[i] = s;
    cursor[i] = s;
}

__global__ void knn_scatter_kernel(int P, const float *pts, const uint32_t *cell_of, uint32_t *cursor, float4 *sorted) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const uint32_t slot = atomicAdd(&cursor[cell_of[i]], 1u);
    sorted[slot] = make_float4(pts[3 * (size_t)i], pts[3 * (size_t)i + 1], pts[3 * (size_t)i + 2],
                               __uint_as_float((uint32_t)i));
}

__device__ __forceinline__ void knn_insert(float d, float &b0, float &b1, float &b2) {
    if (d < b2) {
        if (d < b1) {
            b2 = b1;
            if (d < b0) {
                b1 = b0;
                b0 = d;
            } else {
                b1 = d;
            }
        } else {
            b2 = d;
        }
    }
}

__global__ void __launch_bounds__(KNN_THREADS) knn_query_kernel(int P, KnnGrid g, const float4 *sorted,
                                                                const uint32_t *start, const uint32_t *count,
                                                                float *dist2) {
    const int s = blockIdx.x * KNN_THREADS + threadIdx.x;
    if (s >= P) return;
    const float4 q = sorted[s];
    const uint32_t self = __float_as_uint(q.w);
    int cx, cy, cz;
    knn_cell(g, q.x, q.y, q.z, cx, cy, cz);
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    const int rmax = max(g.gx, max(g.gy, g.gz));
    for (int r = 0; r <= rmax; r++) {
        for (int dz = -r; dz <= r; dz++) {
            const int z = cz + dz;
            if (z < 0 || z >= g.gz) continue;
            for (int dy = -r; dy <= r; dy++) {
                const int y = cy + dy;
                if (y < 0 || y >= g.gy) continue;
                const bool face = dz == -r || dz == r || dy == -r || dy == r;
                for (int dx = -r; dx <= r; dx += (face || r == 0) ? 1 : 2 * r) {  // shell cells only
                    const int x = cx + dx;
                    if (x < 0 || x >= g.gx) continue;
                    const int c = (z * g.gy + y) * g.gx + x;
                    const uint32_t b = start[c], e = b + count[c];
                    for (uint32_t j = b; j < e; j++) {
                        const float4 p = sorted[j];
                        if (__float_as_uint(p.w) == self) continue;
                        const float ex = p.x - q.x, ey = p.y - q.y, ez = p.z - q.z;
                        knn_insert(ex * ex + ey * ey + ez * ez, b0, b1, b2);
                    }
                }
            }
        }
        // every unvisited point is at least r h away (a hair less, for the rounding
        // of the cell index); at r = 0 only three exact duplicates end the search
        const float reach = fmaxf((float)r - 1e-3f, 0.0f) * g.h;
        if (b2 <= reach * reach) break;
    }
    dist2[self] = (b0 + b1 + b2) / 3.0f;
}

size_t knn_scratch_bytes(int P) {
    const size_t cells = KNN_MAX_CELLS, nb = (cells + KNN_THREADS - 1) / KNN_THREADS;
    return 64 + (size_t)P * 16 + (size_t)P * 4 + cells * 4 * 3 + nb * 4;
}

hipError_t launch_knn(int P, const float *pts, float *dist2, void *scratch, uint32_t *pinned6, hipStream_t s) {
    if (P <= 0) return hipSuccess;
    char *base = (char *)scratch;
    uint32_t *bb = (uint32_t *)base;
    float4 *sorted = (float4 *)(base + 64);
    uint32_t *cell_of = (uint32_t *)(base + 64 + (size_t)P * 16);
    uint32_t *count = cell_of + P;
    uint32_t *start = count + KNN_MAX_CELLS;
    uint32_t *cursor = start + KNN_MAX_CELLS;
    uint32_t *bsum = cursor + KNN_MAX_CELLS;
    const uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    hipError_t e = hipMemcpyAsync(bb, init, sizeof init, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(knn_bbox_kernel, dim3(min(1024, (P + KNN_THREADS - 1) / KNN_THREADS)), dim3(KNN_THREADS), 0, s,
                       P, pts, bb);
    e = hipMemcpyAsync(pinned6, bb, 24, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the grid shape depends on the bounding box
    if (e != hipSuccess) return e;
    auto unord = [](uint32_t u) {
        const uint32_t v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
        float f;
        memcpy(&f, &v, 4);
        return f;
    };
    float lo[3], ext[3];
    for (int k = 0; k < 3; k++) {
        lo[k] = unord(pinned6[k]);
        ext[k] = std::fmax(unord(pinned6[3 + k]) - lo[k], 0.0f);
    }
    // cubic cells holding ~2 points on average, at most KNN_MAX_CELLS cells
    const double emax = std::fmax(std::fmax(ext[0], ext[1]), std::fmax(ext[2], 1e-30f));
    double vol = 1.0;
    for (int k = 0; k < 3; k++) vol *= std::fmax((double)ext[k], emax * 1e-3);
    double h = std::cbrt(vol / std::fmax(P / 2.0, 1.0));
    KnnGrid g;
    for (;;) {
        g.gx = (int)std::fmin(std::ceil(ext[0] / h), 4096.0);
        g.gy = (int)std::fmin(std::ceil(ext[1] / h), 4096.0);
        g.gz = (int)std::fmin(std::ceil(ext[2] / h), 4096.0);
        g.gx = g.gx < 1 ? 1 : g.gx;
        g.gy = g.gy < 1 ? 1 : g.gy;
        g.gz = g.gz < 1 ? 1 : g.gz;
        if ((double)g.gx * g.gy * g.gz <= KNN_MAX_CELLS) break;
        h *= 1.25;
    }
    g.ox = lo[0];
    g.oy = lo[1];
    g.oz = lo[2];
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    const int cells = g.gx * g.gy * g.gz, nbc = (cells + KNN_THREADS - 1) / KNN_THREADS;
    e = hipMemsetAsync(count, 0, (size_t)cells * 4, s);
    if (e != hipSuccess) return e;
    const int pb = (P + KNN_THREADS - 1) / KNN_THREADS;
    hipLaunchKernelGGL(knn_count_kernel, dim3(pb), dim3(KNN_THREADS), 0, s, P, pts, g, cell_of, count);
    hipLaunchKernelGGL(knn_scan_blocks_kernel, dim3(nbc), dim3(KNN_THREADS), 0, s, (const uint32_t *)count, cells,
                       start, bsum);
    hipLaunchKernelGGL(knn_scan_carry_kernel, dim3(1), dim3(1024), 0, s, bsum, nbc);
    hipLaunchKernelGGL(knn_scan_add_kernel, dim3(nbc), dim3(KNN_THREADS), 0, s, start, cells, (const uint32_t *)bsum,
                       cursor);
    hipLaunchKernelGGL(knn_scatter_kernel, dim3(pb), dim3(KNN_THREADS), 0, s, P, pts, (const uint32_t *)cell_of,
                       cursor, sorted);
    hipLaunchKernelGGL(knn_query_kernel, dim3(pb), dim3(KNN_THREADS), 0, s, P, g, (const float4 *)sorted,
                       (const uint32_t *)start, (const uint32_t *)count, dist2);
    return hipGetLastError();
}

}  // namespace gsr

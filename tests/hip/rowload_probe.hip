// rowload_probe.hip — HBM read rate of the SH-row access patterns (design probe).
//
// Each thread reads one 192-B row (12 x 16 B) of an N x 192-B table and writes
// one float: "row" = every lane loads its own row (lane stride 192 B: each load
// instruction touches 64 different 128-B lines, what preprocess_fwd / _bwd do);
// "coalesced" = the wave reads the same 12 KB as 12 contiguous 1-KB loads (no
// transpose: the bandwidth ceiling).  Build: hipcc -O3 --offload-arch=gfx950
// rowload_probe.hip -o rowload_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) probe(const float4 *t, float *out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float4 v[12];
    if constexpr (MODE == 0) {
#pragma unroll
        for (int b = 0; b < 12; b++) v[b] = t[(size_t)i * 12 + b];
    } else {
        const size_t w0 = (size_t)(i & ~63) * 12, lane = i & 63;
#pragma unroll
        for (int b = 0; b < 12; b++) v[b] = t[w0 + (size_t)b * 64 + lane];
    }
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < 12; b++) s += (v[b].x + v[b].y) + (v[b].z + v[b].w);
    out[i] = s;
}

template <int MODE>
void run(const char *name, const float4 *t, float *out, int n) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = (n + 255) / 256;
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, t, out, n);
    hipEventRecord(a);
    const int reps = 10;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(256), 0, 0, t, out, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double us = 1e3 * ms / reps, bytes = (double)n * (192 + 4);
    printf("%-10s N=%9d  %8.1f us  %6.2f TB/s\n", name, n, us, bytes / (us * 1e-6) / 1e12);
}

int main() {
    for (int n : {1000000, 5000000}) {
        float4 *t;
        float *out;
        hipMalloc(&t, (size_t)n * 192);
        hipMalloc(&out, (size_t)n * 4);
        hipMemset(t, 0, (size_t)n * 192);
        run<0>("row", t, out, n);
        run<1>("coalesced", t, out, n);
        run<0>("row", t, out, n);
        run<1>("coalesced", t, out, n);
        hipFree(t);
        hipFree(out);
    }
    return 0;
}

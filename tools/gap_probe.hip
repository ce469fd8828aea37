// gap_probe.hip — what sets the idle gap between two dependent kernels on one stream?
// Kernel A streams `mb` MB of stores (plain, nontemporal) or float atomics over a
// buffer; kernel B is tiny.  Run under rocprofv3 --kernel-trace: the gap between A's
// end and B's start, per A variant and size, says whether the dirty L2 lines A
// leaves behind (written back at the kernel boundary on a multi-XCD part) cost time.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gap_probe.hip -o /tmp/gap_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void store_plain(float4 *p, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}
__global__ void store_nt(float4 *p, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store(1.f, &p[i].x);
        __builtin_nontemporal_store(2.f, &p[i].y);
        __builtin_nontemporal_store(3.f, &p[i].z);
        __builtin_nontemporal_store(4.f, &p[i].w);
    }
}
// one atomic per 64-B row, rows in a scrambled order (the render backward's accumulator)
__global__ void atomics(float *p, size_t rows) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < rows; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = (i * 2654435761ull) % rows;
        atomicAdd(p + r * 16 + (threadIdx.x & 15), 1.f);
    }
}
__global__ void tiny(float *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const size_t max_mb = 256;
    float *buf = nullptr, *t = nullptr;
    if (hipMalloc(&buf, max_mb << 20) != hipSuccess || hipMalloc(&t, 256) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, max_mb << 20);
    (void)hipMemset(t, 0, 256);
    const size_t sizes[] = {1, 8, 32, 64, 256};
    for (int v = 0; v < 3; v++) {
        for (size_t mb : sizes) {
            const size_t n4 = (mb << 20) / 16;
            for (int r = 0; r < reps; r++) {
                if (v == 0) store_plain<<<2048, 256>>>((float4 *)buf, n4);
                if (v == 1) store_nt<<<2048, 256>>>((float4 *)buf, n4);
                if (v == 2) atomics<<<2048, 256>>>(buf, (mb << 20) / 64);
                tiny<<<1, 64>>>(t);
            }
            (void)hipDeviceSynchronize();
        }
    }
    printf("done\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

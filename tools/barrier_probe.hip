// Probe (not part of the library): the cost of a grid-wide barrier in a
// cooperative launch on this GPU, with and without a scatter between barriers
// (the dirty L2 lines a release has to write back).  Decides whether a
// one-launch depth sort (barriers instead of kernel boundaries) can pay.
//   hipcc -O3 --offload-arch=gfx950 tools/barrier_probe.hip -o /tmp/barrier_probe
//   ./barrier_probe      (on the box)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

// every word on a 256-B line of its own: polling loads of the generation must
// not share a line with the arrival atomics
struct Bar {
    unsigned count[64];
    unsigned gen[64];
    unsigned abort[64];
    unsigned sub[8][64];  // hierarchical: one arrival counter per XCD (blockIdx % 8)
};

__device__ __forceinline__ bool grid_barrier(Bar *b, unsigned G, int hier) {
    __syncthreads();
    __shared__ int s_ok;
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned g0 = __hip_atomic_load(&b->gen[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool last;
        if (hier) {  // G a multiple of 8: G / 8 arrivals per group, then 8 at the top
            const unsigned x = blockIdx.x & 7u;
            last = __hip_atomic_fetch_add(&b->sub[x][0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == G / 8 - 1;
            if (last) {
                __hip_atomic_store(&b->sub[x][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = __hip_atomic_fetch_add(&b->count[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 7u;
            }
        } else {
            last = __hip_atomic_fetch_add(&b->count[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
        }
        int ok = 1;
        if (last) {
            __hip_atomic_store(&b->count[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&b->gen[0], g0 + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned tries = 0;
            while (__hip_atomic_load(&b->gen[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g0) {
                if (++tries > (1u << 22)) {  // exit condition every wave reaches
                    __hip_atomic_store(&b->abort[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __threadfence();
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

__global__ void __launch_bounds__(256) probe(Bar *b, int nbar, unsigned *buf, unsigned n, int scatter, int hier) {
    const unsigned G = gridDim.x;
    for (int k = 0; k < nbar; k++) {
        if (scatter) {  // every workgroup writes its share of n words, permuted
            for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += G * blockDim.x) {
                const unsigned j = (i * 2654435761u + (unsigned)k) & (n - 1u);
                buf[j] = i + k;
            }
        }
        if (!grid_barrier(b, G, hier)) return;
    }
}

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    int per_cu = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, probe, 256, 0);
    printf("CUs %d, co-resident workgroups per CU %d, coop %d\n", prop.multiProcessorCount, per_cu,
           prop.cooperativeLaunch);
    Bar *b;
    unsigned *buf;
    const unsigned n = 2u << 20;
    hipMalloc(&b, sizeof(Bar));
    hipMemset(b, 0, sizeof(Bar));
    hipMalloc(&buf, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int G : {256, 512, 1024}) {
        if (G > prop.multiProcessorCount * per_cu) continue;
        for (int hier : {0, 1})
        for (int scatter : {0, 1}) {
            for (int nbar : {1, 9, 33}) {
                float best = 1e9f;
                for (int rep = 0; rep < 5; rep++) {
                    void *args[] = {&b, &nbar, &buf, (void *)&n, &scatter, &hier};
                    hipEventRecord(e0, 0);
                    hipError_t err = hipLaunchCooperativeKernel((void *)probe, dim3(G), dim3(256), args, 0, 0);
                    hipEventRecord(e1, 0);
                    hipEventSynchronize(e1);
                    if (err != hipSuccess) {
                        printf("launch failed: %s\n", hipGetErrorString(err));
                        return 1;
                    }
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    best = ms < best ? ms : best;
                }
                Bar hb;
                hipMemcpy(&hb, b, sizeof(Bar), hipMemcpyDeviceToHost);
                printf("G %4d hier %d scatter %d barriers %2d: %8.2f us (abort %u)\n", G, hier, scatter, nbar, best * 1e3f,
                       hb.abort[0]);
                if (hb.abort[0]) return 1;
            }
        }
    }
    return 0;
}

// Probe v_permlane32_swap / v_permlane16_swap semantics on gfx950.
#include <cstdio>
#include <hip/hip_runtime.h>
__global__ void probe(int* out) {
    int lane = threadIdx.x;
    unsigned a = 1000 + lane, b = 2000 + lane;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[lane] = r[0]; out[64 + lane] = r[1];
    auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[128 + lane] = q[0]; out[192 + lane] = q[1];
}
int main() {
    int* d; (void)hipMalloc(&d, 256 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    int h[256]; (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[] = {"p32 r0", "p32 r1", "p16 r0", "p16 r1"};
    for (int s = 0; s < 4; s++) { printf("%s:", nm[s]); for (int l = 0; l < 64; l++) printf(" %d", h[s*64+l]); printf("\n"); }
}

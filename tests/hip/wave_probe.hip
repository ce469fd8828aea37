// Probe of the wave64 DPP reductions in gsr_wave.hpp (run on the GPU box).
#include <cstdio>
#include <hip/hip_runtime.h>
#include "../../3dgs_study_amd/csrc/gsr_wave.hpp"
using namespace gsr;

__global__ void probe(float* out, uint32_t* outs) {
    int lane = threadIdx.x;
    float v = (float)(lane + 1);          // sum = 2080
    float s = wave_sum_to_lane63(v);
    out[lane] = s;
    uint32_t u = wave_inclusive_scan((uint32_t)1);
    outs[lane] = u;
    // staged variants
    float a = v;
    a += dpp_f32<DPP_ROW_SHR1>(a);
    out[64 + lane] = a;
    a += dpp_f32<DPP_ROW_SHR2>(a);
    out[128 + lane] = a;
    a += dpp_f32<DPP_ROW_SHR4, 0xf, 0xe>(a);
    out[192 + lane] = a;
    a += dpp_f32<DPP_ROW_SHR8, 0xf, 0xc>(a);
    out[256 + lane] = a;
    a += dpp_f32<DPP_ROW_BCAST15, 0xa>(a);
    out[320 + lane] = a;
    a += dpp_f32<DPP_ROW_BCAST31, 0xc>(a);
    out[384 + lane] = a;
}

int main() {
    float* d; uint32_t* du;
    hipMalloc(&d, 448 * 4); hipMalloc(&du, 64 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, du);
    float h[448]; uint32_t hu[64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(hu, du, sizeof hu, hipMemcpyDeviceToHost);
    printf("wave_sum lane63 = %g (expect 2080)\n", h[63]);
    const char* names[] = {"shr1", "shr2", "shr4", "shr8", "bcast15", "bcast31"};
    for (int st = 0; st < 6; st++) {
        printf("%-8s:", names[st]);
        for (int l = 0; l < 64; l++) printf(" %g", h[64 * (st + 1) + l]);
        printf("\n");
    }
    printf("scan:");
    for (int l = 0; l < 64; l++) printf(" %u", hu[l]);
    printf("\n");
    return 0;
}

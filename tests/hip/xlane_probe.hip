// xlane_probe.hip — throughput of cross-lane primitives on gfx950 (design probe).
//
// Each kernel runs ITER iterations of 8 independent chains of one operation on
// every lane of a full chip (256 CUs x 8 waves per SIMD) and reports the cost
// per wave-instruction per SIMD in cycles (at the measured clock), so the blend
// kernels' reductions can be priced: plain v_add_f32, DPP row_shr add, DPP
// row_shl mov, v_permlane32_swap, v_permlane16_swap, ds_swizzle, ds_bpermute,
// v_readlane.  Build: hipcc -O3 --offload-arch=gfx950 xlane_probe.hip -o xlane_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITER = 4096;

template <int OP>
__global__ void __launch_bounds__(256) probe(float *out, float seed) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = seed + threadIdx.x * 0.001f + c;
    for (int i = 0; i < ITER; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if constexpr (OP == 0) {
                v[c] = v[c] + 1.0001f;
            } else if constexpr (OP == 1) {
                v[c] += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[c]), 0x111,
                                                                               0xf, 0xf, true));
            } else if constexpr (OP == 2) {
                v[c] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[c]), 0x101,
                                                                              0xf, 0xf, true)) +
                       0.5f;
            } else if constexpr (OP == 3) {
                const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, v[c]),
                                                                __builtin_bit_cast(uint32_t, v[(c + 1) & 7]), false,
                                                                false);
                const uint32_t x = r[0];
                v[c] = __builtin_bit_cast(float, x) + 0.5f;
            } else if constexpr (OP == 4) {
                const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, v[c]),
                                                                __builtin_bit_cast(uint32_t, v[(c + 1) & 7]), false,
                                                                false);
                const uint32_t x = r[0];
                v[c] = __builtin_bit_cast(float, x) + 0.5f;
            } else if constexpr (OP == 5) {
                v[c] += __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v[c]), 0x041f));
            } else if constexpr (OP == 6) {
                v[c] += __builtin_bit_cast(
                    float, __builtin_amdgcn_ds_bpermute(((threadIdx.x ^ 1) & 63) * 4, __builtin_bit_cast(int, v[c])));
            } else if constexpr (OP == 7) {
                v[c] += __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v[c]), (c * 7) & 63));
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += v[c];
    if (s == 12345.f) out[0] = s;
}

template <int OP>
float run(const char *name, float *out, float ghz) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 8;  // 8 waves per SIMD on 256 CUs (4 waves per block)
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(a);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double waves = blocks * 4.0, instr = (double)ITER * 8;  // per wave (the main op)
    const double simds = 256 * 4;
    const double cyc = ms * 1e-3 * ghz * 1e9;
    const double per = cyc / (waves * instr / simds);
    printf("%-22s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (incl. loop + add)\n", name, ms, per);
    return per;
}

int main() {
    float *out;
    hipMalloc(&out, 4);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    const float ghz = clk / 1e6f;
    printf("clock %.3f GHz\n", ghz);
    run<0>("v_add_f32", out, ghz);
    run<1>("dpp row_shr:1 add", out, ghz);
    run<2>("dpp row_shl:1 mov+add", out, ghz);
    run<3>("permlane32_swap+add", out, ghz);
    run<4>("permlane16_swap+add", out, ghz);
    run<5>("ds_swizzle+add", out, ghz);
    run<6>("ds_bpermute+add", out, ghz);
    run<7>("v_readlane+add", out, ghz);
    return 0;
}

// Issue cost of the compositor's instruction mix (measurement tooling, not
// product code): cycles per wave64 instruction of v_fma_f32 and v_exp_f32,
// with every SIMD holding 8 waves.  Each kernel runs ITERS iterations of
// 8 independent chains; time per instruction per SIMD from events.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)(threadIdx.x + i);
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_exp(float* out, float a, float b) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = -(float)(threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_exp_f32_e64 %0, -%0" : "+v"(v[i]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s + a + b;
}

// 1 exp per 8 fma (the compositor has ~1 per 10 VALU): 9 VALU per iteration
__global__ __launch_bounds__(256) void k_mix(float* out, float a, float b) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = -(float)(threadIdx.x + i) * 1e-3f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
        asm volatile("v_exp_f32_e64 %0, -%0" : "+v"(v[3]));
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
    float* out;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4)) return 2;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double clk = p.clockRate * 1e3;  // Hz
    auto run = [&](const char* name, int insts_per_iter, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double waves_per_simd = (double)blocks * 4 / (cus * 4);
        const double insts = waves_per_simd * ITERS * insts_per_iter * 10;
        printf("%-6s %7.3f ms  %.2f cycles per wave instruction per SIMD (clock %.0f MHz)\n", name, ms,
               ms * 1e-3 * clk / insts, clk / 1e6);
    };
    run("fma", 8, [&] { k_fma<<<blocks, 256>>>(out, 0.999f, 1e-3f); });
    run("exp", 8, [&] { k_exp<<<blocks, 256>>>(out, 0.f, 0.f); });  // exp + negate
    run("mix", 9, [&] { k_mix<<<blocks, 256>>>(out, 0.999f, 1e-3f); });
    return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}

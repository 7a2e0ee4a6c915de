// Microbenchmark: wave64 VALU issue rates on gfx950 (scalar f32 FMA, packed
// f32 FMA, v_exp_f32), 8 waves/SIMD.  Measurement tooling, not product code.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float2v p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, sv = {s, s};
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {  // 8 independent scalar FMAs
            a0 = fmaf(a0, s, 0.5f); a1 = fmaf(a1, s, 0.5f); a2 = fmaf(a2, s, 0.5f); a3 = fmaf(a3, s, 0.5f);
            a4 = fmaf(a4, s, 0.5f); a5 = fmaf(a5, s, 0.5f); a6 = fmaf(a6, s, 0.5f); a7 = fmaf(a7, s, 0.5f);
        } else if (KIND == 1) {  // 4 packed FMAs = 8 FMAs
            p0 = p0 * sv + 0.5f; p1 = p1 * sv + 0.5f; p2 = p2 * sv + 0.5f; p3 = p3 * sv + 0.5f;
        } else {  // 8 independent exp2
            a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1); a2 = __builtin_amdgcn_exp2f(a2);
            a3 = __builtin_amdgcn_exp2f(a3); a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
            a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7);
        }
    }
    float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
    if (r == 12345.f) out[0] = r;
}

template <int KIND>
void run(const char* name, float* d, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<KIND><<<blocks, 256>>>(d, iters, 0.999f);
    hipEventRecord(a);
    k<KIND><<<blocks, 256>>>(d, iters, 0.999f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 256 / 64 * iters * (KIND == 1 ? 4 : 8);  // wave-instructions
    const double simd = 1024.0;
    printf("%-14s %8.3f ms  %.3f wave-instr/ns  -> %.2f ns per wave-instr per SIMD\n", name, ms, ops / (ms * 1e6),
           ms * 1e6 * simd / ops);
}

int main() {
    float* d; hipMalloc(&d, 4);
    const int blocks = 256 * 8 * 4;  // 8 blocks/CU of 4 waves (8 waves/SIMD) x 4 rounds
    run<0>("v_fma_f32", d, blocks, 4096);
    run<1>("v_pk_fma_f32", d, blocks, 4096);
    run<2>("v_exp_f32", d, blocks, 4096);
    return 0;
}

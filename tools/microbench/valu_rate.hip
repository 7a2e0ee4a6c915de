// Microbenchmark: wave64 issue rates on gfx950, 8 waves/SIMD: scalar f32 FMA,
// packed f32 FMA, v_exp_f32, SALU ops, and a VALU+SALU mix.
// Measurement tooling, not product code.  Build: hipcc --offload-arch=gfx950 -O3
// -fno-slp-vectorize valu_rate.hip -o valu_rate (no SLP: keep scalar v_fma_f32).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float2v p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, sv = {s, s};
    float b0 = a0 * 0.5f, b1 = a1 * 0.25f, b2 = a2 * 0.125f, b3 = a3 * 0.3f, c0 = a4 * 1e-3f, c1 = a5 * 2e-3f,
          c2 = a6 * 3e-3f, c3 = a7 * 4e-3f;
    uint32_t u0 = blockIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3, u4 = u0 + 4, u5 = u0 + 5, u6 = u0 + 6,
             u7 = u0 + 7, uc = __builtin_amdgcn_readfirstlane((uint32_t)iters);
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {  // 8 independent scalar FMAs
            a0 = fmaf(a0, s, 0.5f); a1 = fmaf(a1, s, 0.5f); a2 = fmaf(a2, s, 0.5f); a3 = fmaf(a3, s, 0.5f);
            a4 = fmaf(a4, s, 0.5f); a5 = fmaf(a5, s, 0.5f); a6 = fmaf(a6, s, 0.5f); a7 = fmaf(a7, s, 0.5f);
        } else if (KIND == 1) {  // 4 packed FMAs = 8 FMAs
            p0 = p0 * sv + 0.5f; p1 = p1 * sv + 0.5f; p2 = p2 * sv + 0.5f; p3 = p3 * sv + 0.5f;
        } else if (KIND == 3 || KIND == 4) {  // 8 independent SALU ops (+ 8 FMAs when KIND 4)
            asm volatile(
                "s_xor_b32 %0, %0, %8\n s_xor_b32 %1, %1, %8\n s_xor_b32 %2, %2, %8\n s_xor_b32 %3, %3, %8\n"
                "s_xor_b32 %4, %4, %8\n s_xor_b32 %5, %5, %8\n s_xor_b32 %6, %6, %8\n s_xor_b32 %7, %7, %8\n"
                : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3), "+s"(u4), "+s"(u5), "+s"(u6), "+s"(u7)
                : "s"(uc)
                : "scc");
            if (KIND == 4) {
                a0 = fmaf(a0, s, 0.5f); a1 = fmaf(a1, s, 0.5f); a2 = fmaf(a2, s, 0.5f); a3 = fmaf(a3, s, 0.5f);
                a4 = fmaf(a4, s, 0.5f); a5 = fmaf(a5, s, 0.5f); a6 = fmaf(a6, s, 0.5f); a7 = fmaf(a7, s, 0.5f);
            }
        } else if (KIND == 5) {  // 8 independent FMAs, three VGPR operands each
            a0 = fmaf(a0, b0, c0); a1 = fmaf(a1, b1, c1); a2 = fmaf(a2, b2, c2); a3 = fmaf(a3, b3, c3);
            a4 = fmaf(a4, b0, c1); a5 = fmaf(a5, b1, c2); a6 = fmaf(a6, b2, c3); a7 = fmaf(a7, b3, c0);
        } else if (KIND == 6) {  // 8 independent muls, two VGPR operands each
            a0 = a0 * b0; a1 = a1 * b1; a2 = a2 * b2; a3 = a3 * b3; a4 = a4 * c0; a5 = a5 * c1; a6 = a6 * c2;
            a7 = a7 * c3;
        } else if (KIND == 7) {  // 8 independent compare+select pairs (VGPR operands)
            a0 = a0 < b0 ? c0 : a0; a1 = a1 < b1 ? c1 : a1; a2 = a2 < b2 ? c2 : a2; a3 = a3 < b3 ? c3 : a3;
        } else {  // 8 independent exp2
            a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1); a2 = __builtin_amdgcn_exp2f(a2);
            a3 = __builtin_amdgcn_exp2f(a3); a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
            a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7);
        }
    }
    a0 += b0 + b1 + b2 + b3 + c0 + c1 + c2 + c3;
    float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
    if (r == 12345.f || (u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7) == 0x9e3779b9u) out[0] = r;
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
    const double ops = (double)blocks * 256 / 64 * iters * (KIND == 1 ? 4 : 8);  // wave-instructions (KIND 7: pairs)
    const double simd = 1024.0;
    printf("%-14s %8.3f ms  %.3f wave-instr/ns  -> %.2f ns per wave-instr per SIMD, %.3f ns per CU\n", name, ms,
           ops / (ms * 1e6), ms * 1e6 * simd / ops, ms * 1e6 * 256.0 / ops);
}

int main() {
    float* d; hipMalloc(&d, 4);
    const int blocks = 256 * 8 * 4;  // 8 blocks/CU of 4 waves (8 waves/SIMD) x 4 rounds
    run<0>("v_fma_f32", d, blocks, 4096);
    run<1>("v_pk_fma_f32", d, blocks, 4096);
    run<2>("v_exp_f32", d, blocks, 4096);
    run<3>("s_xor_b32", d, blocks, 4096);
    run<4>("fma+salu (8+8)", d, blocks, 4096);
    run<5>("fma 3 vgpr", d, blocks, 4096);
    run<6>("mul 2 vgpr", d, blocks, 4096);
    run<7>("cmp+cndmask x4", d, blocks, 4096);
    return 0;
}

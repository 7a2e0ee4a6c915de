// Microbenchmark (measurement tooling, not product code): the preprocess's
// memory pattern -- 15 float4 loads per Gaussian (pos, rot, scale, 12 SH
// planes) and 60 B of stores (a 48-B record, a depth key, an 8-B tile rect, at
// slot n-1-i) -- under different plane layouts and grids, against a float4 copy.
//   soa      plane p of Gaussian i at p*n + i (the product's SceneData layout)
//   aosoa64  the 15 planes of each group of 64 Gaussians together:
//            ((i/64)*15 + p)*64 + i%64 (every load still 1 KB coalesced per wave,
//            a wave's 15 loads one contiguous 15 KB block)
// grid: "stride" = 4 blocks per CU, grid-stride loop (the product);
//       "full"   = one thread per Gaussian.
// Build: hipcc --offload-arch=gfx950 -O3 plane_layout.hip -o plane_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kPlanes = 15;

template <int LAYOUT>
__device__ __forceinline__ int64_t plane_idx(int64_t n, int p, int64_t i) {
    if (LAYOUT == 0) return (int64_t)p * n + i;
    return ((i >> 6) * kPlanes + p) * 64 + (i & 63);
}

template <int LAYOUT>
__global__ __launch_bounds__(256) void k_pre(const float4* __restrict__ in, int64_t n, float4* __restrict__ recs,
                                             uint32_t* __restrict__ keys, uint2* __restrict__ rects) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        float4 v[kPlanes];
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) v[p] = in[plane_idx<LAYOUT>(n, p, i)];
        float4 a = v[0], b = v[1], c = v[2];
#pragma unroll
        for (int p = 3; p < kPlanes; ++p) {
            a.x += v[p].x * b.y; a.y += v[p].y * c.z; a.z += v[p].z * b.x; a.w += v[p].w * c.y;
        }
        const int64_t slot = n - 1 - i;
        recs[slot * 3 + 0] = a;
        recs[slot * 3 + 1] = b;
        recs[slot * 3 + 2] = c;
        keys[slot] = __float_as_uint(a.x);
        rects[slot] = make_uint2(__float_as_uint(a.y), __float_as_uint(a.z));
    }
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ in, float4* __restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    int dev = 0, cus = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    for (int64_t n : {1000000LL, 4000000LL}) {
        float4 *in, *recs, *cp;
        uint32_t* keys;
        uint2* rects;
        hipMalloc(&in, (size_t)n * kPlanes * 16 + 64 * kPlanes * 16);
        hipMalloc(&recs, (size_t)n * 48);
        hipMalloc(&keys, (size_t)n * 4);
        hipMalloc(&rects, (size_t)n * 8);
        hipMalloc(&cp, (size_t)n * kPlanes * 16);
        hipMemset(in, 0, (size_t)n * kPlanes * 16);
        const double bytes = (double)n * (kPlanes * 16 + 60);
        const unsigned g_stride = 4u * cus, g_full = (unsigned)((n + 255) / 256);
        for (unsigned grid : {g_stride, 8u * cus, g_full}) {
            const float t0 = time_ms([&] { k_pre<0><<<grid, 256>>>(in, n, recs, keys, rects); }, 20);
            const float t1 = time_ms([&] { k_pre<1><<<grid, 256>>>(in, n, recs, keys, rects); }, 20);
            printf("n=%lld grid=%u  soa %.1f us %.2f TB/s   aosoa64 %.1f us %.2f TB/s\n", (long long)n, grid,
                   t0 * 1e3, bytes / (t0 * 1e-3) / 1e12, t1 * 1e3, bytes / (t1 * 1e-3) / 1e12);
        }
        const int64_t m = n * kPlanes;
        const float tc = time_ms([&] { k_copy<<<(unsigned)((m + 255) / 256), 256>>>(in, cp, m); }, 20);
        printf("n=%lld float4 copy of the same input: %.1f us %.2f TB/s (read + write)\n", (long long)n, tc * 1e3,
               2.0 * m * 16 / (tc * 1e-3) / 1e12);
        hipFree(in);
        hipFree(recs);
        hipFree(keys);
        hipFree(rects);
        hipFree(cp);
    }
    return 0;
}

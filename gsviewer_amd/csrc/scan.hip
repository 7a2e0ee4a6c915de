// Device-wide exclusive prefix sum over uint32 (reduce-then-scan, 3 launches).
//
// Used for: visible-Gaussian compaction offsets, per-splat tile-instance
// offsets, and the digit-major radix histograms. Each block owns 4096 items
// (256 threads x 16 contiguous items, loaded as 4 x dwordx4).
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTileItems = kThreads * kItems;  // 4096
constexpr int kPartialThreads = 1024;

// Exclusive scan of one value per thread across a block of NT threads.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive(uint32_t v, uint32_t* lds_waves,
                                                    uint32_t& total) {
    constexpr int NW = NT / 64;
    const int w = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive_scan(v);
    if (__lane_id() == 63) lds_waves[w] = inc;
    __syncthreads();
    uint32_t woff = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t t = lds_waves[i];
        woff += (i < w) ? t : 0u;
        tot += t;
    }
    total = tot;
    return woff + inc - v;
}

__device__ __forceinline__ void load16(const uint32_t* in, size_t base, size_t n, uint32_t (&v)[kItems]) {
    if (base + kItems <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 t = p[q];
            v[4 * q + 0] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kItems; ++k) v[k] = (base + k < n) ? in[base + k] : 0u;
    }
}

__global__ __launch_bounds__(kThreads) void k_scan_reduce(const uint32_t* __restrict__ in, size_t n,
                                                          uint32_t* __restrict__ block_sums) {
    __shared__ uint32_t lds[kThreads / 64];
    const size_t base = (size_t)blockIdx.x * kTileItems + (size_t)threadIdx.x * kItems;
    uint32_t v[kItems];
    load16(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) s += v[k];
    s = wave_reduce_sum(s);
    if (__lane_id() == 0) lds[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < kThreads / 64; ++i) t += lds[i];
        block_sums[blockIdx.x] = t;
    }
}

// Single block: exclusive scan of the block sums, in place; writes the grand
// total to total_dev when non-null.
__global__ __launch_bounds__(kPartialThreads) void k_scan_partials(uint32_t* __restrict__ sums, size_t nb,
                                                                   uint32_t* __restrict__ total_dev) {
    __shared__ uint32_t lds[kPartialThreads / 64];
    const size_t per = (nb + kPartialThreads - 1) / kPartialThreads;
    const size_t b0 = (size_t)threadIdx.x * per;
    const size_t b1 = (b0 + per < nb) ? b0 + per : nb;
    uint32_t s = 0;
    for (size_t i = b0; i < b1; ++i) s += sums[i];
    uint32_t total;
    uint32_t run = block_exclusive<kPartialThreads>(s, lds, total);
    for (size_t i = b0; i < b1; ++i) {
        const uint32_t t = sums[i];
        sums[i] = run;
        run += t;
    }
    if (threadIdx.x == 0 && total_dev) *total_dev = total;
}

__global__ __launch_bounds__(kThreads) void k_scan_final(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         size_t n, const uint32_t* __restrict__ block_off) {
    __shared__ uint32_t lds[kThreads / 64];
    const size_t base = (size_t)blockIdx.x * kTileItems + (size_t)threadIdx.x * kItems;
    uint32_t v[kItems];
    load16(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) s += v[k];
    uint32_t total;
    uint32_t run = block_exclusive<kThreads>(s, lds, total) + block_off[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
        const uint32_t t = v[k];
        v[k] = run;
        run += t;
    }
    if (base + kItems <= n) {
        uint4* p = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < kItems; ++k)
            if (base + k < n) out[base + k] = v[k];
    }
}

}  // namespace

size_t scan_tmp_elems(size_t n) {
    const size_t nb = (n + kTileItems - 1) / kTileItems;
    return nb < 1 ? 1 : nb;
}

int scan_exclusive(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp,
                   uint32_t* total_dev, hipStream_t s) {
    if (n == 0) {
        if (total_dev) GSR_HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(uint32_t), s));
        return GSR_OK;
    }
    const size_t nb = (n + kTileItems - 1) / kTileItems;
    k_scan_reduce<<<dim3((unsigned)nb), dim3(kThreads), 0, s>>>(in, n, tmp);
    GSR_LAUNCH_CHECK("scan_reduce");
    k_scan_partials<<<1, kPartialThreads, 0, s>>>(tmp, nb, total_dev);
    GSR_LAUNCH_CHECK("scan_partials");
    k_scan_final<<<dim3((unsigned)nb), dim3(kThreads), 0, s>>>(in, out, n, tmp);
    GSR_LAUNCH_CHECK("scan_final");
    return GSR_OK;
}

}  // namespace gsr

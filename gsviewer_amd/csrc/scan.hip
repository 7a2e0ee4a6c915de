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
constexpr size_t kSingleMax = 131072;  // single-workgroup scan up to this many elements
// Short single-workgroup scans (<= 1024 entries) run as 4-wave blocks: a
// 16-wave block waits for a whole CU's worth of free slots while other views'
// compositors hold the chip (in flight a 1024-thread scan of the binning's
// block sums averaged 68 us against 4.5 us alone; the binning now sums those
// itself, bin_write).  Longer ones (the visibility words, ~16k at 1M) keep 16
// waves: with 4 the cull stage took 8 us longer alone.
constexpr int kSingleThreads = 256;
constexpr size_t kSmallScan = 4 * kSingleThreads;  // one chunk of the 256-thread scan

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
// Optional side job of the single-block kernels: componentwise max over n_kr
// uint2 entries (the per-block depth-key ranges {~kmin, kmax} of k_cull) into
// kr_out[0..1].
template <int NT>
__device__ __forceinline__ void reduce_ranges(const uint2* __restrict__ kr_in, size_t n_kr, uint32_t* __restrict__ kr_out,
                                              uint2* lds) {
    uint2 m = make_uint2(0u, 0u);
    for (size_t i = threadIdx.x; i < n_kr; i += NT) {
        const uint2 v = kr_in[i];
        m.x = max(m.x, v.x);
        m.y = max(m.y, v.y);
    }
    m.x = wave_reduce_max(m.x);
    m.y = wave_reduce_max(m.y);
    if (__lane_id() == 0) lds[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NT / 64; ++w) {
            m.x = max(m.x, lds[w].x);
            m.y = max(m.y, lds[w].y);
        }
        kr_out[0] = m.x;
        kr_out[1] = m.y;
    }
}

__global__ __launch_bounds__(kPartialThreads) void k_scan_partials(uint32_t* __restrict__ sums, size_t nb,
                                                                   uint32_t* __restrict__ total_dev,
                                                                   const uint2* __restrict__ kr_in, size_t n_kr,
                                                                   uint32_t* __restrict__ kr_out) {
    __shared__ uint32_t lds[kPartialThreads / 64];
    __shared__ uint2 lds_kr[kPartialThreads / 64];
    if (kr_in) reduce_ranges<kPartialThreads>(kr_in, n_kr, kr_out, lds_kr);
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

// One workgroup scans everything (n up to ~1e5): one launch instead of three
// for the small arrays of a frame (wave counts, tiles, block sums).  The array
// is walked in 4096-element chunks: coalesced dwordx4 loads (next chunk
// prefetched), a block scan per chunk, a running carry.
template <int NT>
__device__ __forceinline__ void scan_single(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n,
                                            uint32_t* __restrict__ total_dev, uint32_t (*lds)[NT / 64]) {
    constexpr size_t kChunk = 4 * NT;
    const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
    auto load4 = [&](size_t c, uint32_t (&v)[4]) {
        const size_t i = c * kChunk + 4 * (size_t)threadIdx.x;
        if (aligned && i + 4 <= n) {
            const uint4 t = *reinterpret_cast<const uint4*>(in + i);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
        } else {
            for (int k = 0; k < 4; ++k) v[k] = (i + k < n) ? in[i + k] : 0u;
        }
    };
    const size_t nchunks = (n + kChunk - 1) / kChunk;
    uint32_t carry = 0;
    uint32_t cur[4];
    load4(0, cur);
    for (size_t c = 0; c < nchunks; ++c) {
        uint32_t nxt[4] = {0u, 0u, 0u, 0u};
        if (c + 1 < nchunks) load4(c + 1, nxt);
        const uint32_t s = cur[0] + cur[1] + cur[2] + cur[3];
        uint32_t total;
        uint32_t run = carry + block_exclusive<NT>(s, lds[c & 1], total);
        const size_t i = c * kChunk + 4 * (size_t)threadIdx.x;
        uint32_t o[4];
        for (int k = 0; k < 4; ++k) {
            o[k] = run;
            run += cur[k];
        }
        if (aligned && i + 4 <= n) {
            *reinterpret_cast<uint4*>(out + i) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            for (int k = 0; k < 4; ++k)
                if (i + k < n) out[i + k] = o[k];
        }
        carry += total;
        for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
    }
    if (threadIdx.x == 0 && total_dev) *total_dev = carry;
}

// One pass for arrays of at most NT * 16 elements (the visibility words of up
// to ~1M Gaussians): each thread loads 16 contiguous elements (four dwordx4,
// issued with the key-range loads), one block scan, 16 stores.  The chunked
// loop above walks 4 chunks of 4096 with a block scan each (10 us for 15.6K
// words; this: one round of loads and two barriers).
constexpr int kOnePassItems = 16;

template <int NT>
__device__ __forceinline__ void scan_one_pass(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n,
                                              uint32_t* __restrict__ total_dev, const uint2* __restrict__ kr_in,
                                              size_t n_kr, uint32_t* __restrict__ kr_out, uint32_t* lds,
                                              uint2* lds_kr) {
    constexpr int IT = kOnePassItems;
    const size_t base = (size_t)threadIdx.x * IT;
    uint32_t v[IT];
    const bool aligned = (reinterpret_cast<uintptr_t>(in) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
    if (aligned && base + IT <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
        for (int q = 0; q < IT / 4; ++q) {
            const uint4 t = p[q];
            v[4 * q + 0] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < IT; ++k) v[k] = (base + k < n) ? in[base + k] : 0u;
    }
    if (kr_in) reduce_ranges<NT>(kr_in, n_kr, kr_out, lds_kr);
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < IT; ++k) sum += v[k];
    uint32_t total;
    uint32_t run = block_exclusive<NT>(sum, lds, total);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const uint32_t t = v[k];
        v[k] = run;
        run += t;
    }
    if (aligned && base + IT <= n) {
        uint4* p = reinterpret_cast<uint4*>(out + base);
#pragma unroll
        for (int q = 0; q < IT / 4; ++q) p[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (base + k < n) out[base + k] = v[k];
    }
    if (threadIdx.x == 0 && total_dev) *total_dev = total;
}

__global__ __launch_bounds__(kPartialThreads) void k_scan_one_pass(const uint32_t* __restrict__ in,
                                                                   uint32_t* __restrict__ out, size_t n,
                                                                   uint32_t* __restrict__ total_dev,
                                                                   const uint2* __restrict__ kr_in, size_t n_kr,
                                                                   uint32_t* __restrict__ kr_out) {
    __shared__ uint32_t lds[kPartialThreads / 64];
    __shared__ uint2 lds_kr[kPartialThreads / 64];
    scan_one_pass<kPartialThreads>(in, out, n, total_dev, kr_in, n_kr, kr_out, lds, lds_kr);
}

// The visibility scans of a group of views (gsr_render_begin_views) in one
// launch, one workgroup per view (blockIdx.y).
struct ScanViews {
    const uint32_t* in[kMaxViews];
    uint32_t* out[kMaxViews];
    uint32_t* total[kMaxViews];
    const uint2* kr_in[kMaxViews];
    uint32_t* kr_out[kMaxViews];
};

__global__ __launch_bounds__(kPartialThreads) void k_scan_one_pass_views(ScanViews sv, size_t n, size_t n_kr) {
    __shared__ uint32_t lds[kPartialThreads / 64];
    __shared__ uint2 lds_kr[kPartialThreads / 64];
    const int v = blockIdx.y;
    scan_one_pass<kPartialThreads>(sv.in[v], sv.out[v], n, sv.total[v], sv.kr_in[v], n_kr, sv.kr_out[v], lds, lds_kr);
}

template <int NT>
__global__ __launch_bounds__(NT) void k_scan_single(const uint32_t* __restrict__ in,
                                                                 uint32_t* __restrict__ out, size_t n,
                                                                 uint32_t* __restrict__ total_dev,
                                                                 const uint2* __restrict__ kr_in, size_t n_kr,
                                                                 uint32_t* __restrict__ kr_out) {
    __shared__ uint32_t lds[2][NT / 64];
    __shared__ uint2 lds_kr[NT / 64];
    if (kr_in) reduce_ranges<NT>(kr_in, n_kr, kr_out, lds_kr);
    scan_single<NT>(in, out, n, total_dev, lds);
}

}  // namespace

size_t scan_tmp_elems(size_t n) {
    const size_t nb = (n + kTileItems - 1) / kTileItems;
    return nb < 1 ? 1 : nb;
}

int scan_exclusive(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp,
                   uint32_t* total_dev, hipStream_t s, const uint2* kr_in, size_t n_kr, uint32_t* kr_out) {
    if (n == 0) {
        if (total_dev) GSR_HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(uint32_t), s));
        if (kr_out) GSR_HIP_CHECK(hipMemsetAsync(kr_out, 0, 2 * sizeof(uint32_t), s));
        return GSR_OK;
    }
    if (n <= kSingleMax) {
        if (n <= kSmallScan)
            k_scan_single<kSingleThreads><<<1, kSingleThreads, 0, s>>>(in, out, n, total_dev, kr_in, n_kr, kr_out);
        else if (n <= (size_t)kPartialThreads * kOnePassItems)
            k_scan_one_pass<<<1, kPartialThreads, 0, s>>>(in, out, n, total_dev, kr_in, n_kr, kr_out);
        else
            k_scan_single<kPartialThreads><<<1, kPartialThreads, 0, s>>>(in, out, n, total_dev, kr_in, n_kr, kr_out);
        GSR_LAUNCH_CHECK("scan_single");
        return GSR_OK;
    }
    if (!tmp) return set_error(GSR_ERR_INVALID, "scan: temporary buffer required for large n");
    const size_t nb = (n + kTileItems - 1) / kTileItems;
    k_scan_reduce<<<dim3((unsigned)nb), dim3(kThreads), 0, s>>>(in, n, tmp);
    GSR_LAUNCH_CHECK("scan_reduce");
    k_scan_partials<<<1, kPartialThreads, 0, s>>>(tmp, nb, total_dev, kr_in, n_kr, kr_out);
    GSR_LAUNCH_CHECK("scan_partials");
    k_scan_final<<<dim3((unsigned)nb), dim3(kThreads), 0, s>>>(in, out, n, tmp);
    GSR_LAUNCH_CHECK("scan_final");
    return GSR_OK;
}

bool scan_views_fits(size_t n) { return n > 0 && n <= (size_t)kPartialThreads * kOnePassItems; }

int scan_exclusive_views(const uint32_t* const* in, uint32_t* const* out, size_t n, uint32_t* const* total_dev,
                         const uint2* const* kr_in, size_t n_kr, uint32_t* const* kr_out, int k, hipStream_t s) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "scan: view count out of range");
    if (!scan_views_fits(n)) return set_error(GSR_ERR_INVALID, "scan: array too long for the batched one-pass scan");
    ScanViews sv{};
    for (int v = 0; v < k; ++v) {
        sv.in[v] = in[v];
        sv.out[v] = out[v];
        sv.total[v] = total_dev[v];
        sv.kr_in[v] = kr_in[v];
        sv.kr_out[v] = kr_out[v];
    }
    k_scan_one_pass_views<<<dim3(1, (unsigned)k), kPartialThreads, 0, s>>>(sv, n, n_kr);
    GSR_LAUNCH_CHECK("scan_one_pass_views");
    return GSR_OK;
}

}  // namespace gsr

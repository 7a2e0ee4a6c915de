// Stable LSD radix sort of (uint32 key, uint32 value) pairs, 8-bit digits.
//
// One pass = three launches:
//   k_radix_hist   per 1024-item block digit counts (wave digit matching, no
//                  atomics of any kind), stored digit-major;
//   k_radix_offsets one workgroup per digit: exclusive scan of that digit's
//                  row of block counts (in place) and the row total;
//   k_radix_scatter scans the 256 row totals itself (digit bases), then ranks
//                  stably in-block with wave-level digit matching (8 ballots
//                  per 64 items; waves own consecutive item ranges), stages in
//                  LDS in digit order and writes contiguous runs.
// The element count may live in device memory (n_dev): grids are sized by a
// host-side upper bound and blocks past the device count do nothing, so a
// frame needs no host round trip to size its sorts.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRounds = 4;                       // 64-item rounds per wave
constexpr int kBlockItems = kThreads * kRounds;  // 1024: enough blocks to fill 256 CUs at 1M keys
constexpr int kRadix = 256;

__device__ __forceinline__ uint32_t count_of(const uint32_t* n_dev, uint32_t n_host) {
    return n_dev ? min(n_host, n_dev[0]) : n_host;
}

__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ n_dev, uint32_t n_host, int shift,
                                                         uint32_t* __restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[kWaves][kRadix];
    const uint32_t n = count_of(n_dev, n_host);
    const uint32_t block0 = blockIdx.x * kBlockItems;
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
    const int w = threadIdx.x >> 6;
    const uint32_t base = block0 + w * (kBlockItems / kWaves) + __lane_id();
    uint32_t d[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {  // issue every load first
        const uint32_t i = base + r * 64;
        d[r] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
    if (block0 < n) {
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            const bool valid = base + r * 64 < n;
            const uint32_t dg = (d[r] >> shift) & 0xffu;
            const uint64_t peers = match_digit8(dg, valid);
            if (valid && (peers & lanemask_lt()) == 0) h[w][dg] += (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    const int dg = threadIdx.x;  // kThreads == kRadix
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) s += h[k][dg];
    hist[(size_t)dg * nblocks + blockIdx.x] = s;
}

// Block d: exclusive scan of row d (nblocks counts) in place; row total out.
__global__ __launch_bounds__(kThreads) void k_radix_offsets(uint32_t* __restrict__ hist, uint32_t nblocks,
                                                            uint32_t* __restrict__ totals) {
    __shared__ uint32_t lds[kWaves];
    const int d = blockIdx.x;
    const int w = threadIdx.x >> 6;
    uint32_t* row = hist + (size_t)d * nblocks;
    const uint32_t per = (nblocks + kThreads - 1) / kThreads;
    const uint32_t b0 = threadIdx.x * per;
    const uint32_t b1 = min(nblocks, b0 + per);
    uint32_t s = 0;
    for (uint32_t i = b0; i < b1; ++i) s += row[i];
    const uint32_t inc = wave_inclusive_scan(s);
    if (__lane_id() == 63) lds[w] = inc;
    __syncthreads();
    uint32_t run = inc - s, tot = 0;
    for (int k = 0; k < kWaves; ++k) {
        run += (k < w) ? lds[k] : 0u;
        tot += lds[k];
    }
    for (uint32_t i = b0; i < b1; ++i) {
        const uint32_t t = row[i];
        row[i] = run;
        run += t;
    }
    if (threadIdx.x == 0) totals[d] = tot;
}

__global__ __launch_bounds__(kThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, bool identity_vals,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* __restrict__ n_dev,
    uint32_t n_host, int shift, const uint32_t* __restrict__ hist_off, const uint32_t* __restrict__ totals,
    uint32_t nblocks) {
    __shared__ uint32_t s_keys[kBlockItems];
    __shared__ uint32_t s_vals[kBlockItems];
    __shared__ uint32_t wcnt[kWaves][kRadix];  // per-wave digit counts, then per-wave prefixes
    __shared__ uint32_t dbase[kRadix];         // block-local exclusive digit offsets
    __shared__ uint32_t gbase[kRadix];         // global offset of this block's digit run
    __shared__ uint32_t wsum[kWaves];

    const uint32_t n = count_of(n_dev, n_host);
    const uint32_t block0 = blockIdx.x * kBlockItems;
    if (block0 >= n) return;
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&wcnt[0][0])[i] = 0;

    const int w = threadIdx.x >> 6;
    const uint32_t base = block0 + w * (kBlockItems / kWaves) + __lane_id();
    const uint64_t lt = lanemask_lt();

    uint32_t k_reg[kRounds], v_reg[kRounds], rank[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {  // issue every load first
        const uint32_t i = base + r * 64;
        const bool valid = i < n;
        k_reg[r] = valid ? keys_in[i] : 0xffffffffu;
        v_reg[r] = valid ? (identity_vals ? i : vals_in[i]) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const bool valid = base + r * 64 < n;
        const uint32_t d = (k_reg[r] >> shift) & 0xffu;
        const uint64_t peers = match_digit8(d, valid);
        uint32_t rk = 0xffffffffu;
        if (valid) {
            const uint32_t old = wcnt[w][d];
            rk = old + (uint32_t)__popcll(peers & lt);
            if ((peers & lt) == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
        }
        rank[r] = rk;
    }
    __syncthreads();

    {  // per digit: wave prefixes, block-local digit offsets, global run base
        const int d = threadIdx.x;
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) {
            const uint32_t c = wcnt[k][d];
            wcnt[k][d] = tot;
            tot += c;
        }
        const uint32_t inc = wave_inclusive_scan(tot);
        if (__lane_id() == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t woff = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) woff += (k < w) ? wsum[k] : 0u;
        dbase[d] = woff + inc - tot;
        // digit base = exclusive scan of the row totals over digits
        const uint32_t t = totals[d];
        const uint32_t tinc = wave_inclusive_scan(t);
        __syncthreads();
        if (__lane_id() == 63) wsum[w] = tinc;
        __syncthreads();
        uint32_t tb = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) tb += (k < w) ? wsum[k] : 0u;
        gbase[d] = tb + tinc - t + hist_off[(size_t)d * nblocks + blockIdx.x];
    }
    __syncthreads();

#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        if (rank[r] != 0xffffffffu) {
            const uint32_t d = (k_reg[r] >> shift) & 0xffu;
            const uint32_t p = dbase[d] + wcnt[w][d] + rank[r];
            s_keys[p] = k_reg[r];
            s_vals[p] = v_reg[r];
        }
    }
    __syncthreads();

    const uint32_t cnt = min(n - block0, (uint32_t)kBlockItems);
    for (uint32_t j = threadIdx.x; j < cnt; j += kThreads) {
        const uint32_t key = s_keys[j];
        const uint32_t d = (key >> shift) & 0xffu;
        const uint32_t g = gbase[d] + (j - dbase[d]);
        keys_out[g] = key;
        vals_out[g] = s_vals[j];
    }
}

}  // namespace

size_t radix_tmp_elems(size_t n) {
    const size_t nb = (n + kBlockItems - 1) / kBlockItems;
    return (nb < 1 ? 1 : nb) * kRadix;
}

size_t radix_totals_elems() { return (size_t)kRadix; }  // digit totals scratch (rewritten every pass)

int radix_sort_pairs(uint32_t** keys_io, uint32_t** vals_io, uint32_t** keys_alt, uint32_t** vals_alt,
                     bool identity_vals, size_t n, const uint32_t* n_dev, int begin_bit, int end_bit, uint32_t* tmp,
                     uint32_t* totals, hipStream_t s) {
    if (n == 0) return GSR_OK;
    if (n > 0xffffffffull - kBlockItems) return set_error(GSR_ERR_OVERFLOW, "radix sort: n too large");
    if ((end_bit - begin_bit + 7) / 8 > 4) return set_error(GSR_ERR_INVALID, "radix sort: more than 4 passes");
    const uint32_t nb = (uint32_t)((n + kBlockItems - 1) / kBlockItems);
    uint32_t* hist = tmp;
    bool ident = identity_vals;
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        k_radix_hist<<<nb, kThreads, 0, s>>>(*keys_io, n_dev, (uint32_t)n, shift, hist, nb);
        GSR_LAUNCH_CHECK("radix_hist");
        k_radix_offsets<<<kRadix, kThreads, 0, s>>>(hist, nb, totals);
        GSR_LAUNCH_CHECK("radix_offsets");
        k_radix_scatter<<<nb, kThreads, 0, s>>>(*keys_io, *vals_io, ident, *keys_alt, *vals_alt, n_dev, (uint32_t)n,
                                                shift, hist, totals, nb);
        GSR_LAUNCH_CHECK("radix_scatter");
        ident = false;
        uint32_t* t = *keys_io; *keys_io = *keys_alt; *keys_alt = t;
        t = *vals_io; *vals_io = *vals_alt; *vals_alt = t;
    }
    return GSR_OK;
}

}  // namespace gsr

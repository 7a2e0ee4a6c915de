// Stable LSD radix sort of (uint32 key, uint32 value) pairs, 8-bit digits.
//
// One pass = histogram (per 4096-item block, digit-major) -> exclusive scan of
// the digit-major histogram (= every block's global digit offsets) -> scatter.
// The scatter ranks items stably inside the block with wave-level digit
// matching (8 ballots per round, 64 items per round, waves in item order),
// stages the block's items in LDS in digit order and then writes them out in
// digit runs, so global stores are contiguous per run.
//
// Items of block b are [b*4096, (b+1)*4096); wave w of the block owns
// [w*1024, (w+1)*1024) of them in 16 rounds of 64 consecutive items, so the
// global load of each round is one coalesced 256-B line per array.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kRounds = 16;
constexpr int kBlockItems = kThreads * kRounds;  // 4096
constexpr int kRadix = 256;

__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint32_t* __restrict__ keys, uint32_t n,
                                                         int shift, uint32_t* __restrict__ hist,
                                                         uint32_t nblocks) {
    __shared__ uint32_t h[kWaves][kRadix];
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int w = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * kBlockItems + w * (kBlockItems / kWaves) + __lane_id();
#pragma unroll 4
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = base + r * 64;
        const bool valid = i < n;
        const uint32_t d = valid ? ((keys[i] >> shift) & 0xffu) : 0u;
        const uint64_t peers = match_digit8(d, valid);
        if (valid && (peers & lanemask_lt()) == 0) h[w][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    const int d = threadIdx.x;  // kThreads == kRadix
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) s += h[k][d];
    hist[(size_t)d * nblocks + blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, bool identity_vals,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, uint32_t n, int shift,
    const uint32_t* __restrict__ hist_off, uint32_t nblocks) {
    __shared__ uint32_t s_keys[kBlockItems];
    __shared__ uint32_t s_vals[kBlockItems];
    __shared__ uint32_t wcnt[kWaves][kRadix];  // per-wave digit counts, then per-wave prefixes
    __shared__ uint32_t dbase[kRadix];         // block-local exclusive digit offsets
    __shared__ uint32_t gbase[kRadix];         // global offset of this block's digit run
    __shared__ uint32_t wsum[kWaves];

    for (int i = threadIdx.x; i < kWaves * kRadix; i += kThreads) (&wcnt[0][0])[i] = 0;
    __syncthreads();

    const int w = threadIdx.x >> 6;
    const uint32_t block0 = blockIdx.x * kBlockItems;
    const uint32_t base = block0 + w * (kBlockItems / kWaves) + __lane_id();
    const uint64_t lt = lanemask_lt();

    uint32_t k_reg[kRounds], v_reg[kRounds], rank[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = base + r * 64;
        const bool valid = i < n;
        const uint32_t key = valid ? keys_in[i] : 0xffffffffu;
        const uint32_t val = valid ? (identity_vals ? i : vals_in[i]) : 0u;
        const uint32_t d = (key >> shift) & 0xffu;
        const uint64_t peers = match_digit8(d, valid);
        uint32_t rk = 0;
        if (valid) {
            const uint32_t old = wcnt[w][d];
            rk = old + (uint32_t)__popcll(peers & lt);
            if ((peers & lt) == 0) wcnt[w][d] = old + (uint32_t)__popcll(peers);
        }
        k_reg[r] = key;
        v_reg[r] = val;
        rank[r] = valid ? rk : 0xffffffffu;
    }
    __syncthreads();

    // Per digit: wave prefixes, block-local digit offsets, global run base.
    {
        const int d = threadIdx.x;
        uint32_t c[kWaves];
        uint32_t tot = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) {
            c[k] = wcnt[k][d];
            wcnt[k][d] = tot;  // exclusive prefix over waves
            tot += c[k];
        }
        // block-wide exclusive scan of tot over the 256 digits
        const uint32_t inc = wave_inclusive_scan(tot);
        if (__lane_id() == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t woff = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) woff += (k < w) ? wsum[k] : 0u;
        dbase[d] = woff + inc - tot;
        gbase[d] = hist_off[(size_t)d * nblocks + blockIdx.x];
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

    const uint32_t cnt = (n > block0) ? ((n - block0 < (uint32_t)kBlockItems) ? n - block0 : kBlockItems) : 0u;
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
    const size_t h = (nb < 1 ? 1 : nb) * kRadix;
    return h + scan_tmp_elems(h);
}

int radix_sort_pairs(uint32_t** keys_io, uint32_t** vals_io, uint32_t** keys_alt,
                     uint32_t** vals_alt, bool identity_vals, size_t n, int begin_bit,
                     int end_bit, uint32_t* tmp, hipStream_t s) {
    if (n == 0) return GSR_OK;
    if (n > 0xffffffffull - kBlockItems) return set_error(GSR_ERR_OVERFLOW, "radix sort: n too large");
    const uint32_t nb = (uint32_t)((n + kBlockItems - 1) / kBlockItems);
    uint32_t* hist = tmp;
    uint32_t* scan_tmp = tmp + (size_t)nb * kRadix;
    bool ident = identity_vals;
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        k_radix_hist<<<nb, kThreads, 0, s>>>(*keys_io, (uint32_t)n, shift, hist, nb);
        GSR_LAUNCH_CHECK("radix_hist");
        int rc = scan_exclusive(hist, hist, (size_t)nb * kRadix, scan_tmp, nullptr, s);
        if (rc) return rc;
        k_radix_scatter<<<nb, kThreads, 0, s>>>(*keys_io, *vals_io, ident, *keys_alt, *vals_alt,
                                                (uint32_t)n, shift, hist, nb);
        GSR_LAUNCH_CHECK("radix_scatter");
        ident = false;
        uint32_t* t = *keys_io; *keys_io = *keys_alt; *keys_alt = t;
        t = *vals_io; *vals_io = *vals_alt; *vals_alt = t;
    }
    return GSR_OK;
}

}  // namespace gsr

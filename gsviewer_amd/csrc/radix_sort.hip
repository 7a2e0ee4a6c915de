// Stable LSD radix sort of (uint32 key, uint32 value) pairs.
//
// Digit width is chosen per sort, up to 11 bits, so that a 32-bit key needs at
// most 3 passes.  For the depth sort the width is chosen ON THE DEVICE: the
// preprocess records the key range [kmin, kmax] of the frame, keys are sorted
// as key - kmin, and B = bits(kmax - kmin) is split over the host's fixed
// number of passes (w = ceil(B / passes)): a camera's visible depths span
// ~24-27 of the 32 key bits, so 4 passes of <= 8 bits (frames in flight) or 3
// of <= 11 (a frame rendered alone) cover any B and the host never has to
// know it.
//
// One pass = three launches over tiles of 256*R items:
//   k_rs_upsweep   per-tile digit counts (LDS atomics: counts need no
//                  order), stored digit-major: hist[d * ntiles + tile];
//   k_rs_offsets   one wave per digit (4 per block): exclusive scan of that digit's row
//                  (in place) and the row total;
//   k_rs_scatter   digit bases (block scan of the row totals), stable in-tile
//                  ranks (waves own consecutive 64*R-item ranges, R rounds of
//                  64), staged in LDS in digit order, written as contiguous
//                  runs.  The digit bases and this tile's row offsets are
//                  loaded before the keys are ranked, so their latency hides
//                  behind the ranking.
// The element count may live in device memory (n_dev): grids are sized by a
// host-side upper bound and tiles past the device count do nothing, so a
// frame needs no host round trip to size its sorts.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
// Items per thread (64-item rounds per wave) is a template parameter R: a
// tile holds 256*R items.  Bigger tiles mean longer digit runs in the
// scatter's writes and a smaller digit matrix, but fewer blocks to fill the
// chip; every sort uses R = 8 (GSR_*_R build knobs for A/B).
// items per thread for wide digits (> 8 bits: the depth sort); build knob for A/B
#ifndef GSR_WIDE_R
#define GSR_WIDE_R 8
#endif
constexpr int kRWide = GSR_WIDE_R;
// items per thread for device-chosen <= 8-bit digits (the depth sort); build knob for A/B
#ifndef GSR_DEPTH_R
#define GSR_DEPTH_R 8
#endif
constexpr int kRDepth = GSR_DEPTH_R;
// ... and for depth sorts of more than kBigDepthN keys: 4096-key tiles (C3's 6M keys: 2 passes 180 -> 155 us;
// C2's 1M: 53 -> 58 us, profiles/r5_s22)
constexpr int kRDepthBig = 16;
constexpr size_t kBigDepthN = (size_t)1 << 21;
// items per thread for host-known <= 8-bit digits (the tile sort); build knob for A/B.
// 8 since the binning took over the tile sort's first pass: its one remaining
// pass (1.76M instances at C2) ran 1.8 us faster in 2048-item tiles than in
// 4096 (profiles/r3_s32)
#ifndef GSR_TILE_R
#define GSR_TILE_R 8
#endif
constexpr int kRTile = GSR_TILE_R;
// ... and for tile sorts of more than kBigTileN instances (C3's 10.6 M): 4096-item tiles like the big depth sorts
#ifndef GSR_BIG_TILE_N
#define GSR_BIG_TILE_N 0xffffffffu
#endif
constexpr size_t kBigTileN = GSR_BIG_TILE_N;
constexpr int kRMin = kRWide < kRDepth ? (kRWide < kRTile ? kRWide : kRTile) : (kRDepth < kRTile ? kRDepth : kRTile);
constexpr int kMinTileItems = kThreads * kRMin;  // sizes the digit matrix for any R

constexpr int kMaxBits = 11;
constexpr int kMaxRadix = 1 << kMaxBits;         // 2048
// LDS of a pass is sized for its largest radix (kCB: cap bits): the host
// knows the widest digit a sort can have (ceil(bits / passes)), and sorts of
// <= 8-bit digits use kernels sized for 256 digits (about 20 KB less LDS per
// block: more blocks per CU beside the compositor when views are in flight)
template <int kCB>
constexpr int radix_cap() { return 1 << kCB; }
template <int kCB>
constexpr int digits_per_thread() { return radix_cap<kCB>() / kThreads; }

__device__ __forceinline__ uint32_t count_of(const uint32_t* n_dev, uint32_t n_host, const PassArgs& pa) {
    return n_dev && !pa.drop ? min(n_host, n_dev[0]) : n_host;
}

// Per-tile digit counts: one LDS histogram per block, counted with LDS atomics
// (counts need no order; the scatter's stable ranks use digit matching).  The
// ballot-per-digit-bit matching the scatter needs cost ~8 VALU per digit bit
// and item here, and with views in flight the chip is VALU-issue bound.
template <int kR, int kCB>
__device__ __forceinline__ void rs_upsweep(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ n_dev,
                                           uint32_t n_host, const PassArgs& pa, uint32_t* __restrict__ hist,
                                           uint32_t ntiles, uint32_t tile) {
    constexpr int kTileItems = kThreads * kR;
    constexpr int kCap = radix_cap<kCB>();
    __shared__ uint32_t h[kCap];
    const Digit dg = digit_params(pa);
    const uint32_t radix = dg.mask + 1u;
    const uint32_t n = count_of(n_dev, n_host, pa);
    const uint32_t tile0 = tile * kTileItems;
#pragma unroll
    for (int i = 0; i < (kCap + kThreads - 1) / kThreads; ++i)
        if (i * kThreads + (int)threadIdx.x < kCap) h[i * kThreads + threadIdx.x] = 0u;
    const int w = threadIdx.x >> 6;
    const uint32_t base = tile0 + w * (kTileItems / kWaves) + __lane_id();
    uint32_t k[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {  // issue every load first
        const uint32_t i = base + r * 64;
        k[r] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
    if (tile0 < n) {
#pragma unroll
        for (int r = 0; r < kR; ++r)
            if (base + r * 64 < n && (!pa.drop || dg.keep(k[r]))) atomicAdd(&h[dg.of(k[r])], 1u);
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < radix; d += kThreads) hist[(size_t)d * ntiles + tile] = h[d];
}

template <int kR, int kCB>
__global__ __launch_bounds__(kThreads) void k_rs_upsweep(const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ n_dev, uint32_t n_host,
                                                         PassArgs pa, uint32_t* __restrict__ hist, uint32_t ntiles) {
    rs_upsweep<kR, kCB>(keys, n_dev, n_host, pa, hist, ntiles, blockIdx.x);
}

// One wave per digit d: exclusive scan of row d (ntiles counts) in place; row total out.
// Rows of up to 64 * kOffRegs counts (2048-key tiles: 2M keys): lane l owns
// the consecutive counts [l per, (l + 1) per), all loaded in one round trip.
// Longer rows (C3: 2930 depth-sort tiles, 5860 binning blocks, 5190 tile-sort
// tiles) lane-interleaved, count i = 64 r + lane in round r, kOffRegs rounds
// of coalesced loads in flight, a wave scan per round: round 4's lane-owned
// segments made every load instruction touch 64 lines (20-44 us per pass at
// C3, profiles/r5_s16; ~5 us now).
constexpr uint32_t kOffRegs = 16;
__device__ __forceinline__ void rs_offsets(uint32_t* __restrict__ hist, uint32_t ntiles, const PassArgs& pa,
                                           uint32_t* __restrict__ totals, uint32_t d) {
    const Digit dg = digit_params(pa);
    if (d > dg.mask) return;
    uint32_t* row = hist + (size_t)d * ntiles;
    const uint32_t per = (ntiles + 63) / 64;
    const uint32_t lane = __lane_id();
    if (per <= kOffRegs) {
        const uint32_t b0 = lane * per;
        const uint32_t b1 = min(ntiles, b0 + per);
        uint32_t c[kOffRegs];
#pragma unroll
        for (uint32_t k = 0; k < kOffRegs; ++k) c[k] = b0 + k < b1 ? row[b0 + k] : 0u;
        uint32_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < kOffRegs; ++k) s += c[k];
        const uint32_t inc = wave_inclusive_scan(s);
        uint32_t run = inc - s;
#pragma unroll
        for (uint32_t k = 0; k < kOffRegs; ++k) {
            if (b0 + k < b1) row[b0 + k] = run;
            run += c[k];
        }
        if (lane == 63) totals[d] = inc;
        return;
    }
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < ntiles; r0 += 64 * kOffRegs) {
        uint32_t c[kOffRegs];
#pragma unroll
        for (uint32_t k = 0; k < kOffRegs; ++k) {
            const uint32_t i = r0 + k * 64 + lane;
            c[k] = i < ntiles ? row[i] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kOffRegs; ++k) {
            const uint32_t i = r0 + k * 64 + lane;
            const uint32_t inc = wave_inclusive_scan(c[k]);
            if (i < ntiles) row[i] = carry + inc - c[k];
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        }
    }
    if (lane == 0) totals[d] = carry;
}

// 4 digits per 256-thread block (one wave each): a quarter of the workgroups
// of one-wave blocks, which queued for CU slots behind other views' kernels
constexpr int kOffWaves = 4;

__global__ __launch_bounds__(64 * kOffWaves) void k_rs_offsets(uint32_t* __restrict__ hist, uint32_t ntiles,
                                                               PassArgs pa, uint32_t* __restrict__ totals) {
    rs_offsets(hist, ntiles, pa, totals, blockIdx.x * kOffWaves + (threadIdx.x >> 6));
}

// Tile rectangle of a splat packed in 32 bits (tx0 | tx1 << 8 | ty0 << 16 |
// ty1 << 24) for frames of at most 256 x 256 tiles; empty: tx0 > tx1.
__device__ __forceinline__ uint32_t pack_rect(uint2 tr) {
    const uint32_t tx0 = tr.x & 0xffffu, tx1 = tr.x >> 16, ty0 = tr.y & 0xffffu, ty1 = tr.y >> 16;
    return tx0 > tx1 ? 0xffu : (tx0 | tx1 << 8 | ty0 << 16 | ty1 << 24);
}

// kPay: a 32-bit payload travels with each pair (the packed tile rectangle of
// the depth sort, so the binning reads it in sorted order instead of
// gathering it by id).  Its first pass reads the rectangles (rect_in, in
// input order) and packs them; later passes read pay_in.
template <int kR, bool kPay, int kCB>
__device__ __forceinline__ void rs_scatter(const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in,
                                           bool identity_vals, uint32_t* __restrict__ keys_out,
                                           uint32_t* __restrict__ vals_out, const uint32_t* __restrict__ n_dev,
                                           uint32_t n_host, const PassArgs& pa,
                                           const uint32_t* __restrict__ hist_off,
                                           const uint32_t* __restrict__ totals, uint32_t ntiles, uint32_t tile,
                                           const uint2* __restrict__ rect_in = nullptr,
                                           const uint32_t* __restrict__ pay_in = nullptr,
                                           uint32_t* __restrict__ pay_out = nullptr) {
    constexpr int kTileItems = kThreads * kR;
    __shared__ uint32_t s_keys[kTileItems];
    __shared__ uint32_t s_vals[kTileItems];
    __shared__ uint32_t s_pay[kPay ? kTileItems : 1];
    // per-wave digit counts, then per-wave prefixes; after the LDS staging the
    // same bytes hold gbase[d], the global position of LDS index 0 of digit d's
    // run (kept in registers until then): 8 KB less LDS per block, so 3
    // blocks fit a CU instead of 2 for 2048-item tiles
    constexpr int kCap = radix_cap<kCB>();
    constexpr int kDigitsPerThread = digits_per_thread<kCB>();
    __shared__ uint32_t wcnt_gbase[kWaves * kCap / 2];
    static_assert(kWaves * kCap / 2 >= kCap, "gbase overlay");
    uint16_t(&wcnt)[kWaves][kCap] = *reinterpret_cast<uint16_t(*)[kWaves][kCap]>(wcnt_gbase);
    uint32_t* gbase = wcnt_gbase;
    __shared__ uint32_t dbase[kCap];              // tile-local exclusive digit offsets
    __shared__ uint32_t wsum[2][kWaves];

    const uint32_t n = count_of(n_dev, n_host, pa);
    const uint32_t tile0 = tile * kTileItems;
    if (tile0 >= n) return;
    const Digit dg = digit_params(pa);
    const uint32_t radix = dg.mask + 1u;
    // thread t owns digits [t*q, t*q + q): issue their global loads first
    const uint32_t q = (radix + kThreads - 1) / kThreads;
    const uint32_t d0 = threadIdx.x * q;
    uint32_t gt[kDigitsPerThread], ho[kDigitsPerThread];
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        const uint32_t d = d0 + j;
        const bool mine = j < (int)q && d < radix;
        gt[j] = mine ? totals[d] : 0u;
        ho[j] = mine ? hist_off[(size_t)d * ntiles + tile] : 0u;
    }
    {  // clear the per-wave counts (as words: no division by the runtime radix)
        uint32_t* wz = wcnt_gbase;
#pragma unroll
        for (int i = 0; i < (kWaves * kCap / 2 + kThreads - 1) / kThreads; ++i)
            if (i * kThreads + (int)threadIdx.x < kWaves * kCap / 2) wz[i * kThreads + threadIdx.x] = 0u;
    }

    const int w = threadIdx.x >> 6;
    const uint32_t base = tile0 + w * (kTileItems / kWaves) + __lane_id();

    uint32_t k_reg[kR], v_reg[kR], rank[kR], p_reg[kPay ? kR : 1];
#pragma unroll
    for (int r = 0; r < kR; ++r) {  // issue every load first
        const uint32_t i = base + r * 64;
        const bool valid = i < n;
        k_reg[r] = valid ? keys_in[i] : 0u;
        v_reg[r] = valid ? (identity_vals ? i : vals_in[i]) : 0u;
        if constexpr (kPay) p_reg[r] = valid ? (rect_in ? pack_rect(rect_in[i]) : pay_in[i]) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kR; ++r) {
        const bool valid = base + r * 64 < n && (!pa.drop || dg.keep(k_reg[r]));
        const uint32_t d = dg.of(k_reg[r]);
        const uint64_t peers = match_digit(d, dg.w, valid);
        uint32_t rk = 0xffffffffu;
        if (valid) {
            const uint32_t old = wcnt[w][d];
            // peers in lower lanes: mbcnt (2 VALU; the lane mask itself was rebuilt per item)
            const uint32_t below =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
            rk = old + below;
            if (below == 0) wcnt[w][d] = (uint16_t)(old + __popcll(peers));
        }
        rank[r] = rk;
    }
    __syncthreads();

    uint32_t t_loc;  // the tile's items kept (all of them unless pa.drop)
    {
        // per owned digit: wave prefixes, then two block scans over digits
        // (tile-local offsets, global digit bases)
        uint32_t tot[kDigitsPerThread];
        uint32_t s_loc = 0, s_glob = 0;
#pragma unroll
        for (int j = 0; j < kDigitsPerThread; ++j) {
            const uint32_t d = d0 + j;
            tot[j] = 0u;
            if (j < (int)q && d < radix) {
                uint32_t run = 0;
#pragma unroll
                for (int k = 0; k < kWaves; ++k) {
                    const uint32_t c = wcnt[k][d];
                    wcnt[k][d] = (uint16_t)run;
                    run += c;
                }
                tot[j] = run;
            }
            s_loc += tot[j];
            s_glob += gt[j];
        }
        uint32_t t_glob;
        uint32_t e_loc = block_exclusive<kThreads>(s_loc, wsum[0], t_loc);
        uint32_t e_glob = block_exclusive<kThreads>(s_glob, wsum[1], t_glob);
#pragma unroll
        for (int j = 0; j < kDigitsPerThread; ++j) {
            const uint32_t d = d0 + j;
            if (j < (int)q && d < radix) {
                dbase[d] = e_loc;
                ho[j] = e_glob + ho[j] - e_loc;  // gbase[d], stored after the staging
            }
            e_loc += tot[j];
            e_glob += gt[j];
        }
    }
    __syncthreads();

#pragma unroll
    for (int r = 0; r < kR; ++r) {
        if (rank[r] != 0xffffffffu) {
            const uint32_t d = dg.of(k_reg[r]);
            const uint32_t p = dbase[d] + wcnt[w][d] + rank[r];
            s_keys[p] = k_reg[r];
            s_vals[p] = v_reg[r];
            if constexpr (kPay) s_pay[p] = p_reg[r];
        }
    }
    __syncthreads();  // (every wcnt read is done: its bytes now take gbase)
#pragma unroll
    for (int j = 0; j < kDigitsPerThread; ++j) {
        const uint32_t d = d0 + j;
        if (j < (int)q && d < radix) gbase[d] = ho[j];
    }
    __syncthreads();

    for (uint32_t j = threadIdx.x; j < t_loc; j += kThreads) {
        const uint32_t key = s_keys[j];
        const uint32_t g = gbase[dg.of(key)] + j;
        if (keys_out) keys_out[g] = key;  // null: a last pass whose keys nobody reads
        vals_out[g] = s_vals[j];
        if constexpr (kPay) pay_out[g] = s_pay[j];
    }
}

template <int kR, bool kPay, int kCB>
__global__ __launch_bounds__(kThreads) void k_rs_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, bool identity_vals,
    uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, const uint32_t* __restrict__ n_dev,
    uint32_t n_host, PassArgs pa, const uint32_t* __restrict__ hist_off, const uint32_t* __restrict__ totals,
    uint32_t ntiles, const uint2* __restrict__ rect_in, const uint32_t* __restrict__ pay_in,
    uint32_t* __restrict__ pay_out) {
    rs_scatter<kR, kPay, kCB>(keys_in, vals_in, identity_vals, keys_out, vals_out, n_dev, n_host, pa, hist_off, totals,
                         ntiles, blockIdx.x, rect_in, pay_in, pay_out);
}

// Batched: the sorts of several views in one launch per step, view =
// blockIdx.y (gsr_render_begin_sorts: the depth sorts of a group of views).
struct SortView {
    const uint32_t* keys_in;
    const uint32_t* vals_in;
    uint32_t* keys_out;
    uint32_t* vals_out;
    const uint32_t* n_dev;
    uint32_t* hist;
    uint32_t* totals;
    PassArgs pa;
    const uint2* rect_in;  // payload (kPay): first pass
    const uint32_t* pay_in;
    uint32_t* pay_out;
};
struct SortViews {
    SortView v[kMaxViews];
};

template <int kR, int kCB>
__global__ __launch_bounds__(kThreads) void k_rs_upsweep_views(SortViews sv, uint32_t n_host, uint32_t ntiles) {
    const SortView& v = sv.v[blockIdx.y];
    rs_upsweep<kR, kCB>(v.keys_in, v.n_dev, n_host, v.pa, v.hist, ntiles, blockIdx.x);
}

__global__ __launch_bounds__(64 * kOffWaves) void k_rs_offsets_views(SortViews sv, uint32_t ntiles) {
    const SortView& v = sv.v[blockIdx.y];
    rs_offsets(v.hist, ntiles, v.pa, v.totals, blockIdx.x * kOffWaves + (threadIdx.x >> 6));
}

template <int kR, bool kPay, int kCB>
__global__ __launch_bounds__(kThreads) void k_rs_scatter_views(SortViews sv, bool identity_vals, uint32_t n_host,
                                                               uint32_t ntiles) {
    const SortView& v = sv.v[blockIdx.y];
    rs_scatter<kR, kPay, kCB>(v.keys_in, v.vals_in, identity_vals, v.keys_out, v.vals_out, v.n_dev, n_host, v.pa, v.hist,
                         v.totals, ntiles, blockIdx.x, v.rect_in, v.pay_in, v.pay_out);
}

}  // namespace

size_t radix_tmp_elems(size_t n) {
    const size_t nb = (n + kMinTileItems - 1) / kMinTileItems;
    return (nb < 1 ? 1 : nb) * kMaxRadix;
}

size_t radix_totals_elems() { return (size_t)kMaxRadix; }  // digit totals scratch (rewritten every pass)

int radix_passes_for(int bits) { return bits <= 0 ? 0 : (bits + kMaxBits - 1) / kMaxBits; }

template <int kR, int kCB>
static int sort_passes(uint32_t** keys_io, uint32_t** vals_io, uint32_t** keys_alt, uint32_t** vals_alt,
                       bool identity_vals, size_t n, const uint32_t* n_dev, int bits, int passes,
                       const uint32_t* key_range, uint32_t* tmp, uint32_t* totals, hipStream_t s,
                       const uint2* rect_in, uint32_t** pay_io, uint32_t** pay_alt, int first_pass,
                       bool drop_first, uint32_t coarse, bool keys_last) {
    constexpr int kTileItems = kThreads * kR;
    const uint32_t nt = (uint32_t)((n + kTileItems - 1) / kTileItems);
    // upper bound of the radix over the passes (device-chosen widths never exceed it)
    const uint32_t radix_max = 1u << ((bits + passes - 1) / passes);
    bool ident = identity_vals;
    // a payload: the packed rects (rect_in, read by the first pass), or pay_io alone (the tile sort carrying
    // the instances' depth keys)
    const bool pay = rect_in != nullptr || pay_io != nullptr;
    for (int p = first_pass; p < passes; ++p) {
        const PassArgs pa{key_range, (uint32_t)bits, (uint32_t)passes, (uint32_t)p,
                          drop_first && p == first_pass ? 1u : 0u, coarse};
        // keys_last false: the last pass writes no keys, so *keys_io keeps its input
        uint32_t* kout = (keys_last || p + 1 < passes) ? *keys_alt : nullptr;
        k_rs_upsweep<kR, kCB><<<nt, kThreads, 0, s>>>(*keys_io, n_dev, (uint32_t)n, pa, tmp, nt);
        GSR_LAUNCH_CHECK("rs_upsweep");
        k_rs_offsets<<<(radix_max + kOffWaves - 1) / kOffWaves, 64 * kOffWaves, 0, s>>>(tmp, nt, pa, totals);
        GSR_LAUNCH_CHECK("rs_offsets");
        if (pay) {
            k_rs_scatter<kR, true, kCB><<<nt, kThreads, 0, s>>>(*keys_io, *vals_io, ident, kout, *vals_alt, n_dev,
                                                           (uint32_t)n, pa, tmp, totals, nt, p == first_pass ? rect_in : nullptr,
                                                           *pay_io, *pay_alt);
        } else {
            k_rs_scatter<kR, false, kCB><<<nt, kThreads, 0, s>>>(*keys_io, *vals_io, ident, kout, *vals_alt, n_dev,
                                                            (uint32_t)n, pa, tmp, totals, nt, nullptr, nullptr,
                                                            nullptr);
        }
        GSR_LAUNCH_CHECK("rs_scatter");
        ident = false;
        uint32_t* t;
        if (kout) {
            t = *keys_io; *keys_io = *keys_alt; *keys_alt = t;
        }
        t = *vals_io; *vals_io = *vals_alt; *vals_alt = t;
        if (pay) {
            t = *pay_io; *pay_io = *pay_alt; *pay_alt = t;
        }
    }
    return GSR_OK;
}

template <int kR, int kCB>
static int sort_passes_views(RadixViewArgs* views, int k, bool identity_vals, size_t n, int bits, int passes,
                             hipStream_t s, int first_pass) {
    constexpr int kTileItems = kThreads * kR;
    const uint32_t nt = (uint32_t)((n + kTileItems - 1) / kTileItems);
    const uint32_t radix_max = 1u << ((bits + passes - 1) / passes);
    bool ident = identity_vals;
    for (int p = first_pass; p < passes; ++p) {
        SortViews sv{};
        for (int v = 0; v < k; ++v) {
            RadixViewArgs& a = views[v];
            sv.v[v] = SortView{*a.keys_io, *a.vals_io, (a.keys_last || p + 1 < passes) ? *a.keys_alt : nullptr,
                               *a.vals_alt, a.n_dev, a.tmp, a.totals,
                               PassArgs{a.key_range, (uint32_t)bits, (uint32_t)passes, (uint32_t)p,
                                        a.drop_first && p == first_pass ? 1u : 0u, a.coarse},
                               p == first_pass ? a.rect_in : nullptr, a.rect_in ? *a.pay_io : nullptr,
                               a.rect_in ? *a.pay_alt : nullptr};
        }
        const bool pay = views[0].rect_in != nullptr;  // all views or none (radix_sort_pairs_views)
        k_rs_upsweep_views<kR, kCB><<<dim3(nt, k), kThreads, 0, s>>>(sv, (uint32_t)n, nt);
        GSR_LAUNCH_CHECK("rs_upsweep_views");
        k_rs_offsets_views<<<dim3((radix_max + kOffWaves - 1) / kOffWaves, k), 64 * kOffWaves, 0, s>>>(sv, nt);
        GSR_LAUNCH_CHECK("rs_offsets_views");
        if (pay)
            k_rs_scatter_views<kR, true, kCB><<<dim3(nt, k), kThreads, 0, s>>>(sv, ident, (uint32_t)n, nt);
        else
            k_rs_scatter_views<kR, false, kCB><<<dim3(nt, k), kThreads, 0, s>>>(sv, ident, (uint32_t)n, nt);
        GSR_LAUNCH_CHECK("rs_scatter_views");
        ident = false;
        for (int v = 0; v < k; ++v) {
            RadixViewArgs& a = views[v];
            uint32_t* t;
            if (a.keys_last || p + 1 < passes) {
                t = *a.keys_io; *a.keys_io = *a.keys_alt; *a.keys_alt = t;
            }
            t = *a.vals_io; *a.vals_io = *a.vals_alt; *a.vals_alt = t;
            if (a.rect_in) {
                t = *a.pay_io; *a.pay_io = *a.pay_alt; *a.pay_alt = t;
            }
        }
    }
    return GSR_OK;
}

int radix_offsets(uint32_t* hist, uint32_t ntiles, int bits, int passes, int pass, uint32_t* totals,
                  hipStream_t s) {
    if (ntiles == 0 || passes == 0) return GSR_OK;
    if (bits < 1 || bits > 32 || passes < 1 || (bits + passes - 1) / passes > kMaxBits)
        return set_error(GSR_ERR_INVALID, "radix offsets: digit width out of range");
    const uint32_t radix_max = 1u << ((bits + passes - 1) / passes);
    const PassArgs pa{nullptr, (uint32_t)bits, (uint32_t)passes, (uint32_t)pass};
    k_rs_offsets<<<(radix_max + kOffWaves - 1) / kOffWaves, 64 * kOffWaves, 0, s>>>(hist, ntiles, pa, totals);
    GSR_LAUNCH_CHECK("rs_offsets");
    return GSR_OK;
}

int radix_offsets_views(uint32_t* const* hist, uint32_t* const* totals, int k, uint32_t ntiles, int bits,
                        int passes, int pass, hipStream_t s) {
    if (ntiles == 0 || passes == 0) return GSR_OK;
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "radix offsets: view count out of range");
    if (bits < 1 || bits > 32 || passes < 1 || (bits + passes - 1) / passes > kMaxBits)
        return set_error(GSR_ERR_INVALID, "radix offsets: digit width out of range");
    const uint32_t radix_max = 1u << ((bits + passes - 1) / passes);
    SortViews sv{};
    for (int v = 0; v < k; ++v) {
        sv.v[v].hist = hist[v];
        sv.v[v].totals = totals[v];
        sv.v[v].pa = PassArgs{nullptr, (uint32_t)bits, (uint32_t)passes, (uint32_t)pass};
    }
    k_rs_offsets_views<<<dim3((radix_max + kOffWaves - 1) / kOffWaves, k), 64 * kOffWaves, 0, s>>>(sv, ntiles);
    GSR_LAUNCH_CHECK("rs_offsets_views");
    return GSR_OK;
}

int radix_sort_pairs_views(RadixViewArgs* views, int k, bool identity_vals, size_t n, int bits, int passes,
                           hipStream_t s, int first_pass) {
    if (n == 0 || passes == 0 || first_pass >= passes) return GSR_OK;
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "radix sort: view count out of range");
    if (n > 0xffffffffull - 4 * kMinTileItems) return set_error(GSR_ERR_OVERFLOW, "radix sort: n too large");
    if (bits < 1 || bits > 32 || passes < 1 || (bits + passes - 1) / passes > kMaxBits)
        return set_error(GSR_ERR_INVALID, "radix sort: digit width out of range");
    for (int v = 1; v < k; ++v)
        if ((views[v].rect_in != nullptr) != (views[0].rect_in != nullptr))
            return set_error(GSR_ERR_INVALID, "radix sort: payload on some views only");
    if ((bits + passes - 1) / passes <= 8) {
        if (views[0].key_range && n > kBigDepthN)
            return sort_passes_views<kRDepthBig, 8>(views, k, identity_vals, n, bits, passes, s, first_pass);
        if (!views[0].key_range && n > kBigTileN)
            return sort_passes_views<kRDepthBig, 8>(views, k, identity_vals, n, bits, passes, s, first_pass);
        return views[0].key_range
                   ? sort_passes_views<kRDepth, 8>(views, k, identity_vals, n, bits, passes, s, first_pass)
                   : sort_passes_views<kRTile, 8>(views, k, identity_vals, n, bits, passes, s, first_pass);
    }
    return sort_passes_views<kRWide, kMaxBits>(views, k, identity_vals, n, bits, passes, s, first_pass);
}

int radix_sort_pairs(uint32_t** keys_io, uint32_t** vals_io, uint32_t** keys_alt, uint32_t** vals_alt,
                     bool identity_vals, size_t n, const uint32_t* n_dev, int bits, int passes,
                     const uint32_t* key_range, uint32_t* tmp, uint32_t* totals, hipStream_t s,
                     const uint2* rect_in, uint32_t** pay_io, uint32_t** pay_alt, int first_pass,
                     bool drop_first, uint32_t coarse, bool keys_last) {
    if (n == 0 || passes == 0 || first_pass >= passes) return GSR_OK;
    if (coarse && !key_range) return set_error(GSR_ERR_INVALID, "radix sort: a coarse order needs the key range");
    if (drop_first && !key_range) return set_error(GSR_ERR_INVALID, "radix sort: dropping needs the key range");
    if (n > 0xffffffffull - 4 * kMinTileItems) return set_error(GSR_ERR_OVERFLOW, "radix sort: n too large");
    if (bits < 1 || bits > 32 || passes < 1 || (bits + passes - 1) / passes > kMaxBits)
        return set_error(GSR_ERR_INVALID, "radix sort: digit width out of range");
    // measured on MI355X: 2048-item tiles for wide digits, for device-chosen
    // widths (the depth sort) and, since round 3's fused binning, for host-known
    // <= 8-bit digits (the tile sort's remaining pass)
    if ((bits + passes - 1) / passes <= 8) {
        if (key_range && n > kBigDepthN)
            return sort_passes<kRDepthBig, 8>(keys_io, vals_io, keys_alt, vals_alt, identity_vals, n, n_dev, bits,
                                              passes, key_range, tmp, totals, s, rect_in, pay_io, pay_alt, first_pass,
                                              drop_first, coarse, keys_last);
        if (key_range)
            return sort_passes<kRDepth, 8>(keys_io, vals_io, keys_alt, vals_alt, identity_vals, n, n_dev, bits, passes,
                                     key_range, tmp, totals, s, rect_in, pay_io, pay_alt, first_pass, drop_first, coarse,
                                     keys_last);
        if (n > kBigTileN)
            return sort_passes<kRDepthBig, 8>(keys_io, vals_io, keys_alt, vals_alt, identity_vals, n, n_dev, bits,
                                              passes, key_range, tmp, totals, s, rect_in, pay_io, pay_alt, first_pass,
                                              drop_first, coarse, keys_last);
        return sort_passes<kRTile, 8>(keys_io, vals_io, keys_alt, vals_alt, identity_vals, n, n_dev, bits, passes,
                                  key_range, tmp, totals, s, rect_in, pay_io, pay_alt, first_pass, drop_first, coarse,
                                     keys_last);
    }
    return sort_passes<kRWide, kMaxBits>(keys_io, vals_io, keys_alt, vals_alt, identity_vals, n, n_dev, bits, passes,
                                         key_range, tmp, totals, s, rect_in, pay_io, pay_alt, first_pass, drop_first, coarse,
                                     keys_last);
}

}  // namespace gsr

// Per-tile depth sort (round 5): every tile's instance list put in the GL draw
// order restricted to the tile, (depth key, slot), in place.
//
// The frame's instances are binned in slot order (no global depth sort) and
// sorted by tile with the stable tile radix sort, so each tile's list leaves
// the tile sort in ascending slot order with its instances' depth keys beside
// it (the binning and the tile sort carry them).  A stable LSD radix sort of
// one list by depth key then gives exactly (key, slot): the order the global
// depth sort + stable binning produced before (renderer_ogl.py:16-26: GL draws
// back to front in _sort_gaussian's order; the compositor walks it front to
// back; ties in slot order, slot n-1-i for Gaussian i, see preprocess.hip).
//
// Why per tile: the work is a tile's own list, kept on chip (one read and one
// write of each instance), no chain of global passes and launches; the digit
// width follows each list's own key range.  The lists' total is D (1.76 M at
// C2) against N for a global sort, but a frame alone spends its time on the
// launch chain, not on ranking (api.hip: what it replaced).
//
// One launch, 1024-thread workgroups, a work list of the tiles by length
// class, longest first (k_chunk_count / k_chunk_write build it with the chunk
// descriptors, composite.hip):
//   * 1025 .. 24576 instances: one workgroup per tile, the list in registers
//     (24 per thread), per pass a stable ranking (ballot digit matching,
//     per-wave digit counts in LDS) and one LDS exchange; the last pass writes
//     the slots coalesced through LDS;
//   * more (the deepest tiles of C3): one workgroup per tile, sub-blocks of
//     12288 ranked as above and written as contiguous digit runs through global
//     scratch (the tile sort's alternate buffers), an even number of passes so
//     the result lands in place;
//   * 2 .. 1024: one wave per tile, 16 items per lane, wave-local ranking and
//     exchange, no workgroup barriers.
// Block b < n_wg takes work-list entry b; the later blocks' 16 waves take the
// wave-class entries in order.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kTdsThreads = 1024;
constexpr int kTdsWaves = kTdsThreads / 64;
constexpr int kTdsItems = kTdsCapBlock / kTdsThreads;  // per thread, workgroup path
static_assert(kTdsItems * kTdsThreads == (int)kTdsCapBlock, "capacity");
constexpr int kTdsLaneItems = kTdsCapWave / 64;         // per lane, wave path
constexpr int kTdsRadix = 256;                          // digits of <= 8 bits

struct TdsWaveLds {
    uint32_t xch[kTdsCapWave];
    uint32_t cnt[kTdsRadix / 2];  // 16-bit digit counts, then digit offsets
};
struct TdsLds {
    union {
        uint32_t xch[kTdsCapBlock];   // workgroup path: one array at a time (keys, then slots)
        TdsWaveLds wave[kTdsWaves];  // wave path
    };
    uint16_t wcnt[kTdsWaves][kTdsRadix];  // per-wave digit counts, then per-wave prefixes
    uint32_t dbase[kTdsRadix];            // sub-block-local digit offsets (or the segment's digit counts)
    uint32_t gbase[kTdsRadix];            // oversized lists: the next global position of each digit
    uint32_t red[2][kTdsWaves];
};

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return ~wave_reduce_max(~v); }

// Digits of one pass over a list's key range [kmin, kmin + 2^B).
struct TdsPass {
    uint32_t kmin, shift, w, mask;
    __device__ __forceinline__ uint32_t of(uint32_t k) const { return ((k - kmin) >> shift) & mask; }
};

// Passes of <= 8 bits for a B-bit range (even: the oversized path ends in place).
__device__ __forceinline__ uint32_t tds_passes(uint32_t B, bool even) {
    uint32_t p = (B + 7u) / 8u;
    if (even && (p & 1u)) ++p;
    return p;
}

// ---------------------------------------------------------------- wave path
// One wave sorts the list [b, b + L), 2 <= L <= kTdsCapWave.
__device__ void tds_wave(const uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t b, uint32_t L,
                         TdsWaveLds& W, uint32_t dbg) {
    const uint32_t lane = __lane_id();
    const uint32_t nr = (L + 63u) / 64u;
    uint32_t k[kTdsLaneItems], v[kTdsLaneItems], rank[kTdsLaneItems];
    uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
    for (int j = 0; j < kTdsLaneItems; ++j) {
        k[j] = 0u;
        v[j] = 0u;
        if ((uint32_t)j < nr) {
            const uint32_t i = (uint32_t)j * 64u + lane;
            if (i < L) {
                k[j] = keys[b + i];
                v[j] = vals[b + i];
                lo = min(lo, k[j]);
                hi = max(hi, k[j]);
            }
        }
    }
    const uint32_t kmin = wave_min(lo), kmax = wave_reduce_max(hi);
    if (kmax == kmin) return;  // equal keys: the slot order is the order
    const uint32_t B = 32u - (uint32_t)__clz(kmax - kmin);
    uint32_t P = tds_passes(B, false);
    TdsPass dg;
    dg.kmin = kmin;
    dg.w = (B + P - 1u) / P;
    if (dbg & 4u) P = 1u;  // (timing knob: the first digit only, <= 8 bits)
    dg.mask = (1u << dg.w) - 1u;
    uint16_t* c16 = reinterpret_cast<uint16_t*>(W.cnt);
    for (uint32_t p = 0; p < P; ++p) {
        dg.shift = p * dg.w;
        W.cnt[lane] = 0u;
        W.cnt[lane + 64] = 0u;
        __builtin_amdgcn_wave_barrier();
        // stable ranks: rounds in item order, lanes in order within a round
#pragma unroll
        for (int j = 0; j < kTdsLaneItems; ++j) {
            if ((uint32_t)j < nr) {  // (no `break`: it stops the unrolling, and the arrays go to scratch)
                const bool ok = (uint32_t)j * 64u + lane < L;
                const uint32_t d = dg.of(k[j]);
                const uint64_t peers = match_digit(d, dg.w, ok);
                const uint32_t below = mbcnt64(peers);
                const uint32_t old = c16[d];
                rank[j] = old + below;
                if (ok && below == 0u) c16[d] = (uint16_t)(old + (uint32_t)__popcll(peers));
                __builtin_amdgcn_wave_barrier();
            }
        }
        // digit offsets: lane l owns digits 4l .. 4l + 3
        {
            const uint32_t w0 = W.cnt[2 * lane], w1 = W.cnt[2 * lane + 1];
            const uint32_t c0 = w0 & 0xffffu, c1 = w0 >> 16, c2 = w1 & 0xffffu, c3 = w1 >> 16;
            const uint32_t s = c0 + c1 + c2 + c3;
            const uint32_t e = wave_inclusive_scan(s) - s;
            __builtin_amdgcn_wave_barrier();
            W.cnt[2 * lane] = e | (e + c0) << 16;
            W.cnt[2 * lane + 1] = (e + c0 + c1) | (e + c0 + c1 + c2) << 16;
            __builtin_amdgcn_wave_barrier();
        }
        const bool last = p + 1u == P;
        // keys, then slots, through the exchange in their new order
#pragma unroll
        for (int j = 0; j < kTdsLaneItems; ++j) {
            if ((uint32_t)j < nr) {
                rank[j] += c16[dg.of(k[j])];  // the new position
                if (!last && (uint32_t)j * 64u + lane < L) W.xch[rank[j]] = k[j];
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (!last) {
#pragma unroll
            for (int j = 0; j < kTdsLaneItems; ++j)
                if ((uint32_t)j < nr) k[j] = W.xch[(uint32_t)j * 64u + lane];
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int j = 0; j < kTdsLaneItems; ++j)
            if ((uint32_t)j < nr && (uint32_t)j * 64u + lane < L) W.xch[rank[j]] = v[j];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kTdsLaneItems; ++j) {
            const uint32_t i = (uint32_t)j * 64u + lane;
            if ((uint32_t)j < nr) {
                v[j] = W.xch[i];
                if (last && i < L) vals[b + i] = v[j];
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------- workgroup path
// Block-wide min and max (every thread gets them).
__device__ __forceinline__ void block_minmax(uint32_t& lo, uint32_t& hi, TdsLds& S) {
    lo = wave_min(lo);
    hi = wave_reduce_max(hi);
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        S.red[0][w] = lo;
        S.red[1][w] = hi;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kTdsWaves; ++q) {
        lo = min(lo, S.red[0][q]);
        hi = max(hi, S.red[1][q]);
    }
    __syncthreads();  // (red is reused)
}

// One sub-block of at most kTdsCapBlock items, [0, Lc) in item order, in
// registers: item j*64 + lane of wave w's span.  Ranks each item stably by
// digit; leaves in rank[j] its position within the sub-block, in S.dbase the
// sub-block's digit offsets and in `tot` (threads 0..255: digit t) its digit
// counts.  The per-wave digit counts become each wave's first position of the
// digit in place, so an item's position is its rank plus one LDS read.
template <int kI>
__device__ __forceinline__ void tds_rank_block(const uint32_t (&k)[kI], uint32_t (&rank)[kI], uint32_t span,
                                               uint32_t Lc, const TdsPass& dg, TdsLds& S, uint32_t& tot) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    const uint32_t nr = span / 64u;
    {
        uint32_t* wz = reinterpret_cast<uint32_t*>(&S.wcnt[0][0]);
        wz[t] = 0u;
        wz[t + kTdsThreads] = 0u;
        static_assert(kTdsWaves * kTdsRadix / 2 == 2 * kTdsThreads, "wcnt clearing");
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        if ((uint32_t)j < nr) {
            const bool ok = w * span + (uint32_t)j * 64u + lane < Lc;
            const uint32_t d = dg.of(k[j]);
            const uint64_t peers = match_digit(d, dg.w, ok);
            const uint32_t below = mbcnt64(peers);
            const uint32_t old = S.wcnt[w][d];
            rank[j] = old + below;
            if (ok && below == 0u) S.wcnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    // thread t < 256 owns digit t: per-wave prefixes, its total, the block scan of the totals
    tot = 0u;
    if (t < (uint32_t)kTdsRadix) {
#pragma unroll
        for (int q = 0; q < kTdsWaves; ++q) {
            const uint32_t c = S.wcnt[q][t];
            S.wcnt[q][t] = (uint16_t)tot;
            tot += c;
        }
    }
    const uint32_t inc = wave_inclusive_scan(tot);
    if (lane == 63 && w < (uint32_t)(kTdsRadix / 64)) S.red[0][w] = inc;
    __syncthreads();
    if (t < (uint32_t)kTdsRadix) {
        uint32_t e = inc - tot;
        for (uint32_t q = 0; q < w; ++q) e += S.red[0][q];
        S.dbase[t] = e;
        // each wave's first position of digit t (< kTdsCapBlock: 16 bits), so an item's position is one read
#pragma unroll
        for (int q = 0; q < kTdsWaves; ++q) S.wcnt[q][t] = (uint16_t)(S.wcnt[q][t] + e);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kI; ++j) {
        if ((uint32_t)j < nr) rank[j] += S.wcnt[w][dg.of(k[j])];
    }
}

// One workgroup sorts [b, b + L), kTdsCapWave < L <= kTdsCapBlock, in registers.
__device__ void tds_block(const uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t b, uint32_t L,
                          TdsLds& S, uint32_t dbg) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    // wave w's span: items [w * span, (w + 1) * span), rounds of 64
    const uint32_t span = (L + kTdsThreads - 1u) / kTdsThreads * 64u;
    const uint32_t nr = span / 64u;
    uint32_t k[kTdsItems], v[kTdsItems], rank[kTdsItems];
    uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
    for (int j = 0; j < kTdsItems; ++j) {
        k[j] = 0u;
        v[j] = 0u;
        if ((uint32_t)j < nr) {
            const uint32_t i = w * span + (uint32_t)j * 64u + lane;
            if (i < L) {
                k[j] = keys[b + i];
                v[j] = vals[b + i];
                lo = min(lo, k[j]);
                hi = max(hi, k[j]);
            }
        }
    }
    block_minmax(lo, hi, S);
    if (hi == lo) return;
    const uint32_t B = 32u - (uint32_t)__clz(hi - lo);
    uint32_t P = tds_passes(B, false);
    TdsPass dg;
    dg.kmin = lo;
    dg.w = (B + P - 1u) / P;
    if (dbg & 4u) P = 1u;  // (timing knob: the first digit only, <= 8 bits)
    dg.mask = (1u << dg.w) - 1u;
    for (uint32_t p = 0; p < P; ++p) {
        dg.shift = p * dg.w;
        uint32_t tot;
        tds_rank_block<kTdsItems>(k, rank, span, L, dg, S, tot);
        const bool last = p + 1u == P;
        if (!last) {
#pragma unroll
            for (int j = 0; j < kTdsItems; ++j)
                if ((uint32_t)j < nr && w * span + (uint32_t)j * 64u + lane < L) S.xch[rank[j]] = k[j];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kTdsItems; ++j)
                if ((uint32_t)j < nr) k[j] = S.xch[w * span + (uint32_t)j * 64u + lane];
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < kTdsItems; ++j)
            if ((uint32_t)j < nr && w * span + (uint32_t)j * 64u + lane < L) S.xch[rank[j]] = v[j];
        __syncthreads();
        if (last) {  // the sorted slots, coalesced
            for (uint32_t i = t; i < L; i += kTdsThreads) vals[b + i] = S.xch[i];
        } else {
#pragma unroll
            for (int j = 0; j < kTdsItems; ++j)
                if ((uint32_t)j < nr) v[j] = S.xch[w * span + (uint32_t)j * 64u + lane];
            __syncthreads();
        }
    }
}

// One workgroup sorts [b, b + L), L > kTdsCapBlock: an even number of LSD
// passes between (keys, vals) and the scratch (keys_alt, vals_alt), each pass a
// digit histogram of the whole list, then its sub-blocks of kTdsSub in order,
// each ranked in registers, restaged in LDS in digit order (keys and slots side
// by side) and written as contiguous digit runs.
constexpr uint32_t kTdsSub = kTdsCapBlock / 2;
constexpr int kTdsSubItems = (int)kTdsSub / kTdsThreads;

__device__ void tds_global(uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ keys_alt,
                           uint32_t* __restrict__ vals_alt, uint32_t b, uint32_t L, TdsLds& S) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (uint32_t i = t; i < L; i += kTdsThreads) {
        const uint32_t kk = keys[b + i];
        lo = min(lo, kk);
        hi = max(hi, kk);
    }
    block_minmax(lo, hi, S);
    if (hi == lo) return;
    const uint32_t B = 32u - (uint32_t)__clz(hi - lo);
    const uint32_t P = tds_passes(B, true);
    TdsPass dg;
    dg.kmin = lo;
    dg.w = (B + P - 1u) / P;
    dg.mask = (1u << dg.w) - 1u;
    uint32_t *ks = keys + b, *vs = vals + b, *kd = keys_alt + b, *vd = vals_alt + b;
    uint32_t* xk = S.xch;
    uint32_t* xv = S.xch + kTdsSub;
    for (uint32_t p = 0; p < P; ++p) {
        dg.shift = p * dg.w;
        const bool last = p + 1u == P;
        // the list's digit counts -> the digits' first global positions
        if (t < (uint32_t)kTdsRadix) S.dbase[t] = 0u;
        __syncthreads();
        for (uint32_t i = t; i < L; i += kTdsThreads) atomicAdd(&S.dbase[dg.of(ks[i])], 1u);
        __syncthreads();
        {
            const uint32_t c = t < (uint32_t)kTdsRadix ? S.dbase[t] : 0u;
            const uint32_t inc = wave_inclusive_scan(c);
            if (lane == 63 && w < (uint32_t)(kTdsRadix / 64)) S.red[1][w] = inc;
            __syncthreads();
            if (t < (uint32_t)kTdsRadix) {
                uint32_t e = inc - c;
                for (uint32_t q = 0; q < w; ++q) e += S.red[1][q];
                S.gbase[t] = e;
            }
        }
        for (uint32_t c0 = 0; c0 < L; c0 += kTdsSub) {
            const uint32_t Lc = min(kTdsSub, L - c0);
            const uint32_t span = (Lc + kTdsThreads - 1u) / kTdsThreads * 64u;
            const uint32_t nr = span / 64u;
            uint32_t k[kTdsSubItems], v[kTdsSubItems], rank[kTdsSubItems];
#pragma unroll
            for (int j = 0; j < kTdsSubItems; ++j) {
                const uint32_t i = w * span + (uint32_t)j * 64u + lane;
                const bool ok = (uint32_t)j < nr && i < Lc;
                k[j] = ok ? ks[c0 + i] : 0u;
                v[j] = ok ? vs[c0 + i] : 0u;
            }
            uint32_t tot;
            tds_rank_block<kTdsSubItems>(k, rank, span, Lc, dg, S, tot);  // (its first barrier orders gbase's writes)
#pragma unroll
            for (int j = 0; j < kTdsSubItems; ++j)
                if ((uint32_t)j < nr && w * span + (uint32_t)j * 64u + lane < Lc) {
                    xk[rank[j]] = k[j];
                    xv[rank[j]] = v[j];
                }
            __syncthreads();
            // out as contiguous digit runs
            for (uint32_t i = t; i < Lc; i += kTdsThreads) {
                const uint32_t kk = xk[i];
                const uint32_t d = dg.of(kk);
                const uint32_t g = S.gbase[d] + (i - S.dbase[d]);
                if (!last) kd[g] = kk;
                vd[g] = xv[i];
            }
            __syncthreads();
            if (t < (uint32_t)kTdsRadix) S.gbase[t] += tot;  // the next sub-block continues each run
        }
        uint32_t* x;
        x = ks; ks = kd; kd = x;
        x = vs; vs = vd; vd = x;
        __syncthreads();
    }
}

struct TdsView {
    const uint2* ranges;
    const uint32_t* list;    // tiles by length class (chunk_write)
    const uint32_t* counts;  // {workgroup-class tiles, wave-class tiles}
    uint32_t* keys;          // the instances' depth keys (tile sort payload); the oversized path permutes them
    uint32_t* vals;          // the tile list (slots), sorted in place
    uint32_t* keys_alt;      // scratch for the oversized path (n_dup words each)
    uint32_t* vals_alt;
};
struct TdsViews {
    TdsView v[kMaxViews];
};

// Persistent: a grid of at most one workgroup per CU (the LDS allows one)
// walks the work units in order, unit u < n_wg a workgroup-class list, the
// later units 16 wave-class lists each.  (A grid sized for the host's upper
// bound of the workgroup-class lists, ~1700 blocks at C2 that mostly exit at
// once, cost ~30 us of workgroup churn: profiles/r5_s6.)
__global__ __launch_bounds__(kTdsThreads) void k_tile_depth_sort(TdsViews vs, uint32_t dbg) {
    __shared__ TdsLds S;
    const TdsView& V = vs.v[blockIdx.y];
    const uint32_t n_wg = V.counts[0], n_wave = V.counts[1];
    const uint32_t units = n_wg + (n_wave + kTdsWaves - 1) / kTdsWaves;
    const uint32_t w = threadIdx.x >> 6;
    for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {  // (u is uniform: every barrier is reached)
        if (u < n_wg) {
            if (!(dbg & 1u)) {
                const uint2 r = V.ranges[V.list[u]];
                const uint32_t L = r.y - r.x;
                if (L > kTdsCapBlock)
                    tds_global(V.keys, V.vals, V.keys_alt, V.vals_alt, r.x, L, S);
                else
                    tds_block(V.keys, V.vals, r.x, L, S, dbg);
            }
        } else {
            const uint32_t j = (u - n_wg) * kTdsWaves + w;
            if (j < n_wave && !(dbg & 2u)) {
                const uint2 r = V.ranges[V.list[n_wg + j]];
                tds_wave(V.keys, V.vals, r.x, r.y - r.x, S.wave[w], dbg);
            }
        }
        __syncthreads();  // (the next unit reuses the LDS)
    }
}

}  // namespace

int launch_tile_depth_sort(const TileSortView* views, int k, int num_tiles, hipStream_t s, uint32_t debug) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "tile depth sort: view count out of range");
    TdsViews tv{};
    uint32_t wg_max = 0;
    for (int i = 0; i < k; ++i) {
        const TileSortView& a = views[i];
        tv.v[i] = TdsView{a.ranges, a.list, a.counts, a.keys, a.vals, a.keys_alt, a.vals_alt};
        // an upper bound of the workgroup-class tiles: each holds more than kTdsCapWave instances
        wg_max = std::max(wg_max, std::min((uint32_t)num_tiles, a.n_dup / (kTdsCapWave + 1u)));
    }
    // at most the work units, and one block per CU per view (a block takes one CU: its LDS)
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    }
    const uint32_t units = wg_max + (uint32_t)(num_tiles + kTdsWaves - 1) / kTdsWaves;
    const uint32_t grid = std::min(units, (uint32_t)cus);
    if (units == 0) return GSR_OK;
    k_tile_depth_sort<<<dim3(grid, (unsigned)k), kTdsThreads, 0, s>>>(tv, debug);
    GSR_LAUNCH_CHECK("tile_depth_sort");
    return GSR_OK;
}

}  // namespace gsr

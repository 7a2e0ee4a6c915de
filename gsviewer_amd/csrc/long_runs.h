// The coarse depth order's long runs (round 5): the stretches of one tile's
// list whose instances share the coarse depth key and that are too long for
// k_tile_ranges' in-thread repair (RunFix, composite.hip), put in the GL draw
// order restricted to the tile, (full depth key, slot), in place.
//
// The frame alone sorts depth by the top bits of its key range only (two
// 8-bit passes, api.hip depth_sort); the binning and the tile sort are stable
// and carry each instance's full key, so every tile's list leaves them in runs
// of equal coarse key, ascending, each run in slot order.  A stable sort of a
// run by full key gives exactly (key, slot): the order an exact depth sort and
// the stable binning produce (renderer_ogl.py:16-26: GL draws back to front in
// _sort_gaussian's order; the compositor walks it front to back; ties in slot
// order, slot n-1-i for Gaussian i, see preprocess.hip).  Runs of up to
// kFixRunMax are repaired in k_tile_ranges; the longer ones, listed there, are
// rare in a scene of spread depths (none at C2) and unbounded in a degenerate
// one (a fronto-parallel plane: a deep tile's whole list is one run), so they
// get on-chip sorts of bounded cost, not round 4's single-thread O(L^2).
//
// Per-run or per-tile sorting as the DEFAULT order was measured and dropped:
// it is latency-bound (one wave ~5 us per run, a workgroup 20-25 us,
// profiles/r5_s13); here it only covers what the coarse order leaves.
//
// Device code only, included by composite.hip: the runs are sorted by extra
// blocks of the chunk-count launch (k_chunk_count_long), or by a launch of
// their own (k_long_runs) where no chunks are built (the RGBA8 framebuffer).
// A fixed set of G 1024-thread blocks; block b takes the listed runs
// b, b + G, ...:
//   * each wave finds one run's end (a 64-way search between its start and
//     its tile's end: tile key and coarse key are nondecreasing along the
//     list, so "still in the run" is a prefix) and, up to 1024 instances,
//     sorts it (16 items per lane, wave-local ranking by ballot digit
//     matching and an LDS exchange, no workgroup barriers);
//   * then the block sorts its longer runs one at a time: up to 24576 in
//     registers (24 per thread), per pass a stable ranking with per-wave digit
//     counts in LDS and one LDS exchange, the last pass writing the slots
//     coalesced; longer ones through global scratch (the tile sort's
//     alternate buffers), an even number of passes so the result lands in place.
// Concurrent blocks read other runs only while searching: the tile keys are
// never written and a run's permutation keeps its coarse key, so the search's
// answer does not depend on it.

#pragma once
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr uint32_t kTdsCapWave = 1024;    // runs sorted by one wave (16 items per lane)
constexpr uint32_t kTdsCapBlock = 24576;  // runs sorted by one workgroup in registers (24 per thread)
constexpr int kTdsThreads = 1024;
constexpr int kLongGrid = 256;  // blocks of the long-run launch (one per CU: 108 KB of LDS each)
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
__device__ __forceinline__ void tds_wave(const uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t b, uint32_t L,
                         TdsWaveLds& W) {
    const uint32_t lane = __lane_id();
    const uint32_t nr = (L + 63u) / 64u;
    uint32_t k[kTdsLaneItems], v[kTdsLaneItems], rank[kTdsLaneItems];
    // every load issued before any is used (a use right after each guarded load
    // waited for it: 16 serial round trips per run, profiles/r5_s11)
#pragma unroll
    for (int j = 0; j < kTdsLaneItems; ++j) {
        const uint32_t i = (uint32_t)j * 64u + lane;
        const bool ok = (uint32_t)j < nr && i < L;
        k[j] = ok ? keys[b + i] : 0xffffffffu;
        v[j] = ok ? vals[b + i] : 0u;
    }
    uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
    for (int j = 0; j < kTdsLaneItems; ++j) {
        const bool ok = (uint32_t)j < nr && (uint32_t)j * 64u + lane < L;
        lo = min(lo, k[j]);
        hi = ok ? max(hi, k[j]) : hi;
    }
    const uint32_t kmin = wave_min(lo), kmax = wave_reduce_max(hi);
    if (kmax == kmin) return;  // equal keys: the slot order is the order
    const uint32_t B = 32u - (uint32_t)__clz(kmax - kmin);
    const uint32_t P = tds_passes(B, false);
    TdsPass dg;
    dg.kmin = kmin;
    dg.w = (B + P - 1u) / P;
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
__device__ __forceinline__ void tds_block(const uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t b, uint32_t L,
                          TdsLds& S) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    // wave w's span: items [w * span, (w + 1) * span), rounds of 64
    const uint32_t span = (L + kTdsThreads - 1u) / kTdsThreads * 64u;
    const uint32_t nr = span / 64u;
    uint32_t k[kTdsItems], v[kTdsItems], rank[kTdsItems];
#pragma unroll
    for (int j = 0; j < kTdsItems; ++j) {  // (every load issued before any is used)
        const uint32_t i = w * span + (uint32_t)j * 64u + lane;
        const bool ok = (uint32_t)j < nr && i < L;
        k[j] = ok ? keys[b + i] : 0xffffffffu;
        v[j] = ok ? vals[b + i] : 0u;
    }
    uint32_t lo = 0xffffffffu, hi = 0u;
#pragma unroll
    for (int j = 0; j < kTdsItems; ++j) {
        const bool ok = (uint32_t)j < nr && w * span + (uint32_t)j * 64u + lane < L;
        lo = min(lo, k[j]);
        hi = ok ? max(hi, k[j]) : hi;
    }
    block_minmax(lo, hi, S);
    if (hi == lo) return;
    const uint32_t B = 32u - (uint32_t)__clz(hi - lo);
    const uint32_t P = tds_passes(B, false);
    TdsPass dg;
    dg.kmin = lo;
    dg.w = (B + P - 1u) / P;
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
constexpr int kSweep = 8;  // loads in flight per thread in the global path's sweeps
constexpr int kTdsSubItems = (int)kTdsSub / kTdsThreads;

__device__ __forceinline__ void tds_global(uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ keys_alt,
                           uint32_t* __restrict__ vals_alt, uint32_t b, uint32_t L, TdsLds& S) {
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    uint32_t lo = 0xffffffffu, hi = 0u;
    for (uint32_t i0 = 0; i0 < L; i0 += kSweep * kTdsThreads) {  // kSweep loads in flight per thread
        uint32_t kk[kSweep];
#pragma unroll
        for (int j = 0; j < kSweep; ++j) {
            const uint32_t i = i0 + (uint32_t)j * kTdsThreads + t;
            kk[j] = i < L ? keys[b + i] : 0xffffffffu;
        }
#pragma unroll
        for (int j = 0; j < kSweep; ++j) {
            lo = min(lo, kk[j]);
            hi = i0 + (uint32_t)j * kTdsThreads + t < L ? max(hi, kk[j]) : hi;
        }
    }
    block_minmax(lo, hi, S);
    if (hi == lo) return;
    const uint32_t B = 32u - (uint32_t)__clz(hi - lo);
    const uint32_t P = tds_passes(B, true);
    // The result lands in (keys, vals) only after an even number of passes
    // (each pass swaps source and scratch); an odd count would leave the
    // sorted run in the scratch and the list half permuted.  Trap rather than
    // composite such a list (the sorters' invariants checked
    // on the device; uniform, one scalar test per long run).
    if (P & 1u) __builtin_trap();
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
        for (uint32_t i0 = 0; i0 < L; i0 += kSweep * kTdsThreads) {
            uint32_t kk[kSweep];
#pragma unroll
            for (int j = 0; j < kSweep; ++j) {
                const uint32_t i = i0 + (uint32_t)j * kTdsThreads + t;
                kk[j] = i < L ? ks[i] : 0u;
            }
#pragma unroll
            for (int j = 0; j < kSweep; ++j)
                if (i0 + (uint32_t)j * kTdsThreads + t < L) atomicAdd(&S.dbase[dg.of(kk[j])], 1u);
        }
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

struct LongRunArgs {
    const uint32_t* tile_keys;  // the sorted tile keys (never written)
    const uint2* ranges;        // each tile's [begin, end) in the list
    uint32_t* inst_keys;        // each position's full depth key (the global path permutes them with the slots)
    uint32_t* vals;             // the tile lists (slots), sorted in place
    uint32_t* keys_alt;         // scratch for the global path (n words each)
    uint32_t* vals_alt;
    const uint32_t* key_range;  // the frame's {~kmin, kmax}
    uint32_t coarse;
    const uint32_t* starts;     // the runs' first positions (k_tile_ranges), *count of them
    const uint32_t* count;
    uint32_t* lens;             // each run's length, for the block pass
};

// The end of the run starting at b (tile `tile`, coarse key cv), at most hi:
// 64 probes a round, the first failing one narrows the bracket 64-fold.
__device__ __forceinline__ uint32_t run_end(const LongRunArgs& a, uint32_t b, uint32_t hi, uint32_t tile, uint32_t cv, uint32_t kmin,
                            uint32_t s0) {
    const uint32_t lane = __lane_id();
    uint32_t lo = b, up = hi;  // p(lo) holds; every position >= up fails (or is past the tile)
    while (up - lo > 1u) {
        const uint32_t step = (up - lo + 63u) / 64u;
        const uint32_t pos = lo + (lane + 1u) * step;
        bool in = false;
        if (pos < up) {
            const uint32_t tk = a.tile_keys[pos], f = a.inst_keys[pos];
            in = tk == tile && ((f - kmin) >> s0) == cv;
        }
        const uint32_t c = (uint32_t)__popcll(__ballot(in));  // a prefix of the lanes
        up = min(up, lo + (c + 1u) * step);
        lo += c * step;
    }
    return up;
}

// The runs of block `bid` of G (S: the block's LDS; every thread of the block calls it).
__device__ __forceinline__ void long_runs_block(const LongRunArgs& a, TdsLds& S, uint32_t bid, uint32_t G) {
    const uint32_t n_long = *a.count;
    if (bid >= n_long) return;
    const uint32_t w = threadIdx.x >> 6, lane = __lane_id();
    uint32_t kmin;
    const uint32_t s0 = coarse_shift(a.key_range, a.coarse, kmin);  // > 0: a long run was listed
    const uint32_t mine = (n_long - bid + G - 1u) / G;  // this block's runs: bid + j G, j < mine
    // 1. one wave per run: its end, and the sort of a run of <= kTdsCapWave
    for (uint32_t j = w; j < mine; j += kTdsWaves) {
        const uint32_t r = bid + j * G;
        const uint32_t b = a.starts[r];
        const uint32_t tile = a.tile_keys[b];
        const uint32_t cv = (a.inst_keys[b] - kmin) >> s0;
        const uint32_t L = run_end(a, b, a.ranges[tile].y, tile, cv, kmin, s0) - b;
        // (a listed run lies in its tile's list: b < run end <= the tile's end, so every sorter below reads and
        // writes [b, b + L) of the list and its scratch only)
        if (L <= kTdsCapWave) tds_wave(a.inst_keys, a.vals, b, L, S.wave[w]);
        if (lane == 0) a.lens[r] = L;
    }
    __syncthreads();  // (the lengths are this block's own writes)
    // 2. the whole block per longer run
    for (uint32_t j = 0; j < mine; ++j) {
        const uint32_t r = bid + j * G;
        const uint32_t L = a.lens[r];
        if (L <= kTdsCapWave) continue;
        const uint32_t b = a.starts[r];
        if (L > kTdsCapBlock)
            tds_global(a.inst_keys, a.vals, a.keys_alt, a.vals_alt, b, L, S);
        else
            tds_block(a.inst_keys, a.vals, b, L, S);
        __syncthreads();  // (the next run reuses the LDS)
    }
}

__global__ __launch_bounds__(kTdsThreads) void k_long_runs(LongRunArgs a) {
    __shared__ TdsLds S;
    long_runs_block(a, S, blockIdx.x, gridDim.x);
}

// The launch arguments of the runs of a frame (null-checked).
inline int long_run_args(const uint32_t* tile_keys, uint32_t n_dup, const uint2* ranges, const RunFix& fix,
                         LongRunArgs& a) {
    if (!tile_keys || !ranges || !fix.inst_keys || !fix.vals || !fix.scratch_keys || !fix.scratch_vals ||
        !fix.long_starts || !fix.long_count || !fix.key_range)
        return set_error(GSR_ERR_INVALID, "long runs: null buffer");
    a = LongRunArgs{tile_keys, ranges, fix.inst_keys, fix.vals, fix.scratch_keys, fix.scratch_vals,
                    fix.key_range, fix.coarse, fix.long_starts, fix.long_count,
                    fix.long_starts + long_run_cap(n_dup)};
    return GSR_OK;
}

}  // namespace
}  // namespace gsr

// Per-tile depth sort (round 5): every tile's instance list put in the GL draw
// order restricted to the tile, (depth key, slot), in place.
//
// The frame's instances are binned in slot order (no global depth sort) under
// the key (tile << cb) | bucket, the bucket the top cb bits of the splat's
// depth key in the frame's key range (InstKey, composite.hip), and sorted by
// that key with the stable tile radix sort: each tile's list leaves it in
// runs of equal bucket, buckets ascending, each run in ascending slot order,
// with its instances' depth keys beside it (the binning and the tile sort
// carry them).  A stable LSD radix sort of every run by depth key then gives
// exactly (key, slot): the order the global depth sort + stable binning
// produced (renderer_ogl.py:16-26: GL draws back to front in _sort_gaussian's
// order; the compositor walks it front to back; ties in slot order, slot
// n-1-i for Gaussian i, see preprocess.hip).  The cb bits cost no tile-sort
// pass: the passes are fixed by the tile id's width and their 8-bit digits
// have room for them (api.hip TileBits: 3 bits at 1080p, 1 at 4K; 11-bit
// digits for 9 bits cost the binning and the tile sort 105 us, profiles/r5_s9).
//
// Why runs: a deep tile (22 K instances at C2) sorted by one workgroup keeps
// one CU busy for ~40 us (the ranking is VALU issue: ~50 instructions per
// instance and pass at 4 cycles each, profiles/r5_s8), while the depth
// buckets cut it into runs (at C2 the longest 9.4 K) that spread over the
// chip, and the runs' narrower key ranges take fewer passes.  Why no global sort:
// the work is each run's own instances, kept on chip (one read and one
// write each), one launch instead of a chain of global passes.
//
// One launch, one 1024-thread block per kTdsSpan instances:
//   * runs of more than 1024 instances (k_tile_ranges lists them; a few
//     hundred at C2) are dealt to the blocks in turn, each sorted by one whole
//     block: up to 24576 the run in registers (24 per thread), per
//     pass a stable ranking (ballot digit matching, per-wave digit counts in
//     LDS) and one LDS exchange; the last pass writes the slots coalesced
//     through LDS;
//   * longer (a run that fills a deep tile: a depth range too narrow for the
//     frame's buckets, the deepest tiles of C3): the whole block, sub-blocks
//     of 12288 ranked as above and written as contiguous digit runs through
//     global scratch (the tile sort's alternate buffers), an even number of
//     passes so the result lands in place;
//   * then each block finds the runs that start in its span (the last one may
//     end past it) and sorts those of 2 .. 1024 instances, one wave per run,
//     16 items per lane, wave-local ranking and exchange, no workgroup
//     barriers.
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
constexpr int kSweep = 8;  // loads in flight per thread in the global path's sweeps
constexpr int kTdsSubItems = (int)kTdsSub / kTdsThreads;

__device__ void tds_global(uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t* __restrict__ keys_alt,
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

struct TdsView {
    const uint32_t* tkeys;  // the tile sort's keys: a run is a stretch of equal ones
    uint32_t* keys;         // the instances' depth keys; the global path permutes them
    uint32_t* vals;         // the tile lists (slots), sorted in place
    uint32_t* keys_alt;     // scratch for the global path (n words each)
    uint32_t* vals_alt;
    uint32_t n;
    const uint2* big_runs;  // the runs of > kTdsCapWave (k_tile_ranges)
    const uint32_t* big_count;
};
struct TdsViews {
    TdsView v[kMaxViews];
    uint64_t* stamps;  // (timing knob GSR_DEBUG_TDS & 8: per block 4 clock stamps + 4 counts; else null)
};

constexpr int kSpanItems = (int)kTdsSpan / kTdsThreads;  // instances per thread when finding the runs

// Runs of a span, outside the sort's LDS (TdsLds): their starts (offsets from
// the span's first instance) and the last one's end.
struct TdsRunLds {
    uint16_t start[kTdsSpan];
    uint32_t n_runs, last_end;
    uint32_t scan[kTdsWaves];
};

__global__ __launch_bounds__(kTdsThreads) void k_tile_depth_sort(TdsViews vs, uint32_t dbg) {
    __shared__ TdsLds S;
    __shared__ TdsRunLds R;
    const TdsView& V = vs.v[blockIdx.y];
    if (blockIdx.x * kTdsSpan >= V.n) return;  // (a view smaller than the grid's largest)
    const uint32_t t = threadIdx.x, w = t >> 6, lane = __lane_id();
    uint64_t* st = vs.stamps && blockIdx.y == 0 ? vs.stamps + 8 * (size_t)blockIdx.x : nullptr;
    if (st && t == 0) st[0] = __builtin_amdgcn_s_memrealtime();
    // A. the long runs, one workgroup each, dealt to the view's blocks in turn
    const uint32_t n_big = *V.big_count;
    const uint32_t blocks = (V.n + kTdsSpan - 1) / kTdsSpan;
    uint32_t big_done = 0, big_items = 0;
    for (uint32_t i = blockIdx.x; i < n_big; i += blocks) {
        const uint2 br = V.big_runs[i];
        ++big_done;
        big_items += br.y;
        if (!(dbg & 1u)) {
            if (br.y > kTdsCapBlock)
                tds_global(V.keys, V.vals, V.keys_alt, V.vals_alt, br.x, br.y, S);
            else
                tds_block(V.keys, V.vals, br.x, br.y, S, dbg);
        }
        __syncthreads();  // (the next run reuses the LDS)
    }
    if (st && t == 0) st[1] = __builtin_amdgcn_s_memrealtime();
    // B. the runs of 2 .. kTdsCapWave that start in this block's span, one wave each
    const uint32_t p0 = blockIdx.x * kTdsSpan;
    const uint32_t p1 = min(p0 + kTdsSpan, V.n);
    {
        const uint32_t q0 = p0 + t * kSpanItems;
        uint32_t flags = 0, cnt = 0;
        if (q0 < p1) {
            uint32_t kk[kSpanItems];  // (every load issued before any is used)
#pragma unroll
            for (int j = 0; j < kSpanItems; ++j) kk[j] = q0 + (uint32_t)j < p1 ? V.tkeys[q0 + j] : 0u;
            uint32_t prev = q0 > 0 ? V.tkeys[q0 - 1] : ~kk[0];
#pragma unroll
            for (int j = 0; j < kSpanItems; ++j) {
                if (q0 + (uint32_t)j < p1 && kk[j] != prev) flags |= 1u << j;
                prev = kk[j];
            }
            cnt = (uint32_t)__popc(flags);
        }
        uint32_t total;
        uint32_t o = block_exclusive<kTdsThreads>(cnt, R.scan, total);
#pragma unroll
        for (int j = 0; j < kSpanItems; ++j)
            if (flags & (1u << j)) R.start[o++] = (uint16_t)(t * kSpanItems + (uint32_t)j);
        if (t == 0) R.n_runs = total;
    }
    __syncthreads();
    const uint32_t n_runs = R.n_runs;  // (0: the whole span continues a run begun before it)
    // where the span's last run ends (it may go on past p1; a long one is not this block's): wave 0 looks
    // at most kTdsCapWave + 1 instances past p1, 64 at a time
    if (w == 0) {
        uint32_t e = p1;
        if (n_runs > 0 && p1 < V.n) {
            const uint32_t key = V.tkeys[p0 + R.start[n_runs - 1]];
            constexpr int kLook = (int)(kTdsCapWave + 64) / 64;  // 17 loads per lane, all in flight
            uint32_t kk[kLook];
#pragma unroll
            for (int c = 0; c < kLook; ++c) {
                const uint32_t i = p1 + (uint32_t)c * 64u + lane;
                kk[c] = i < V.n ? V.tkeys[i] : ~key;
            }
            e = 0xffffffffu;
#pragma unroll
            for (int c = kLook - 1; c >= 0; --c) {  // the first mismatch: the lowest chunk that has one
                const uint64_t m = __ballot(kk[c] != key);
                if (m) e = p1 + (uint32_t)c * 64u + (uint32_t)__builtin_ctzll(m);
            }
            if (e == 0xffffffffu) e = V.n;  // longer than kTdsCapWave: a long run (part A)
        }
        if (lane == 0) R.last_end = min(e, V.n);
    }
    __syncthreads();
    if (st && t == 0) st[2] = __builtin_amdgcn_s_memrealtime();
    uint32_t small_items = 0;
    if (!(dbg & 2u)) {
        for (uint32_t r = w; r < n_runs; r += kTdsWaves) {
            const uint32_t b = p0 + R.start[r];
            const uint32_t e = r + 1 < n_runs ? p0 + R.start[r + 1] : R.last_end;
            const uint32_t L = e - b;
            if (L >= 2u && L <= kTdsCapWave) {
                tds_wave(V.keys, V.vals, b, L, S.wave[w], dbg);
                small_items += L;
            }
        }
    }
    if (st) {
        __syncthreads();
        if (t == 0) {
            st[3] = __builtin_amdgcn_s_memrealtime();
            st[4] = big_done;
            st[5] = big_items;
            st[6] = n_runs;
        }
        if (lane == 0) atomicAdd(reinterpret_cast<unsigned long long*>(st + 7), (unsigned long long)small_items);
    }
}

}  // namespace

int launch_tile_depth_sort(const TileSortView* views, int k, hipStream_t s, uint32_t debug, uint64_t* stamps) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "tile depth sort: view count out of range");
    TdsViews tv{};
    tv.stamps = stamps;
    uint32_t n_max = 0;
    for (int i = 0; i < k; ++i) {
        const TileSortView& a = views[i];
        if (a.n_dup && (!a.tile_keys || !a.keys || !a.vals || !a.keys_alt || !a.vals_alt || !a.big_runs ||
                        !a.big_count))
            return set_error(GSR_ERR_INVALID, "tile depth sort: null buffer");
        tv.v[i] = TdsView{a.tile_keys, a.keys, a.vals, a.keys_alt, a.vals_alt, a.n_dup, a.big_runs, a.big_count};
        n_max = std::max(n_max, a.n_dup);
    }
    if (n_max == 0) return GSR_OK;
    const uint32_t grid = (n_max + kTdsSpan - 1) / kTdsSpan;
    k_tile_depth_sort<<<dim3(grid, (unsigned)k), kTdsThreads, 0, s>>>(tv, debug);
    GSR_LAUNCH_CHECK("tile_depth_sort");
    return GSR_OK;
}

}  // namespace gsr

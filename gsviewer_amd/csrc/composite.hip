// Tile binning + 16x16-tile front-to-back compositing.
//
// Binning: splats are visited in front-to-back depth order (the result of the
// depth radix sort); splat at sorted position r writes one (tile, record)
// instance per 16x16 tile its covered pixel rectangle touches, at the offset
// given by the prefix sum of the per-splat tile counts.  A stable radix sort by
// tile id then groups instances per tile WITHOUT disturbing depth order, and
// k_tile_ranges marks each tile's [begin, end).
//
// Compositing (the fragment stage gau_frag.glsl:14-53 + GL SRC_ALPHA /
// ONE_MINUS_SRC_ALPHA blending, evaluated front-to-back with transmittance):
// one wave64 per chunk of a tile's list (see k_build_chunks), 4 pixels per lane
// (four horizontal 16x4 slices), records staged per wave through LDS, no
// workgroup barriers; a wave retires as soon as all its 256 pixels are
// saturated (transmittance < t_min).  Slices a splat's row span misses are
// skipped with a scalar branch.
#include <algorithm>
#include <cstdlib>

#include "gsr_internal.h"
#include "long_runs.h"

#ifndef GSR_COMP_PIPE
#define GSR_COMP_PIPE 0  // (experiment: software-pipelined record reads in the compositor, composite_chunk)
#endif

namespace gsr {
namespace {

constexpr int kThreads = 256;

// Binning: tile instances of the depth-sorted splats.  Each 256-thread block
// owns 1024 consecutive sorted splats (4 per thread); the tile rectangle of a
// splat comes from the compact 8-B trect written by the preprocess.
constexpr int kBinItems = 4;
constexpr int kBinBlock = kThreads * kBinItems;  // 1024
// instances a k_bin_write block stages in LDS (16 KB: keys + values) before one
// coalesced write of its run; blocks with more write directly.  The bench
// scene averages 1.76 instances per splat (1800 per block).
#ifndef GSR_BIN_STAGE
#define GSR_BIN_STAGE 2048
#endif
constexpr int kBinStage = GSR_BIN_STAGE;

// Blocks of at most stage_limit instances take the staged write (default and
// upper bound kBinStage; the context's GSR_BIN_STAGE_LIMIT, read at creation,
// lowers it so a test can make one frame mix staged and direct blocks).
__device__ __forceinline__ uint32_t rect_tiles(uint2 tr) {
    const uint32_t tx0 = tr.x & 0xffffu, tx1 = tr.x >> 16, ty0 = tr.y & 0xffffu, ty1 = tr.y >> 16;
    return (tx0 <= tx1) ? (tx1 - tx0 + 1) * (ty1 - ty0 + 1) : 0u;
}

// Packed rectangle (radix_sort_pairs payload, pack_rect) back to the uint2 form.
__device__ __forceinline__ uint2 unpack_rect(uint32_t p) {
    return make_uint2((p & 0xffu) | ((p >> 8) & 0xffu) << 16, ((p >> 16) & 0xffu) | (p >> 24) << 16);
}

// Also writes the gathered rects in depth order (trect_sorted), so that
// k_bin_write reads them coalesced instead of gathering them a second time.
// kPacked: the depth sort carried the rects (rect4_sorted, in depth order):
// nothing is gathered.
template <bool kPacked>
__device__ __forceinline__ void bin_reduce(const uint32_t* __restrict__ sorted_ids, const uint2* __restrict__ trect,
                                           const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                           uint32_t* __restrict__ block_sums, uint2* __restrict__ trect_sorted,
                                           uint32_t blk, uint32_t* lds) {
    const uint32_t base = blk * kBinBlock + threadIdx.x;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t r = base + k * kThreads;
        if (r < n_vis) {
            if constexpr (kPacked) {
                s += rect_tiles(unpack_rect(rect4_sorted[r]));
            } else {
                const uint32_t id = sorted_ids[r];
                // (ids are record slots the depth sort produced: always in range, and
                // not below n_vis with the fused cull's uncompacted slots)
                const uint2 tr = trect[id];
                trect_sorted[r] = tr;
                s += rect_tiles(tr);
            }
        }
    }
    s = wave_reduce_sum(s);
    if (__lane_id() == 0) lds[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) block_sums[blk] = lds[0] + lds[1] + lds[2] + lds[3];
}

template <bool kPacked>
__global__ __launch_bounds__(kThreads) void k_bin_reduce(const uint32_t* __restrict__ sorted_ids,
                                                         const uint2* __restrict__ trect,
                                                         const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                                         uint32_t* __restrict__ block_sums,
                                                         uint2* __restrict__ trect_sorted) {
    __shared__ uint32_t lds[kThreads / 64];
    bin_reduce<kPacked>(sorted_ids, trect, rect4_sorted, n_vis, block_sums, trect_sorted, blockIdx.x, lds);
}

// Exclusive offsets of the block's splats (block prefix + in-block scan), then
// one (tile key, record slot) instance per covered tile, row-major.  The
// block prefix is the sum of the earlier blocks' totals (bin_reduce), read
// here (a few thousand words at most, L2-resident) instead of scanned by a
// launch of its own.
template <bool kPacked>
__device__ __forceinline__ void bin_write(const uint32_t* __restrict__ sorted_ids,
                                          const uint2* __restrict__ trect_sorted,
                                          const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                          const uint32_t* __restrict__ block_sums, int tiles_x,
                                          uint32_t* __restrict__ tile_keys, uint32_t* __restrict__ tile_vals,
                                          uint32_t blk, uint32_t* lds, uint32_t* stage, uint32_t stage_limit) {
    uint32_t pre = 0;  // this thread's share of the earlier blocks' totals
    for (uint32_t b = threadIdx.x; b < blk; b += kThreads) pre += block_sums[b];
    const uint32_t base = blk * kBinBlock + threadIdx.x * kBinItems;  // 4 consecutive per thread
    uint32_t id[kBinItems];
    uint2 tr[kBinItems];
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t r = base + k;
        id[k] = r < n_vis ? sorted_ids[r] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        if constexpr (kPacked)
            tr[k] = (base + k < n_vis) ? unpack_rect(rect4_sorted[base + k]) : make_uint2(0xffffu, 0u);
        else
            tr[k] = (base + k < n_vis) ? trect_sorted[base + k] : make_uint2(0xffffu, 0u);
        s += rect_tiles(tr[k]);
    }
    const int w = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive_scan(s);
    pre = wave_reduce_sum(pre);
    if (__lane_id() == 63) lds[w] = inc;
    if (__lane_id() == 0) lds[kThreads / 64 + w] = pre;
    __syncthreads();
    uint32_t o = inc - s;  // this thread's offset within the block's instances
    uint32_t block_base = 0, block_total = 0;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) {
        o += (k < w) ? lds[k] : 0u;
        block_total += lds[k];
        block_base += lds[kThreads / 64 + k];
    }
    if (block_total <= stage_limit) {  // (stage_limit <= kBinStage)
        // staged: instances into LDS, then the block's run written coalesced
        // (direct per-thread writes scatter 2 words per instance across lanes)
#pragma unroll
        for (int k = 0; k < kBinItems; ++k) {
            const uint32_t tx0 = tr[k].x & 0xffffu, tx1 = tr[k].x >> 16, ty0 = tr[k].y & 0xffffu, ty1 = tr[k].y >> 16;
            if (tx0 > tx1) continue;
            for (uint32_t ty = ty0; ty <= ty1; ++ty)
                for (uint32_t tx = tx0; tx <= tx1; ++tx) {
                    stage[o] = ty * (uint32_t)tiles_x + tx;
                    stage[kBinStage + o] = id[k];
                    ++o;
                }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < block_total; i += kThreads) {
            tile_keys[block_base + i] = stage[i];
            tile_vals[block_base + i] = stage[kBinStage + i];
        }
        return;
    }
    o += block_base;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t tx0 = tr[k].x & 0xffffu, tx1 = tr[k].x >> 16, ty0 = tr[k].y & 0xffffu, ty1 = tr[k].y >> 16;
        if (tx0 > tx1) continue;
        for (uint32_t ty = ty0; ty <= ty1; ++ty)
            for (uint32_t tx = tx0; tx <= tx1; ++tx) {
                tile_keys[o] = ty * (uint32_t)tiles_x + tx;
                tile_vals[o] = id[k];
                ++o;
            }
    }
}

template <bool kPacked>
__global__ __launch_bounds__(kThreads) void k_bin_write(const uint32_t* __restrict__ sorted_ids,
                                                        const uint2* __restrict__ trect_sorted,
                                                        const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                                        const uint32_t* __restrict__ block_sums, int tiles_x,
                                                        uint32_t* __restrict__ tile_keys,
                                                        uint32_t* __restrict__ tile_vals, uint32_t stage_limit) {
    __shared__ uint32_t lds[2 * kThreads / 64];
    __shared__ uint32_t stage[2 * kBinStage];
    bin_write<kPacked>(sorted_ids, trect_sorted, rect4_sorted, n_vis, block_sums, tiles_x, tile_keys, tile_vals,
                       blockIdx.x, lds, stage, stage_limit);
}

// Views of a group (blockIdx.y = view); the grid covers the largest view.
struct BinView {
    const uint32_t* sorted_ids;
    const uint2* trect;
    const uint32_t* rect4_sorted;
    uint2* trect_sorted;
    uint32_t* block_sums;
    uint32_t* tile_keys;
    uint32_t* tile_vals;
    uint32_t n_vis;
};
struct BinViews {
    BinView v[kMaxViews];
};

template <bool kPacked>
__global__ __launch_bounds__(kThreads) void k_bin_reduce_views(BinViews vs) {
    __shared__ uint32_t lds[kThreads / 64];
    const BinView& v = vs.v[blockIdx.y];
    if (blockIdx.x * kBinBlock >= v.n_vis) return;
    bin_reduce<kPacked>(v.sorted_ids, v.trect, v.rect4_sorted, v.n_vis, v.block_sums, v.trect_sorted, blockIdx.x,
                        lds);
}

template <bool kPacked>
__global__ __launch_bounds__(kThreads) void k_bin_write_views(BinViews vs, int tiles_x, uint32_t stage_limit) {
    __shared__ uint32_t lds[2 * kThreads / 64];
    __shared__ uint32_t stage[2 * kBinStage];
    const BinView& v = vs.v[blockIdx.y];
    if (blockIdx.x * kBinBlock >= v.n_vis) return;
    bin_write<kPacked>(v.sorted_ids, v.trect_sorted, v.rect4_sorted, v.n_vis, v.block_sums, tiles_x, v.tile_keys,
                       v.tile_vals, blockIdx.x, lds, stage, stage_limit);
}

// ------------------------------------------------------------------------
// The tile sort's first radix pass fused into the binning (the default).
// The tile sort is a stable LSD radix over the instances in binning order
// (depth order, then row-major tiles of each splat).  Its first pass orders
// the instances by digit 0 of the tile id; the binning produces them anyway,
// so it writes each one straight to that pass's position:
//   k_bin_hist:    per block of 1024 depth-sorted splats, its instances per
//                  digit 0 (LDS atomics), digit-major hist[d * blocks + b];
//   radix_offsets: the per-digit exclusive prefix over the blocks (the radix
//                  sort's own offsets kernel) and the digit totals;
//   k_bin_scatter: the block's instances in generation order staged in LDS
//                  (windows of kBinStage), ranked stably by digit (ballot
//                  matching, per-wave digit counts), restaged in digit order
//                  and written as contiguous runs to their pass-0 positions.
// The instances leave the binning already sorted by digit 0: the tile sort's
// pass-0 upsweep and scatter launches and one read + write of every instance
// are gone.  The remaining passes run as before (radix_sort_pairs from pass 1).
template <int kCB>
struct BinScatterLds {
    uint32_t k[kBinStage], v[kBinStage];    // a window of the block's instances, generation order
    uint32_t k2[kBinStage], v2[kBinStage];  // ... restaged in digit order
    uint16_t wcnt[kThreads / 64][1 << kCB];  // per-wave digit counts, then per-wave prefixes
    uint32_t dbase[1 << kCB];                // window-local digit offsets
    uint32_t gbase[1 << kCB];                // global position of the digit's next instance
    uint32_t scan[2][kThreads / 64];
    uint32_t own_o[kThreads + 1];            // balanced fill: each thread's first instance, then the total
    uint32_t wmax[kThreads / 64];
};

// A block whose splats cover more than this many tiles each is enumerated
// balanced (instance_at): every thread takes every kThreads-th instance of
// the block.  Otherwise each thread walks its own splats' rectangles, which
// costs as many serial steps as its largest splat has tiles: a block of
// large near-camera splats (they are adjacent in depth order) would run
// almost single-lane.
constexpr uint32_t kSerialTiles = 64;

// Instance idx (generation order: depth-sorted splats, each one's tiles
// row-major) of block blk -> (tile key, record slot), given own_o: the
// exclusive offsets of the block's threads' instances (thread t owns splats
// blk * kBinBlock + 4t .. 4t + 3), own_o[kThreads] = the block's total.
template <bool kPacked>
__device__ __forceinline__ void instance_at(uint32_t idx, const uint32_t* own_o, uint32_t blk,
                                            const uint32_t* __restrict__ sorted_ids,
                                            const uint2* __restrict__ trect_sorted,
                                            const uint32_t* __restrict__ rect4_sorted, int tiles_x, uint32_t& key,
                                            uint32_t& val, bool sorted_pos = false) {
    uint32_t lo = 0, hi = kThreads;  // own_o[lo] <= idx < own_o[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (own_o[mid] <= idx) lo = mid;
        else hi = mid;
    }
    uint32_t local = idx - own_o[lo];
    const uint32_t base = blk * kBinBlock + lo * kBinItems;
    key = 0xffffffffu;
    val = 0u;
    // (thread lo's instances all come from its splats below n_vis, which come first)
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t r = base + k;
        const uint2 tr = kPacked ? unpack_rect(rect4_sorted[r]) : trect_sorted[r];
        const uint32_t n = rect_tiles(tr);
        if (local < n) {
            const uint32_t tx0 = tr.x & 0xffffu, tx1 = tr.x >> 16, ty0 = tr.y & 0xffffu;
            const uint32_t w = tx1 - tx0 + 1u;
            const uint32_t dy = local / w;
            key = (ty0 + dy) * (uint32_t)tiles_x + tx0 + (local - dy * w);
            val = sorted_pos ? r : sorted_ids[r];
            return;
        }
        local -= n;
    }
}

// Block-wide unsigned max (every thread gets it); scratch: kThreads / 64 words.
__device__ __forceinline__ uint32_t block_max(uint32_t v, uint32_t* scratch) {
    v = wave_reduce_max(v);
    if (__lane_id() == 0) scratch[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) m = max(m, scratch[k]);
    return m;
}

// (sorted rect of depth-sorted splat r)
template <bool kPacked>
__device__ __forceinline__ uint2 sorted_rect(const uint32_t* __restrict__ sorted_ids, const uint2* __restrict__ trect,
                                             const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis, uint32_t r,
                                             uint2* __restrict__ trect_sorted) {
    if constexpr (kPacked) {
        return unpack_rect(rect4_sorted[r]);
    } else {
        const uint2 tr = trect[sorted_ids[r]];  // (a record slot: not below n_vis with the fused cull)
        trect_sorted[r] = tr;
        return tr;
    }
}

// Per-block digit counts.  The rects are read in the coalesced strided layout
// (and written in depth order for the non-packed form); a block with a splat
// over kSerialTiles tiles counts its instances balanced instead (instance_at,
// the consecutive layout bin_scatter uses).  own: kThreads + 1 + 2 kThreads / 64
// words of LDS.
template <bool kPacked, int kCB>
__device__ __forceinline__ void bin_hist(const uint32_t* __restrict__ sorted_ids, const uint2* __restrict__ trect,
                                         const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis, int tiles_x,
                                         const PassArgs& pa, uint32_t* __restrict__ hist, uint32_t nbb,
                                         uint2* __restrict__ trect_sorted, uint32_t blk, uint32_t* h,
                                         uint32_t* own) {
    const Digit dg = digit_params(pa);
    const uint32_t radix = dg.mask + 1u;
    for (uint32_t d = threadIdx.x; d < radix; d += kThreads) h[d] = 0u;
    const uint32_t base = blk * kBinBlock + threadIdx.x;
    uint2 tr[kBinItems];
    uint32_t nmax = 0;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t r = base + k * kThreads;
        tr[k] = r < n_vis ? sorted_rect<kPacked>(sorted_ids, trect, rect4_sorted, n_vis, r, trect_sorted)
                          : make_uint2(0xffffu, 0u);
        nmax = max(nmax, rect_tiles(tr[k]));
    }
    uint32_t* own_o = own;
    if (block_max(nmax, own + kThreads + 1) <= kSerialTiles) {  // (its barrier also orders the zeroing of h)
#pragma unroll
        for (int k = 0; k < kBinItems; ++k) {
            const uint32_t tx0 = tr[k].x & 0xffffu, tx1 = tr[k].x >> 16, ty0 = tr[k].y & 0xffffu, ty1 = tr[k].y >> 16;
            if (tx0 > tx1) continue;
            for (uint32_t ty = ty0; ty <= ty1; ++ty)
                for (uint32_t tx = tx0; tx <= tx1; ++tx) atomicAdd(&h[dg.of(ty * (uint32_t)tiles_x + tx)], 1u);
        }
    } else {
        // thread t's instances in the consecutive layout: splats blk * kBinBlock + 4t .. 4t + 3
        const uint32_t cb = blk * kBinBlock + threadIdx.x * kBinItems;
        uint32_t sc = 0;
#pragma unroll
        for (int k = 0; k < kBinItems; ++k)
            if (cb + k < n_vis) sc += rect_tiles(kPacked ? unpack_rect(rect4_sorted[cb + k]) : trect_sorted[cb + k]);
        uint32_t total;
        const uint32_t o = block_exclusive<kThreads>(sc, own + kThreads + 1 + kThreads / 64, total);
        own_o[threadIdx.x] = o;
        if (threadIdx.x == kThreads - 1) own_o[kThreads] = total;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < total; i += kThreads) {
            uint32_t key, val;
            instance_at<kPacked>(i, own_o, blk, sorted_ids, trect_sorted, rect4_sorted, tiles_x, key, val);
            atomicAdd(&h[dg.of(key)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < radix; d += kThreads) hist[(size_t)d * nbb + blk] = h[d];
}

template <bool kPacked, int kCB>
__global__ __launch_bounds__(kThreads) void k_bin_hist(const uint32_t* __restrict__ sorted_ids,
                                                       const uint2* __restrict__ trect,
                                                       const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                                       int tiles_x, PassArgs pa, uint32_t* __restrict__ hist,
                                                       uint32_t nbb, uint2* __restrict__ trect_sorted) {
    __shared__ uint32_t h[1 << kCB];
    __shared__ uint32_t own[kThreads + 1 + 2 * kThreads / 64];
    bin_hist<kPacked, kCB>(sorted_ids, trect, rect4_sorted, n_vis, tiles_x, pa, hist, nbb, trect_sorted, blockIdx.x,
                           h, own);
}

// kKeys: each instance also carries its splat's depth key (sorted_keys, in
// depth order) to inst_keys, for the coarse depth order's run repair.  The
// window then stages each instance's depth-sorted position instead of its
// slot, and the writes look up both (this block's 1024 splats: cache-hot):
// staging the keys as well took 16 KB more LDS (a block fewer per CU).
template <bool kPacked, int kCB, bool kKeys = false>
__device__ __forceinline__ void bin_scatter(const uint32_t* __restrict__ sorted_ids,
                                            const uint2* __restrict__ trect_sorted,
                                            const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis, int tiles_x,
                                            const PassArgs& pa, const uint32_t* __restrict__ hist_off,
                                            const uint32_t* __restrict__ totals, uint32_t nbb,
                                            uint32_t* __restrict__ tile_keys, uint32_t* __restrict__ tile_vals,
                                            uint32_t blk, BinScatterLds<kCB>& L,
                                            const uint32_t* __restrict__ sorted_keys = nullptr,
                                            uint32_t* __restrict__ inst_keys = nullptr) {
    constexpr int kCap = 1 << kCB;
    constexpr int kDpt = kCap / kThreads > 0 ? kCap / kThreads : 1;  // digits per thread
    constexpr int kWaveItems = kBinStage / (kThreads / 64);           // window items per wave
    constexpr int kRounds = kWaveItems / 64;
    const Digit dg = digit_params(pa);
    const uint32_t radix = dg.mask + 1u;
    const int w = threadIdx.x >> 6;
    // digits of this thread: [d0, d0 + q); their totals and this block's offsets
    const uint32_t q = (radix + kThreads - 1) / kThreads;
    const uint32_t d0 = threadIdx.x * q;
    uint32_t gt[kDpt], ho[kDpt];
#pragma unroll
    for (int j = 0; j < kDpt; ++j) {
        const uint32_t d = d0 + j;
        const bool mine = j < (int)q && d < radix;
        gt[j] = mine ? totals[d] : 0u;
        ho[j] = mine ? hist_off[(size_t)d * nbb + blk] : 0u;
    }
    // this thread's 4 consecutive depth-sorted splats
    const uint32_t base = blk * kBinBlock + threadIdx.x * kBinItems;
    uint32_t id[kBinItems];
    uint2 tr[kBinItems];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) {
        const uint32_t r = base + k;
        id[k] = kKeys ? r : r < n_vis ? sorted_ids[r] : 0u;  // kKeys: the sorted position
        if constexpr (kPacked)
            tr[k] = r < n_vis ? unpack_rect(rect4_sorted[r]) : make_uint2(0xffffu, 0u);
        else
            tr[k] = r < n_vis ? trect_sorted[r] : make_uint2(0xffffu, 0u);
        s += rect_tiles(tr[k]);
    }
    {  // global start of each digit's run of this block: digit base + the earlier blocks' counts
        uint32_t sg = 0;
#pragma unroll
        for (int j = 0; j < kDpt; ++j) sg += gt[j];
        uint32_t tg;
        uint32_t eg = block_exclusive<kThreads>(sg, L.scan[0], tg);
#pragma unroll
        for (int j = 0; j < kDpt; ++j) {
            const uint32_t d = d0 + j;
            if (j < (int)q && d < radix) L.gbase[d] = eg + ho[j];
            eg += gt[j];
        }
    }
    uint32_t total;
    const uint32_t o = block_exclusive<kThreads>(s, L.scan[1], total);  // (its barrier publishes gbase)
    uint32_t nmax = 0;
#pragma unroll
    for (int k = 0; k < kBinItems; ++k) nmax = max(nmax, rect_tiles(tr[k]));
    const bool balanced = block_max(nmax, L.wmax) > kSerialTiles;
    if (balanced) {
        L.own_o[threadIdx.x] = o;
        if (threadIdx.x == 0) L.own_o[kThreads] = total;
        __syncthreads();
    }
    for (uint32_t c0 = 0; c0 < total; c0 += (uint32_t)kBinStage) {
        // 1. this window's instances, in generation order
        if (balanced) {
            const uint32_t cnt = min((uint32_t)kBinStage, total - c0);
            for (uint32_t j = threadIdx.x; j < cnt; j += kThreads)
                instance_at<kPacked>(c0 + j, L.own_o, blk, sorted_ids, trect_sorted, rect4_sorted, tiles_x, L.k[j],
                                     L.v[j], kKeys);
        } else if (o < c0 + (uint32_t)kBinStage && o + s > c0) {
            uint32_t idx = o;
#pragma unroll
            for (int k = 0; k < kBinItems; ++k) {
                const uint32_t tx0 = tr[k].x & 0xffffu, tx1 = tr[k].x >> 16, ty0 = tr[k].y & 0xffffu,
                               ty1 = tr[k].y >> 16;
                if (tx0 > tx1) continue;
                for (uint32_t ty = ty0; ty <= ty1; ++ty)
                    for (uint32_t tx = tx0; tx <= tx1; ++tx, ++idx)
                        if (idx >= c0 && idx < c0 + (uint32_t)kBinStage) {
                            L.k[idx - c0] = ty * (uint32_t)tiles_x + tx;
                            L.v[idx - c0] = id[k];
                        }
            }
        }
        {
            uint32_t* wz = reinterpret_cast<uint32_t*>(&L.wcnt[0][0]);
            for (uint32_t i = threadIdx.x; i < (uint32_t)(kThreads / 64 * kCap / 2); i += kThreads) wz[i] = 0u;
        }
        __syncthreads();
        const uint32_t cnt = min((uint32_t)kBinStage, total - c0);
        // 2. stable ranks: wave w owns window items [w * kWaveItems, (w + 1) * kWaveItems)
        uint32_t key[kRounds], rank[kRounds];
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            const uint32_t j = (uint32_t)(w * kWaveItems + r * 64) + __lane_id();
            const bool valid = j < cnt;
            key[r] = valid ? L.k[j] : 0u;
            const uint32_t d = dg.of(key[r]);
            const uint64_t peers = match_digit(d, dg.w, valid);
            uint32_t rk = 0xffffffffu;
            if (valid) {
                const uint32_t old = L.wcnt[w][d];
                const uint32_t below =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
                rk = old + below;
                if (below == 0) L.wcnt[w][d] = (uint16_t)(old + __popcll(peers));
            }
            rank[r] = rk;
        }
        __syncthreads();
        // 3. per owned digit: wave prefixes, the window-local digit offsets
        uint32_t tot[kDpt];
        {
            uint32_t sl = 0;
#pragma unroll
            for (int j = 0; j < kDpt; ++j) {
                const uint32_t d = d0 + j;
                tot[j] = 0u;
                if (j < (int)q && d < radix) {
                    uint32_t run = 0;
#pragma unroll
                    for (int k = 0; k < kThreads / 64; ++k) {
                        const uint32_t c = L.wcnt[k][d];
                        L.wcnt[k][d] = (uint16_t)run;
                        run += c;
                    }
                    tot[j] = run;
                }
                sl += tot[j];
            }
            uint32_t tl;
            uint32_t el = block_exclusive<kThreads>(sl, L.scan[0], tl);
#pragma unroll
            for (int j = 0; j < kDpt; ++j) {
                const uint32_t d = d0 + j;
                if (j < (int)q && d < radix) L.dbase[d] = el;
                el += tot[j];
            }
        }
        __syncthreads();
        // 4. restage in digit order
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            if (rank[r] != 0xffffffffu) {
                const uint32_t j = (uint32_t)(w * kWaveItems + r * 64) + __lane_id();
                const uint32_t d = dg.of(key[r]);
                const uint32_t p = L.dbase[d] + L.wcnt[w][d] + rank[r];
                L.k2[p] = key[r];
                L.v2[p] = L.v[j];
            }
        }
        __syncthreads();
        // 5. contiguous runs to the pass-0 positions
        for (uint32_t j = threadIdx.x; j < cnt; j += kThreads) {
            const uint32_t kk = L.k2[j];
            const uint32_t d = dg.of(kk);
            const uint32_t g = L.gbase[d] + (j - L.dbase[d]);
            tile_keys[g] = kk;
            if constexpr (kKeys) {
                const uint32_t r = L.v2[j];
                tile_vals[g] = sorted_ids[r];
                inst_keys[g] = sorted_keys[r];
            } else {
                tile_vals[g] = L.v2[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kDpt; ++j) {
            const uint32_t d = d0 + j;
            if (j < (int)q && d < radix) L.gbase[d] += tot[j];  // the next window continues each run
        }
        __syncthreads();
    }
}

template <bool kPacked, int kCB, bool kKeys>
__global__ __launch_bounds__(kThreads) void k_bin_scatter(const uint32_t* __restrict__ sorted_ids,
                                                          const uint2* __restrict__ trect_sorted,
                                                          const uint32_t* __restrict__ rect4_sorted, uint32_t n_vis,
                                                          int tiles_x, PassArgs pa,
                                                          const uint32_t* __restrict__ hist_off,
                                                          const uint32_t* __restrict__ totals, uint32_t nbb,
                                                          uint32_t* __restrict__ tile_keys,
                                                          uint32_t* __restrict__ tile_vals,
                                                          const uint32_t* __restrict__ sorted_keys,
                                                          uint32_t* __restrict__ inst_keys) {
    __shared__ BinScatterLds<kCB> L;
    bin_scatter<kPacked, kCB, kKeys>(sorted_ids, trect_sorted, rect4_sorted, n_vis, tiles_x, pa, hist_off, totals,
                                     nbb, tile_keys, tile_vals, blockIdx.x, L, sorted_keys, inst_keys);
}

// Views of a group (blockIdx.y = view): hist / totals per view.
struct BinSortViews {
    BinView v[kMaxViews];
    uint32_t* hist[kMaxViews];
    const uint32_t* totals[kMaxViews];
};

// Every view's count matrix has nbb (the largest view's blocks) columns; a
// view's blocks past its own splats count zeros, so its offsets are exact.
template <bool kPacked, int kCB>
__global__ __launch_bounds__(kThreads) void k_bin_hist_views(BinSortViews vs, int tiles_x, PassArgs pa,
                                                             uint32_t nbb) {
    __shared__ uint32_t h[1 << kCB];
    __shared__ uint32_t own[kThreads + 1 + 2 * kThreads / 64];
    const BinView& v = vs.v[blockIdx.y];
    bin_hist<kPacked, kCB>(v.sorted_ids, v.trect, v.rect4_sorted, v.n_vis, tiles_x, pa, vs.hist[blockIdx.y], nbb,
                           v.trect_sorted, blockIdx.x, h, own);
}

template <bool kPacked, int kCB>
__global__ __launch_bounds__(kThreads) void k_bin_scatter_views(BinSortViews vs, int tiles_x, PassArgs pa,
                                                                uint32_t nbb) {
    __shared__ BinScatterLds<kCB> L;
    const BinView& v = vs.v[blockIdx.y];
    if (blockIdx.x * kBinBlock >= v.n_vis) return;
    bin_scatter<kPacked, kCB>(v.sorted_ids, v.trect_sorted, v.rect4_sorted, v.n_vis, tiles_x, pa, vs.hist[blockIdx.y],
                              vs.totals[blockIdx.y], nbb, v.tile_keys, v.tile_vals, blockIdx.x, L);
}

// Tile ranges from the tile-sorted keys: kRangeItems consecutive instances per
// thread (four dwordx4 loads plus the two neighbours), a write at each tile
// boundary only.  (One instance per thread meant 7K blocks per view at 1080p,
// each doing almost nothing: with views in flight they queued behind the
// compositors for CU slots.)
constexpr int kRangeItems = 16;

// The repair of one run of a coarse depth order, [i, i + L): instances of one
// tile with equal coarse keys, in slot order (the stable coarse sort's).  The
// exact order is (full key, slot); a run without a descent of the full key is
// already in it.  Otherwise each slot is written at its rank (the count of
// smaller keys, and of equal keys earlier in the run: slots ascend along it;
// an odd-even transposition here took 151 VGPRs: 64.7 -> 75.2 us at C3).
// One thread owns the run (the thread holding its first instance); other
// threads read the run's slots only for their (tile, coarse key), which the
// permutation leaves unchanged.  The kFixRunMax + 1 instances from the start
// are loaded at once and ranked in registers (round 4 scanned the run load by
// load, ~1 us per instance, and ranked it in global memory: C3's k_tile_ranges
// took 166 us, profiles/r5_s16).  A longer run is listed for the long-run
// sorts (long_runs.h), which sort it on chip in bounded time (round 4's
// unbounded form could spend ~5e8 serial steps on one dense tile).
__device__ __noinline__ void fix_run(const uint32_t* __restrict__ keys, uint32_t n, uint32_t* vals,
                                     const uint32_t* __restrict__ inst_keys, uint32_t* __restrict__ long_starts,
                                     uint32_t* __restrict__ long_count, uint32_t i, uint32_t tile, uint32_t cv,
                                     uint32_t kmin, uint32_t s0) {
    constexpr int M = (int)kFixRunMax + 1;
    uint32_t kk[M], ff[M], vv[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
        const bool ok = i + (uint32_t)j < n;
        kk[j] = ok ? keys[i + j] : ~tile;
        ff[j] = ok ? inst_keys[i + j] : 0u;
        vv[j] = ok ? vals[i + j] : 0u;
    }
    uint32_t L = 1;
    bool open = true, descent = false;
#pragma unroll
    for (int j = 1; j < M; ++j) {
        open = open && kk[j] == tile && ((ff[j] - kmin) >> s0) == cv;
        if (open) {
            ++L;
            descent |= ff[j] < ff[j - 1];
        }
    }
    if (L > kFixRunMax) {  // a long run: the long-run sorts find its end and sort it
        long_starts[atomicAdd(long_count, 1u)] = i;
        return;
    }
    if (!descent) return;
#pragma unroll
    for (int r = 0; r < M - 1; ++r) {
        uint32_t rank = 0;
#pragma unroll
        for (int q = 0; q < M - 1; ++q)
            rank += ((uint32_t)q < L && (ff[q] < ff[r] || (ff[q] == ff[r] && q < r))) ? 1u : 0u;
        if ((uint32_t)r < L) vals[i + rank] = vv[r];
    }
}

// The thread's kRangeItems instances: every run of equal (tile, coarse key)
// that starts among them is repaired, in registers over a window of the
// thread's items and the kFixExtra after them (all loads issued at once: a
// chain of dependent loads per run cost ~200 us at C2).  Runs are short (C2,
// 16 coarse bits: 41 % of the instances in runs, the longest 8; 22 bits: 1 %,
// 4), so an odd-even transposition sort restricted to pairs inside one run,
// as many rounds as the longest run, puts each in (full key, slot) order.  A
// run that reaches the window's end is left to fix_run (global memory).
constexpr int kFixExtra = 8;
// instances per thread of the repairing kernel (GSR_FIX_ITEMS build knob): 8
// (twice the waves of 16, the window's loads overlap more): 13.9 -> 10.8 us,
// 12: 12.0 (profiles/r4_s32/c9)
#ifndef GSR_FIX_ITEMS
#define GSR_FIX_ITEMS 8
#endif
constexpr int kFixItems = GSR_FIX_ITEMS;
static_assert(kFixItems % 4 == 0 && kFixItems + kFixExtra <= 32, "run masks are 32-bit");

template <int kItems>
__device__ __forceinline__ void fix_coarse_runs(const uint32_t* __restrict__ keys, uint32_t n, const RunFix& fx,
                                                uint32_t base, const uint32_t (&k)[kItems], uint32_t prev) {
    constexpr int kFixWin = kItems + kFixExtra;
    uint32_t kw[kFixWin], vw[kFixWin], fw[kFixWin];
    // the window's slots: with carried keys only once a run needs sorting (most windows' runs are in order)
    auto load_vals = [&]() {
        if (base + kFixWin <= n) {
            const uint4* pv = reinterpret_cast<const uint4*>(fx.vals + base);  // (base: a multiple of 16)
#pragma unroll
            for (int q = 0; q < kFixWin / 4; ++q) {
                const uint4 v = pv[q];
                vw[4 * q] = v.x; vw[4 * q + 1] = v.y; vw[4 * q + 2] = v.z; vw[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kFixWin; ++j) vw[j] = base + j < n ? fx.vals[base + j] : 0u;
        }
    };
#pragma unroll
    for (int j = 0; j < kItems; ++j) kw[j] = k[j];
    if (base + kFixWin <= n) {
        const uint4* pk = reinterpret_cast<const uint4*>(keys + base + kItems);
#pragma unroll
        for (int q = 0; q < kFixExtra / 4; ++q) {
            const uint4 v = pk[q];
            kw[kItems + 4 * q] = v.x; kw[kItems + 4 * q + 1] = v.y;
            kw[kItems + 4 * q + 2] = v.z; kw[kItems + 4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = kItems; j < kFixWin; ++j) kw[j] = base + j < n ? keys[base + j] : 0xffffffffu;
    }
    // the keys carried with the instances (binning + tile sort payload): coalesced
    if (base + kFixWin <= n) {
        const uint4* pf = reinterpret_cast<const uint4*>(fx.inst_keys + base);
#pragma unroll
        for (int q = 0; q < kFixWin / 4; ++q) {
            const uint4 v = pf[q];
            fw[4 * q] = v.x; fw[4 * q + 1] = v.y; fw[4 * q + 2] = v.z; fw[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kFixWin; ++j) fw[j] = base + j < n ? fx.inst_keys[base + j] : 0u;
    }
    const uint32_t fprev = base > 0 ? fx.inst_keys[base - 1] : 0u;
    uint32_t kmin;  // (the window's loads are in flight meanwhile)
    const uint32_t s0 = coarse_shift(fx.key_range, fx.coarse, kmin);
    if (s0 == 0u) return;  // the coarse sort was exact
    // same bit j: items j and j + 1 are one run (both valid, same tile and coarse key)
    uint32_t same = 0;
#pragma unroll
    for (int j = 0; j + 1 < kFixWin; ++j)
        if (base + j + 1 < n && kw[j] == kw[j + 1] && ((fw[j] - kmin) >> s0) == ((fw[j + 1] - kmin) >> s0))
            same |= 1u << j;
    // own bit j: item j is in a run that starts among the thread's items
    const bool cont0 = base > 0 && prev == kw[0] && ((fprev - kmin) >> s0) == ((fw[0] - kmin) >> s0);
    uint32_t own = cont0 ? 0u : 1u;
#pragma unroll
    for (int j = 1; j < kFixWin; ++j) {
        const bool in = ((same >> (j - 1)) & 1u) ? ((own >> (j - 1)) & 1u) != 0u : j < kItems;
        if (in) own |= 1u << j;
    }
    // a run that may go on past the window: fix_run from its start, out of the register sort
    if ((own >> (kFixWin - 1)) & 1u) {
        int st = kFixWin - 1;
#pragma unroll
        for (int j = kFixWin - 2; j >= 0; --j)
            if (st == j + 1 && ((same >> j) & 1u)) st = j;
        own &= (1u << st) - 1u;
        uint32_t kst = 0, fst = 0;  // items st (selected: a dynamic index would put the arrays in scratch)
#pragma unroll
        for (int j = 0; j < kFixWin; ++j)
            if (j == st) kst = kw[j], fst = fw[j];
        fix_run(keys, n, fx.vals, fx.inst_keys, fx.long_starts, fx.long_count, base + (uint32_t)st, kst,
                (fst - kmin) >> s0, kmin, s0);
    }
    const uint32_t pairs = same & own;  // adjacent pairs inside one owned run
    uint32_t descent = 0;
#pragma unroll
    for (int j = 0; j + 1 < kFixWin; ++j)
        if (((pairs >> j) & 1u) && fw[j] > fw[j + 1]) descent = 1u;  // slots ascend in a run: only keys descend
#ifdef GSR_EXP_FIX_NOSORT  // experiment build: the window's loads and tests only (timing; lists unrepaired)
    asm volatile("" ::"v"(descent));
    return;
#endif
    if (!descent) return;
    load_vals();
    // the longest owned run: rounds of the transposition sort
    uint32_t len = 1, rounds = 1;
#pragma unroll
    for (int j = 0; j + 1 < kFixWin; ++j) {
        len = ((pairs >> j) & 1u) ? len + 1u : 1u;
        rounds = max(rounds, len);
    }
    uint32_t v0[kFixWin];
#pragma unroll
    for (int j = 0; j < kFixWin; ++j) v0[j] = vw[j];
    // Rounds in pairs (an even pass, then an odd one: the pass parity is static, so each pass is half the
    // window's pairs with no parity test; one extra pass is harmless).  Strict > only: the slots ascend in a
    // run and adjacent swaps of strictly greater keys never cross equal ones, so the sort is stable and ties
    // stay in slot order (round 4's tie-break compared the slots too: C3's repair 78 -> 52 us, profiles/r5_s35).
    auto cx = [&](int j) {
        const bool gt = ((pairs >> j) & 1u) && fw[j] > fw[j + 1];
        const uint32_t fa = fw[j], va = vw[j];
        fw[j] = gt ? fw[j + 1] : fa;
        vw[j] = gt ? vw[j + 1] : va;
        fw[j + 1] = gt ? fa : fw[j + 1];
        vw[j + 1] = gt ? va : vw[j + 1];
    };
    for (uint32_t r = 0; r < rounds; r += 2) {
#pragma unroll
        for (int j = 0; j + 1 < kFixWin; j += 2) cx(j);
#pragma unroll
        for (int j = 1; j + 1 < kFixWin; j += 2) cx(j);
    }
#pragma unroll
    for (int j = 0; j < kFixWin; ++j)
        if (((own >> j) & 1u) && vw[j] != v0[j]) fx.vals[base + j] = vw[j];
}

// kFix: the coarse depth order's run repair (a separate instantiation: its
// registers (153 VGPRs) made the plain kernel wait for room beside the
// compositors in flight)
template <bool kFix, int kItems = kFix ? kFixItems : kRangeItems>
__device__ __forceinline__ void tile_ranges(const uint32_t* __restrict__ keys, uint32_t n, uint2* __restrict__ ranges,
                                            uint32_t t, const RunFix& fx) {
    const uint32_t base = t * kItems;
    if (base >= n) return;
    uint32_t k[kItems];
    if (base + kItems <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(keys + base);  // (base: a multiple of 16)
#pragma unroll
        for (int q = 0; q < kItems / 4; ++q) {
            const uint4 v = p[q];
            k[4 * q] = v.x; k[4 * q + 1] = v.y; k[4 * q + 2] = v.z; k[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kItems; ++j) k[j] = base + j < n ? keys[base + j] : 0xffffffffu;
    }
    const uint32_t prev = base > 0 ? keys[base - 1] : 0xffffffffu;
    const uint32_t next = base + kItems < n ? keys[base + kItems] : 0xffffffffu;
    // the run repair first: its window loads are issued before the range stores
    if constexpr (kFix) fix_coarse_runs<kItems>(keys, n, fx, base, k, prev);
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint32_t i = base + j;
        if (i >= n) break;
        const uint32_t before = j == 0 ? prev : k[j - 1];
        const uint32_t after = (j + 1 < kItems) ? (i + 1 < n ? k[j + 1] : 0xffffffffu) : next;
        if (i == 0 || before != k[j]) ranges[k[j]].x = i;
        if (i == n - 1 || after != k[j]) ranges[k[j]].y = i + 1;
    }
}

template <bool kFix>
__global__ __launch_bounds__(kThreads) void k_tile_ranges(const uint32_t* __restrict__ keys, uint32_t n,
                                                          uint2* __restrict__ ranges, RunFix fx) {
    tile_ranges<kFix>(keys, n, ranges, blockIdx.x * kThreads + threadIdx.x, fx);
}

struct RangeViews {
    const uint32_t* keys[kMaxViews];
    uint2* ranges[kMaxViews];
    uint32_t n[kMaxViews];
    RunFix fix[kMaxViews];
};

template <bool kFix>
__global__ __launch_bounds__(kThreads) void k_tile_ranges_views(RangeViews vs) {
    const int v = blockIdx.y;
    tile_ranges<kFix>(vs.keys[v], vs.n[v], vs.ranges[v], blockIdx.x * kThreads + threadIdx.x, vs.fix[v]);
}

struct CompositeArgs {
    int width, height, tiles_x, num_tiles;
    float t_min;
    float bg[3];
    int out_layout;
    int tail_merge;  // a multi-chunk tile's last chunk to finish folds the tile (no merge launch)
    uint32_t debug_handoff;  // test knob (GSR_DEBUG_HANDOFF, 0 in production): see composite_chunk's tail merge
};

constexpr int kBatch = 64;  // records staged per wave per LDS batch

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// kFragGauss keep test in two VALU ops, with no compare and lane-mask select
// (whose VCC hand-off also costs an s_nop on gfx950).  With m = -mid > 0 and
// pw' = pw - mid, a fragment is kept iff |pw'| <= m (SplatRec).
//   u = fma(-K, |pw'|, K m (1 + 2^-22)),  K = 2^64
// is K (m (1 + 2^-22) - |pw'|) rounded once, so its sign is exact, and when it
// is >= 0 it is >= K m 2^-23 >= 1 for any m > 2^-41; so
//   alpha = med3(u, 0, a1)  (a1 in [0, 1])
// is a1 inside the interval and 0 outside it.  The interval is widened by
// 2^-22 relative (a few ulps): fragments exactly on its ends are kept, as the
// reference's non-strict tests keep them; ulp-level boundary flips are inside
// the tolerance the evaluation order already has (the quadratic is not the
// reference's expression).
constexpr float kKeepScale = 18446744073709551616.0f;      // K = 2^64
constexpr float kKeepScaleWide = 18446748471756062720.0f;  // K (1 + 2^-22), exact
#ifdef GSR_COMP_TRACE
constexpr uint32_t kTraceMax = 1u << 16;  // waves traced per launch
#endif

// Chunks: every tile's instance list is cut into pieces of at most `chunk`
// instances (an empty tile gets one empty chunk so it still writes the
// background).  Front-to-back "over" is associative:
//   (C1, T1) then (C2, T2)  ==  (C1 + T1*C2, T1*T2)
// so chunks of one tile are composited by different waves in parallel and
// folded in depth order afterwards (k_merge).  This bounds the work of one
// wave, which is what the heavy tiles of a real scene (horizon lines,
// dense cores) need.
//
// Chunk slots (where a chunk's descriptor, partial and maxima live): slot t
// (< num_tiles) is chunk 0 of tile t; chunks k >= 1 of tile t are at
// num_tiles + extra_off[t] + k - 1.
//
// Dispatch order (longest first): order[i] is the slot the i-th compositing
// wave takes.  Chunks are dispatched by length class: every full chunk
// (`chunk` instances) first, then the partial ones (a tile's last, shorter
// chunk, or its only one) from the longest class to the shortest, in tile
// order within a class, so the waves that start last are the short ones.  In
// slot order the full extra chunks of the deep tiles started last and ran alone
// at the end of the launch (trace: the last third of the launch at falling
// occupancy).  A group's compositing launch interleaves its views by class
// (k_composite_views), so no view's long chunks start at the end.
__device__ __forceinline__ uint32_t chunks_of(uint2 r, uint32_t chunk) {
    const uint32_t len = r.y - r.x;
    return len == 0 ? 1u : (len + chunk - 1) / chunk;
}

// Chunks of a tile that hold exactly `chunk` instances (all but the last).
__device__ __forceinline__ uint32_t full_chunks_of(uint2 r, uint32_t chunk) { return (r.y - r.x) / chunk; }

// Length class of a tile's partial chunk, 1 (longest) .. classes - 1, or 0 if
// the tile has none (its list is a positive multiple of `chunk`).
__device__ __forceinline__ uint32_t partial_class_of(uint2 r, uint32_t chunk, uint32_t classes) {
    const uint32_t len = r.y - r.x;
    const uint32_t rem = len % chunk;
    if (len != 0 && rem == 0) return 0u;
    return (classes - 1u) - rem * (classes - 1u) / chunk;
}

// Chunk descriptors in two parallel launches (one thread per tile):
// k_chunk_count writes each block's totals (extra chunks beyond the first per
// tile; full chunks; partial chunks of each length class) into `tot`, array j
// at tot + j * gridDim.x; k_chunk_write takes its block's offsets as sums of
// the earlier block totals (a few dozen at 1080p), ranks its tiles' chunks,
// and writes the descriptors (tile, begin, end, count << 16 | index), each
// chunk's dispatch position and (block 0) the frame's chunks per class, at
// tot + (1 + classes) * gridDim.x.
// First-major order (a group's frames, `first_major`): every tile's first
// chunk (full ones, then by length class) before any later chunk (tile
// order).  A deep tile's chunk 0 then usually runs, and often saturates,
// before its later chunks start, so they find its saturation word and skip
// (sequential early termination visits 33 % of the instances, 3072-instance
// chunks started together 57 %: tools/comp_stats.py).
__device__ __forceinline__ uint32_t first_full_of(uint2 r, uint32_t chunk, bool first_major) {
    return first_major ? ((r.y - r.x) >= chunk ? 1u : 0u) : full_chunks_of(r, chunk);
}
__device__ __forceinline__ uint32_t first_class_of(uint2 r, uint32_t chunk, uint32_t classes, bool first_major) {
    return first_major && (r.y - r.x) >= chunk ? 0u : partial_class_of(r, chunk, classes);
}

// Tiles [grp * kThreads, (grp + 1) * kThreads) of ngrp such groups, thread lt
// of the group's kThreads (every thread of the launch's blocks calls it: one
// workgroup barrier)
__device__ __forceinline__ void chunk_count(const uint2* __restrict__ ranges, int num_tiles, uint32_t chunk,
                                            uint32_t classes, bool first_major, uint32_t* __restrict__ tot,
                                            uint32_t (*lds)[kThreads / 64], uint32_t grp, uint32_t ngrp, uint32_t lt) {
    const int t = (int)(grp * kThreads + lt);
    const bool valid = t < num_tiles;
    const uint2 r = valid ? ranges[t] : make_uint2(0u, 0u);
    const uint32_t e = wave_reduce_sum(valid ? chunks_of(r, chunk) - 1u : 0u);
    const uint32_t f = wave_reduce_sum(first_full_of(r, chunk, first_major));
    const uint32_t pc = valid ? first_class_of(r, chunk, classes, first_major) : 0u;
    const int w = (int)(lt >> 6);
    if (__lane_id() == 0) {
        lds[0][w] = e;
        lds[1][w] = f;
    }
    for (uint32_t k = 1; k < classes; ++k) {
        const uint32_t n = (uint32_t)__popcll(__ballot(pc == k));
        if (__lane_id() == 0) lds[1 + k][w] = n;
    }
    __syncthreads();
    if (lt <= classes && grp < ngrp) tot[lt * ngrp + grp] = lds[lt][0] + lds[lt][1] + lds[lt][2] + lds[lt][3];
}

__global__ __launch_bounds__(kThreads) void k_chunk_count(const uint2* __restrict__ ranges, int num_tiles,
                                                          uint32_t chunk, uint32_t classes,
                                                          uint32_t* __restrict__ tot, uint32_t first_major) {
    __shared__ uint32_t lds[1 + kMaxLenClasses][kThreads / 64];
    chunk_count(ranges, num_tiles, chunk, classes, first_major != 0, tot, lds, blockIdx.x, gridDim.x, threadIdx.x);
}

// The chunk counts with the coarse depth order's long runs (long_runs.h) in
// the same launch: blocks [0, n_cc) count (four tile groups of kThreads each,
// k_chunk_count's blocks), the rest sort the listed runs.  Saves the runs'
// own launch (4.7 us when there are none, profiles/r5_s14).
constexpr int kCountGroups = kTdsThreads / kThreads;
__global__ __launch_bounds__(kTdsThreads) void k_chunk_count_long(const uint2* __restrict__ ranges, int num_tiles,
                                                                  uint32_t chunk, uint32_t classes,
                                                                  uint32_t* __restrict__ tot, uint32_t first_major,
                                                                  uint32_t n_cc, LongRunArgs la) {
    __shared__ TdsLds S;
    __shared__ uint32_t lds[kCountGroups][1 + kMaxLenClasses][kThreads / 64];
    if (blockIdx.x < n_cc) {
        const uint32_t g = threadIdx.x / kThreads;
        const uint32_t ngrp = (uint32_t)((num_tiles + kThreads - 1) / kThreads);
        chunk_count(ranges, num_tiles, chunk, classes, first_major != 0, tot, lds[g], blockIdx.x * kCountGroups + g,
                    ngrp, threadIdx.x % kThreads);
        return;
    }
    long_runs_block(la, S, blockIdx.x - n_cc, gridDim.x - n_cc);
}

struct ChunkWriteLds {
    uint32_t scan[2][kThreads / 64];
    uint32_t cls[kMaxLenClasses][kThreads / 64];  // partials of class k per wave
    uint32_t pre[1 + kMaxLenClasses];             // sums over the earlier blocks
    uint32_t base[kMaxLenClasses];                // first dispatch position of each class
    // the block's multi-chunk tiles for the flattened emission of chunks j >= 1:
    // inclusive scan of (chunks - 1) per thread, and each thread's tile terms
    uint32_t incl[kThreads];
    uint32_t tile[kThreads][8];  // t, r.x, r.y, count, full, base, full_before, part_pos
};

__device__ __forceinline__ void chunk_write(const uint2* __restrict__ ranges, int num_tiles, uint32_t chunk,
                                            uint32_t classes, bool first_major, const uint32_t* __restrict__ tot,
                                            uint32_t* __restrict__ chunk_cnt, uint32_t* __restrict__ chunk_base,
                                            uint32_t* __restrict__ n_extra_dev, uint4* __restrict__ desc,
                                            uint32_t* __restrict__ order, float4* __restrict__ tmax,
                                            ChunkWriteLds& sh) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    const int w = threadIdx.x >> 6;
    if (w == 0) {  // wave 0: offsets of this block = sums of the earlier blocks' totals
        uint32_t* cls_tot = const_cast<uint32_t*>(tot) + (1 + classes) * gridDim.x;
        // every row's loads issued before any is summed: one memory round trip,
        // not one per class (a row-by-row loop waited 1 + classes times)
        uint32_t ps[1 + kMaxLenClasses], as[1 + kMaxLenClasses];
#pragma unroll
        for (int j = 0; j <= kMaxLenClasses; ++j) ps[j] = as[j] = 0u;
        for (uint32_t b = __lane_id(); b < gridDim.x; b += 64) {
            uint32_t v[1 + kMaxLenClasses];
#pragma unroll
            for (int j = 0; j <= kMaxLenClasses; ++j) v[j] = (uint32_t)j <= classes ? tot[j * gridDim.x + b] : 0u;
#pragma unroll
            for (int j = 0; j <= kMaxLenClasses; ++j) {
                ps[j] += b < blockIdx.x ? v[j] : 0u;
                as[j] += v[j];
            }
        }
        uint32_t run = 0;  // class bases: full chunks, then the partial classes in order
#pragma unroll
        for (int jj = 0; jj <= kMaxLenClasses; ++jj) {
            const uint32_t j = (uint32_t)jj;
            if (j > classes) continue;  // (uniform; `break` blocks the unrolling)
            const uint32_t p = wave_reduce_sum(ps[jj]);
            const uint32_t a = wave_reduce_sum(as[jj]);
            if (__lane_id() == 0) {
                sh.pre[j] = p;
                if (j == 0 && blockIdx.x == 0) cls_tot[classes] = a;  // the later chunks (first-major order)
                if (j >= 1) {
                    sh.base[j - 1] = run;
                    run += a;
                    if (blockIdx.x == 0) cls_tot[j - 1] = a;
                }
            }
        }
    }
    const bool valid = t < num_tiles;
    const uint2 r = valid ? ranges[t] : make_uint2(0u, 0u);
    const uint32_t cnt = chunks_of(r, chunk);
    const uint32_t full = first_full_of(r, chunk, first_major);
    const uint32_t pc = valid ? first_class_of(r, chunk, classes, first_major) : 0u;
    uint32_t rank = 0;  // among this wave's partials of class pc
    for (uint32_t k = 1; k < classes; ++k) {
        const uint64_t m = __ballot(pc == k);
        if (pc == k) rank = (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
        if (__lane_id() == 0) sh.cls[k][w] = (uint32_t)__popcll(m);
    }
    const uint32_t mine = valid ? cnt - 1u : 0u;
    uint32_t total, total_f;
    const uint32_t excl = block_exclusive<kThreads>(mine, sh.scan[0], total);  // (its barrier also publishes sh)
    const uint32_t excl_f = block_exclusive<kThreads>(full, sh.scan[1], total_f);
    const uint32_t extra = sh.pre[0] + excl;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_extra_dev = sh.pre[0] + total;
    const uint32_t base = (uint32_t)num_tiles + extra;
    // dispatch positions: full chunks in tile order from 0, the partial one
    // (at most one per tile) after the earlier partials of its class
    const uint32_t full_before = sh.pre[1] + excl_f;
    uint32_t part_pos = 0;
    if (pc != 0) {
        part_pos = sh.base[pc] + sh.pre[1 + pc] + rank;
        for (int i = 0; i < w; ++i) part_pos += sh.cls[pc][i];
    }
    // chunk j of this tile: descriptor, dispatch position, published maxima
    auto emit = [&](uint32_t tt, uint32_t rx, uint32_t ry, uint32_t c, uint32_t f, uint32_t bs, uint32_t fb,
                    uint32_t pp, uint32_t j) {
        const uint32_t b = rx + j * chunk;
        const uint32_t e = min(ry, b + chunk);
        const uint32_t slot = j == 0 ? tt : bs + j - 1;
        desc[slot] = make_uint4(tt, b, e, (c << 16) | j);
        // first-major: chunk j >= 1 goes after every first chunk, in slot order
        order[first_major && j > 0 ? slot : (j < f ? fb + j : pp)] = slot;
        if (tmax && c > 1) tmax[slot] = make_float4(1.f, 1.f, 1.f, 1.f);  // nothing composited yet
    };
    if (valid) {
        chunk_cnt[t] = cnt;
        chunk_base[t] = base;
        emit((uint32_t)t, r.x, r.y, cnt, full, base, full_before, part_pos, 0u);
    }
    // chunks j >= 1 of the multi-chunk tiles, flattened over the block: extra
    // chunk e of the block belongs to the tile whose inclusive count first
    // exceeds e (a binary search in LDS), so every thread stores about the
    // same number.  (Round 4's form, each wave walking its multi-chunk tiles
    // one at a time, ran ~40 serial steps per wave with only 128 waves at C2.)
    sh.incl[threadIdx.x] = excl + mine;
    {
        uint32_t* tp = sh.tile[threadIdx.x];
        tp[0] = (uint32_t)t; tp[1] = r.x; tp[2] = r.y; tp[3] = cnt;
        tp[4] = full; tp[5] = base; tp[6] = full_before; tp[7] = part_pos;
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < total; e += kThreads) {
        uint32_t lo = 0, hi = kThreads - 1;  // the first i with incl[i] > e (incl[kThreads - 1] = total > e)
#pragma unroll
        for (int step = 0; step < 8; ++step) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sh.incl[mid] > e) hi = mid; else lo = mid + 1;
        }
        const uint32_t* tp = sh.tile[lo];
        const uint32_t c = tp[3];
        const uint32_t j = e - (sh.incl[lo] - (c - 1u)) + 1u;
        emit(tp[0], tp[1], tp[2], c, tp[4], tp[5], tp[6], tp[7], j);
    }
}

__global__ __launch_bounds__(kThreads) void k_chunk_write(const uint2* __restrict__ ranges, int num_tiles,
                                                          uint32_t chunk, uint32_t classes,
                                                          const uint32_t* __restrict__ tot,
                                                          uint32_t* __restrict__ chunk_cnt,
                                                          uint32_t* __restrict__ chunk_base,
                                                          uint32_t* __restrict__ n_extra_dev,
                                                          uint4* __restrict__ desc, uint32_t* __restrict__ order,
                                                          float4* __restrict__ tmax, uint32_t first_major) {
    __shared__ ChunkWriteLds sh;
    chunk_write(ranges, num_tiles, chunk, classes, first_major != 0, tot, chunk_cnt, chunk_base, n_extra_dev, desc,
                order, tmax, sh);
}

// The chunk descriptors of a frame of at most kCsMaxTiles tiles and
// kCsMaxExtra extra chunks in ONE block (k_chunk_single): the count launch's
// block totals and the write launch's prefix sums become one block's scans,
// saving a launch and the totals' round trip through global memory (round 6,
// 16.8 us of k_chunk_count_long + k_chunk_write at C2).  Same
// descriptors, slots, dispatch order and class totals as chunk_count +
// chunk_write.  Thread t takes tiles [t T, t T + T); the extra chunks
// (j >= 1) are emitted flattened over the block: owner[e] = the tile of extra
// chunk e, filled by a prefix max over the tiles' first extra chunks.  The
// coarse order's long runs ride along as blocks 1.. (long_runs.h).
constexpr int kCsThreads = 1024;
constexpr int kCsWaves = kCsThreads / 64;
constexpr uint32_t kCsMaxTiles = 8192;    // 1080p: 8160
constexpr uint32_t kCsMaxExtra = 16384;   // extra chunks (fb, pp, excl in 16 bits: < 2^16 with the tiles)
static_assert(kCsMaxTiles + kCsMaxExtra < 65536u, "16-bit prefixes");
constexpr int kCsPer = (int)(kCsMaxTiles / kCsThreads);  // tiles per thread
constexpr int kCsClasses = 8;                            // length classes it handles (the default; more: two launches)
constexpr int kCsVals = 1 + kCsClasses;                  // scanned per thread: extra, full, partials of each class

struct ChunkSingleLds {
    uint2 info[kCsMaxTiles];            // per tile: its range, then excl extra | full before << 16, partial position
    uint16_t owner[kCsMaxExtra];        // extra chunk -> its tile (after the prefix max)
    uint32_t red[kCsVals][kCsWaves];    // per-wave sums of the scanned values
    uint32_t seg[kCsWaves];             // per-wave maxima of the owner segments
};
union ChunkSingleShared {
    ChunkSingleLds c;
    TdsLds t;
};

// chunks_of, first_full_of and first_class_of of one tile with two divisions
// (the single block keeps each tile's three terms in registers between its
// counting and its emission)
__device__ __forceinline__ void tile_chunk_terms(uint2 r, uint32_t chunk, uint32_t classes, bool first_major,
                                                 uint32_t& cnt, uint32_t& f, uint32_t& pc) {
    const uint32_t len = r.y - r.x;
    const uint32_t q = len / chunk, rem = len - q * chunk;
    cnt = len == 0 ? 1u : q + (rem != 0u ? 1u : 0u);
    f = first_major ? (len >= chunk ? 1u : 0u) : q;
    pc = (len != 0 && rem == 0) ? 0u : (classes - 1u) - rem * (classes - 1u) / chunk;
    if (first_major && len >= chunk) pc = 0u;
}

__device__ __forceinline__ void chunk_single(const uint2* __restrict__ ranges, int num_tiles, uint32_t chunk,
                                            uint32_t classes, bool first_major, uint32_t* __restrict__ chunk_cnt,
                                            uint32_t* __restrict__ chunk_base, uint32_t* __restrict__ n_extra_dev,
                                            uint4* __restrict__ desc, uint32_t* __restrict__ order,
                                            float4* __restrict__ tmax, uint32_t* __restrict__ cls_tot,
                                            ChunkSingleLds& sh) {
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = __lane_id();
    const uint32_t nt = (uint32_t)num_tiles;
    const uint32_t per = (nt + kCsThreads - 1) / kCsThreads;
    const uint32_t t0 = tid * per;
    // the ranges, loaded coalesced into LDS (info[] holds them until each thread has read its own tiles)
    for (uint32_t t = tid; t < nt; t += kCsThreads) sh.info[t] = ranges[t];
    __syncthreads();
    uint32_t v[kCsVals];
    uint32_t tc[kCsPer], tfp[kCsPer];  // per tile: chunks; full | partial class << 24
#pragma unroll
    for (int k = 0; k < kCsVals; ++k) v[k] = 0u;
#pragma unroll
    for (int i = 0; i < kCsPer; ++i) {
        tc[i] = 0u;
        tfp[i] = 0u;
        if ((uint32_t)i < per && t0 + i < nt) {
            uint32_t cnt, f, pc;
            tile_chunk_terms(sh.info[t0 + i], chunk, classes, first_major, cnt, f, pc);
            tc[i] = cnt;
            tfp[i] = f | (pc << 24);
            v[0] += cnt - 1u;
            v[1] += f;
#pragma unroll
            for (int k = 1; k < kCsClasses; ++k) v[1 + k] += (pc == (uint32_t)k) ? 1u : 0u;
        }
    }
    // one block scan of every value: exclusive prefixes in v, totals in tot
    uint32_t tot[kCsVals];
#pragma unroll
    for (int k = 0; k < kCsVals; ++k) {
        const uint32_t inc = wave_inclusive_scan(v[k]);
        if (lane == 63) sh.red[k][w] = inc;
        v[k] = inc - v[k];
    }
    __syncthreads();
    // lane q < kCsWaves holds wave q's sum; a wave scan over those lanes gives the waves before w
#pragma unroll
    for (int k = 0; k < kCsVals; ++k) {
        const uint32_t x = lane < (uint32_t)kCsWaves ? sh.red[k][lane] : 0u;
        const uint32_t inc = wave_inclusive_scan(x);
        const uint32_t before = w > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)inc, (int)w - 1) : 0u;
        v[k] += before;
        tot[k] = (uint32_t)__builtin_amdgcn_readlane((int)inc, kCsWaves - 1);
    }
    // class bases (first dispatch position of each class): full chunks, then the partial classes in order
    uint32_t base[kCsClasses];
    {
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < kCsClasses; ++k) {
            base[k] = run;
            run += (uint32_t)k < classes ? tot[1 + k] : 0u;  // (base[0] = 0: tot[1] full chunks, then class 1 ...)
        }
    }
    const uint32_t E = tot[0];
    if (tid == 0) {
        *n_extra_dev = E;
#pragma unroll
        for (int k = 0; k < kCsClasses; ++k)  // (unrolled: a runtime index would put tot in scratch)
            if ((uint32_t)k < classes) cls_tot[k] = tot[1 + k];
        cls_tot[classes] = E;  // the later chunks (first-major order)
    }
    for (uint32_t e = tid; e < E; e += kCsThreads) sh.owner[e] = 0;
    __syncthreads();  // (owner cleared before any tile marks its first extra chunk)
    // each tile's prefixes (over its own tiles, in order) into info[], its first extra chunk's owner mark
    uint32_t ex = v[0], fu = v[1];
#pragma unroll
    for (int i = 0; i < kCsPer; ++i) {
        const uint32_t t = t0 + (uint32_t)i;
        if ((uint32_t)i < per && t < nt) {
            const uint32_t cnt = tc[i], f = tfp[i] & 0xffffffu, pc = tfp[i] >> 24;
            uint32_t pp = 0;
#pragma unroll
            for (int k = 1; k < kCsClasses; ++k)
                if (pc == (uint32_t)k) {
                    pp = base[k] + v[1 + k];
                    v[1 + k] += 1u;
                }
            sh.info[t] = make_uint2(ex | (fu << 16), pp);  // (this thread's own tiles: read above)
            if (cnt > 1) sh.owner[ex] = (uint16_t)t;
            ex += cnt - 1u;
            fu += f;
        }
    }
    __syncthreads();
    // owner[e] = the last marked tile at or before e (tiles mark in increasing order): a prefix max,
    // each thread over a contiguous segment
    const uint32_t sp = (E + kCsThreads - 1) / kCsThreads;
    const uint32_t e0 = min(E, tid * sp), e1 = min(E, e0 + sp);
    uint32_t m = 0;
    for (uint32_t e = e0; e < e1; ++e) m = max(m, (uint32_t)sh.owner[e]);
    const uint32_t wm = wave_reduce_max(m);  // (a wave's segments are consecutive)
    uint32_t incl_m = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl_m, o, 64);
        if (lane >= (uint32_t)o) incl_m = max(incl_m, x);
    }
    if (lane == 63) sh.seg[w] = wm;
    __syncthreads();
    uint32_t run = __shfl_up(incl_m, 1, 64);
    if (lane == 0) run = 0;
    for (uint32_t q = 0; q < w; ++q) run = max(run, sh.seg[q]);
    for (uint32_t e = e0; e < e1; ++e) {
        run = max(run, (uint32_t)sh.owner[e]);
        sh.owner[e] = (uint16_t)run;
    }
    __syncthreads();
    auto emit = [&](uint32_t tt, uint2 rr, uint32_t c, uint32_t f, uint32_t slot, uint32_t fb, uint32_t pp, uint32_t j) {
        const uint32_t b = rr.x + j * chunk;
        desc[slot] = make_uint4(tt, b, min(rr.y, b + chunk), (c << 16) | j);
        order[first_major && j > 0 ? slot : (j < f ? fb + j : pp)] = slot;
        if (tmax && c > 1) tmax[slot] = make_float4(1.f, 1.f, 1.f, 1.f);  // nothing composited yet
    };
    // chunk 0 of every tile, then the extra chunks: consecutive lanes write consecutive tiles and slots
    // (the stores of a thread's own contiguous tiles touched a line per lane: 29 us against 17 for the
    // two launches)
    for (uint32_t t = tid; t < nt; t += kCsThreads) {
        const uint2 rr = ranges[t];
        const uint2 in = sh.info[t];
        uint32_t cnt, f, pc;
        tile_chunk_terms(rr, chunk, classes, first_major, cnt, f, pc);
        chunk_cnt[t] = cnt;
        chunk_base[t] = nt + (in.x & 0xffffu);
        emit(t, rr, cnt, f, t, in.x >> 16, in.y, 0u);
    }
    for (uint32_t e = tid; e < E; e += kCsThreads) {
        const uint32_t t = sh.owner[e];
        const uint2 in = sh.info[t];
        const uint2 rr = ranges[t];
        uint32_t cnt, f, pc;
        tile_chunk_terms(rr, chunk, classes, first_major, cnt, f, pc);
        emit(t, rr, cnt, f, nt + e, in.x >> 16, in.y, e - (in.x & 0xffffu) + 1u);
    }
}

__global__ __launch_bounds__(kCsThreads) void k_chunk_single(const uint2* __restrict__ ranges, int num_tiles,
                                                             uint32_t chunk, uint32_t classes, uint32_t first_major,
                                                             uint32_t* __restrict__ chunk_cnt,
                                                             uint32_t* __restrict__ chunk_base,
                                                             uint32_t* __restrict__ n_extra_dev,
                                                             uint4* __restrict__ desc, uint32_t* __restrict__ order,
                                                             float4* __restrict__ tmax, uint32_t* __restrict__ cls_tot,
                                                             LongRunArgs la) {
    __shared__ ChunkSingleShared S;
    if (blockIdx.x == 0)
        chunk_single(ranges, num_tiles, chunk, classes, first_major != 0, chunk_cnt, chunk_base, n_extra_dev, desc,
                     order, tmax, cls_tot, S.c);
    else
        long_runs_block(la, S.t, blockIdx.x - 1, gridDim.x - 1);
}

struct ChunkView {
    const uint2* ranges;
    uint32_t* chunk_cnt;  // block totals after its num_tiles entries
    uint32_t* chunk_base;
    uint32_t* n_extra_dev;
    uint4* desc;
    uint32_t* order;
    float4* tmax;
};
struct ChunkViews {
    ChunkView v[kMaxViews];
};

__global__ __launch_bounds__(kThreads) void k_chunk_count_views(ChunkViews vs, int num_tiles, uint32_t chunk,
                                                                uint32_t classes, uint32_t first_major) {
    __shared__ uint32_t lds[1 + kMaxLenClasses][kThreads / 64];
    const ChunkView& v = vs.v[blockIdx.y];
    chunk_count(v.ranges, num_tiles, chunk, classes, first_major != 0, v.chunk_cnt + num_tiles, lds, blockIdx.x,
                gridDim.x, threadIdx.x);
}

__global__ __launch_bounds__(kThreads) void k_chunk_write_views(ChunkViews vs, int num_tiles, uint32_t chunk,
                                                                uint32_t classes, uint32_t first_major) {
    __shared__ ChunkWriteLds sh;
    const ChunkView& v = vs.v[blockIdx.y];
    chunk_write(v.ranges, num_tiles, chunk, classes, first_major != 0, v.chunk_cnt + num_tiles, v.chunk_cnt,
                v.chunk_base, v.n_extra_dev, v.desc, v.order, v.tmax, sh);
}

// Bits [lo, hi] of a 16-bit mask, clamped to [0, 15]; 0 if the range is empty.
__device__ __forceinline__ uint32_t span_bits16(int lo, int hi) {
    lo = max(lo, 0);
    hi = min(hi, 15);
    return hi >= lo ? ((2u << hi) - (1u << lo)) : 0u;
}

__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The current value of a word other workgroups update by agent-scope atomics,
// read by an atomic (max with 0 changes nothing), which is performed at the
// coherence point.  An agent-scope load is served by this XCD's L2, which may
// still hold the line from an earlier load in the same launch (the other
// chunks' saturation polls), so a fold deciding which chunks count must not
// use one.
__device__ __forceinline__ uint32_t ld_atomic(uint32_t* p) {
    return __hip_atomic_fetch_max(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// readfirstlane of a float's bits (the builtin takes int: a float argument
// would be value-converted)
__device__ __forceinline__ float uniform_f(float v) {
    return __uint_as_float((uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(v)));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ float wave_prod(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v *= __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ const uint32_t* chunk_tmax(const float4* tmax, uint32_t tile, uint32_t base, uint32_t j) {
    return reinterpret_cast<const uint32_t*>(tmax + (j == 0 ? tile : base + j - 1));
}

// Issue (no wait) the loads of the published slice maxima of chunks
// 0..min(kk,64)-1, one chunk per lane; other lanes hold 1.0.
// The cross-chunk bound for a group's frames: an experiment build only
// (-DGSR_COMP_BOUND, profiles/r2_s53: slower in flight).  A frame alone takes
// it per frame (launch_composite's tmax, api.hip frame_chunk).
#ifdef GSR_COMP_BOUND
constexpr bool kBoundViews = true;
#else
constexpr bool kBoundViews = false;
#endif

__device__ __forceinline__ void load_prior(const float4* tmax, uint32_t tile, uint32_t base, uint32_t kk,
                                           uint32_t prior[4]) {
    const uint32_t j = __lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k) prior[k] = 0x3f800000u;
    if (j < kk) {
        const uint32_t* w = chunk_tmax(tmax, tile, base, j);
#pragma unroll
        for (int k = 0; k < 4; ++k) prior[k] = ld_relaxed(w + k);
    }
}

// B[k] = product over chunks j < min(kk, 64) of their published maxima of
// slice k: an upper bound of the transmittance entering chunk kk (the factors
// of chunks 64 .. kk - 1 are at most 1; reading them synchronously every batch
// cost the deepest tiles more than the tighter bound saved, profiles/r5_s19).
__device__ __forceinline__ void prior_bound(const float4* tmax, uint32_t tile, uint32_t base, uint32_t kk,
                                            const uint32_t prior[4], float B[4]) {
    (void)tmax, (void)tile, (void)base, (void)kk;
#pragma unroll
    for (int k = 0; k < 4; ++k) B[k] = uniform_f(wave_prod(__uint_as_float(prior[k])));
}

// The image is written non-temporally: nothing in the frame reads it back, and
// default-policy stores kept its lines in the L2s and the MALL over the
// records and lists the other chunks (and, in flight, other views) still
// gather (20 views in flight: 0.1323-0.1334 -> 0.1308-0.1321 ms per frame on
// one box, profiles/r5_s51; within the spread on another, r5_s52).  The tile
// lists read non-temporally too: no change (r5_s52).
__device__ __forceinline__ void st_out(float* p, float v) { __builtin_nontemporal_store(v, p); }

#ifdef GSR_COMP_STATS
// Tooling build only (tools/comp_stats.py): {slice evaluations, evaluations
// of an already saturated slice, records visited, records in the chunks}.
__device__ unsigned long long g_comp_stats[5];
#endif

// One wave per chunk, 4 pixels per lane (four 16x4 slices of the 16x16 tile).
// Records of the chunk are gathered 64 at a time (one 48-B record per lane,
// prefetched one batch ahead in registers) into a wave-private LDS buffer and
// then read back with wave-uniform (broadcast) ds_read_b128.  No workgroup
// barriers: the four waves of a block are independent chunks.
//
// Early termination across the chunks of a tile (multi-chunk tiles only).
// After every batch a chunk publishes, per 16x4 slice, the maximum over its 64
// pixels of its LOCAL transmittance: tmax[slot].s (1.0 until first written;
// it only decreases).  Chunk kk bounds the ABSOLUTE transmittance entering it
// by B = prod_{j<kk} tmax[chunk j] (published values are upper bounds of the
// final local ones, unstarted chunks count 1) and stops a slice once
// B * (its own local max) < t_min: everything behind that point, in this and
// all later chunks, contributes less than t_min -- the bound of sequential
// front-to-back early termination, reached while the chunks run in parallel.
// A later chunk's bound then falls below t_min too, so it skips the slice.
// Saturation words sat[tile*4 + slice] hold ~(smallest stopping chunk index)
// (atomicMax of the complement; zero = none): k_merge folds each slice only up
// to that chunk.  All words are accessed relaxed at agent scope; a stale read
// only costs work, never accuracy.
// Wave priority by remaining work (experiment, GSR_COMP_PRIO: bit 0 a frame
// alone's launch, bit 1 a group's): at each batch the wave sets its priority to
// min(3, batches left), so on a SIMD the waves with the most work left issue
// first instead of the oldest (the SIMD's default arbitration, priority then
// age: the youngest of 8 resident waves barely advanced until the older ones
// retired, then ran alone at the launch's end, profiles/r6_s18).
#ifndef GSR_COMP_PRIO
#define GSR_COMP_PRIO 0
#endif
#ifndef GSR_COMP_PRIO_MODE
#define GSR_COMP_PRIO_MODE 0  // 0: batches left; 1: batches done (least progress first)
#endif
__device__ __forceinline__ void batch_priority(uint32_t begin, uint32_t b, uint32_t end) {
    const uint32_t left = (uint32_t)__builtin_amdgcn_readfirstlane((int)((end - b + kBatch - 1) / kBatch));
    const uint32_t done = (uint32_t)__builtin_amdgcn_readfirstlane((int)((b - begin) / kBatch));
    const uint32_t p = GSR_COMP_PRIO_MODE == 0 ? min(left, 3u) : 3u - min(done, 3u);
    if (p >= 3) __builtin_amdgcn_s_setprio(3);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else if (p == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

template <int FRAG, bool kBound, bool kPrio = false>
__device__ __forceinline__ void composite_chunk(const uint4 d, const uint32_t slot, float4* __restrict__ my,
                                                const uint32_t* __restrict__ list,
                                                const SplatRec* __restrict__ recs, const CompositeArgs& a,
                                                float* __restrict__ out, float4* __restrict__ partial,
                                                uint32_t* __restrict__ sat, float4* __restrict__ tmax,
                                                const uint32_t* __restrict__ chunk_base,
                                                uint32_t* __restrict__ trace_evals = nullptr) {
    const int tile = (int)d.x;
    const uint32_t begin = d.y, end = d.z;
    const uint32_t nchunks = d.w >> 16;
    const uint32_t kk = d.w & 0xffffu;
    const int lane = __lane_id();
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int lcol = lane & 15;
    const int col_base = tx * kTile;
    const int x = col_base + lcol;
    const int row_base = ty * kTile;
    const int lrow = lane >> 4;
    const float px = (float)x + 0.5f;
    float pyw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) pyw[k] = (float)(a.height - 1 - (row_base + 4 * k + lrow)) + 0.5f;

    // per slice: (r, g) and (b, T), updated with packed FMAs (v_pk_fma_f32:
    // one issue slot for two channels)
    f32x2 rg[4], bt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rg[k] = f32x2{0.f, 0.f};
        bt[k] = f32x2{0.f, 1.f};
    }
    // transmittance coefficient of the packed (b, T) update: T -= 0.99 w in
    // interval form (the 0.99 of the alpha), T -= w otherwise
    const float kT = FRAG == kFragGauss ? -0.99f : -1.0f;
    const float t_min = a.t_min;
    const bool track = (nchunks > 1) && (t_min > 0.f);
    uint32_t* my_sat = sat + (size_t)tile * 4;
    [[maybe_unused]] uint32_t* my_tmax = reinterpret_cast<uint32_t*>(tmax + slot);
    // slots of the earlier chunks: chunk 0 at `tile`, chunk j >= 1 at base + j - 1
    [[maybe_unused]] const uint32_t base = slot - kk + 1;
    const bool poll = track && kk > 0;
    // live slices (bit k): not yet stopped
    uint32_t live = 0xfu;
    [[maybe_unused]] uint32_t prior[4];  // (kBound) lane i < min(kk, 64): chunk i's published slice maxima (async)
    if constexpr (kBound) {
        if (poll) load_prior(tmax, (uint32_t)tile, base, kk, prior);
    }

    // Two-stage prefetch: the records of batch b+1 and the list indices of
    // batch b+2 are in flight while batch b is composited, so neither the
    // index load nor the dependent record gather is ever waited on directly.
    float4 f0, f1, f2;
    uint32_t idx_next = 0;
    if (live) {
        const uint32_t i = begin + lane;
        if (i < end) {
            const float4* r = reinterpret_cast<const float4*>(recs + list[i]);
            f0 = r[0]; f1 = r[1]; f2 = r[2];
        }
        const uint32_t i2 = begin + kBatch + lane;
        if (i2 < end) idx_next = list[i2];
    }
    if (kBound && poll) {  // a chunk that starts behind saturated ones computes nothing
        float B[4];
        prior_bound(tmax, (uint32_t)tile, base, kk, prior, B);
        uint32_t dead = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (B[k] < t_min) dead |= 1u << k;
        dead = __builtin_amdgcn_readfirstlane(dead);
        if (dead && lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (dead & (1u << k)) atomicMax(my_sat + k, 0xffffffffu - kk);
        }
        live &= ~dead;
    }
    if (!kBound && poll) {  // slices an earlier chunk already saturated
        uint32_t dead = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (0xffffffffu - ld_relaxed(my_sat + k) < kk) dead |= 1u << k;
        live &= ~__builtin_amdgcn_readfirstlane(dead);
    }
    if (a.debug_handoff && nchunks > 1 && kk == 0) {
        // Test knob (tests/test_gpu_handoff.py), chunk 0 of a multi-chunk tile,
        // before any other chunk can have finished: bit 1 polls the tile's
        // saturation words (agent-scope loads, as the later chunks' polls do),
        // bit 2 plain-loads the other chunks' partial slots, so this XCD's L2
        // holds those lines with their old contents when chunk 0 folds.
        float junk = 0.f;
        if (a.debug_handoff & 2u) {
#pragma unroll
            for (int k = 0; k < 4; ++k) junk += __uint_as_float(ld_relaxed(my_sat + k));
        }
        if (a.debug_handoff & 4u) {
            const uint32_t cb = chunk_base[tile];
            for (uint32_t c = 1; c < nchunks; ++c) {
                const float4* q = partial + (size_t)(cb + c - 1) * 256;
#pragma unroll
                for (int k = 0; k < 4; ++k) junk += q[k * 64 + lane].w;
            }
        }
        asm volatile("" ::"v"(junk));
    }
#ifdef GSR_COMP_STATS
    uint32_t st_evals = 0, st_wasted = 0, st_records = 0, st_empty = 0;
#endif
#ifdef GSR_COMP_TRACE
    uint32_t tr_evals = 0;  // (record, slice) evaluations of this chunk (tools/comp_trace.py)
#endif
    for (uint32_t b = begin; b < end && live; b += kBatch) {
        if constexpr (kPrio) batch_priority(begin, b, end);
        __builtin_amdgcn_wave_barrier();
        // sb[k] bit j: record j of the batch touches 16x4 slice k (and the
        // slice is live): one ballot per slice and batch instead of a
        // readfirstlane of a slice mask per record
        uint64_t sb[4];
        {
            // Tile-relative coverage of this lane's record, computed once per
            // record (not per pixel): .w of q0 = 16-bit column mask | 16-bit
            // row mask << 16.
            const uint32_t xs = __float_as_uint(f0.w), ys = __float_as_uint(f1.w);
            const uint32_t covx = span_bits16((int)(xs & 0xffffu) - col_base, (int)(xs >> 16) - col_base);
            const uint32_t covy = span_bits16((int)(ys & 0xffffu) - row_base, (int)(ys >> 16) - row_base);
            // LDS record: (cx, cy, opacity, coverage), (qa, qb, qc, mid), (r, g, b, T coefficient)
            my[lane * 3 + 0] = make_float4(f0.x, f0.y, f0.z, __uint_as_float(covx | (covy << 16)));
            my[lane * 3 + 1] = make_float4(f1.x, f1.y, f1.z, f2.w);
            my[lane * 3 + 2] = make_float4(f2.x, f2.y, f2.z, kT);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                sb[k] = ((live >> k) & 1u) ? (uint64_t)__ballot(((covy >> (4 * k)) & 0xfu) != 0u) : 0ull;
        }
        __builtin_amdgcn_wave_barrier();
        // earlier chunks' published maxima (kBound), or the saturation words of
        // the other chunks, consumed after this batch
        [[maybe_unused]] uint32_t satw[4];
        if (kBound && poll) load_prior(tmax, (uint32_t)tile, base, kk, prior);
        if (!kBound && poll) {
#pragma unroll
            for (int k = 0; k < 4; ++k) satw[k] = ld_relaxed(my_sat + k);
        }
        {  // prefetch: records of batch b+1, list indices of batch b+2
            const uint32_t i = b + kBatch + lane;
            if (i < end) {
                const float4* r = reinterpret_cast<const float4*>(recs + idx_next);
                f0 = r[0]; f1 = r[1]; f2 = r[2];
            }
            const uint32_t i2 = b + 2 * kBatch + lane;
            if (i2 < end) idx_next = list[i2];
        }
        const int nb = __builtin_amdgcn_readfirstlane((int)min((uint32_t)kBatch, end - b));
        // records touching a live slice only (sb: live slices only): once a
        // slice has stopped, records covering nothing else skip their setup
        // (not unrolled: unrolled by 2, the register allocator copies every
        // packed accumulator at each slice branch and needs 128 VGPRs)
        // Bottom-tested, the record's bit cleared by one s_andn2_b64 with the
        // 1 << j the slice tests use: 3 fewer scalar instructions per record
        // than a top-tested loop clearing the lowest bit (the loop is co-bound
        // by VALU and SALU issue: profiles/r4_s16)
        uint64_t todo = (sb[0] | sb[1] | sb[2] | sb[3]) & (nb >= 64 ? ~0ull : ((1ull << nb) - 1ull));
        if (todo) {
#if GSR_COMP_PIPE
        // experiment: the next record's three broadcast reads issued before this
        // record's arithmetic, so they are not waited on one record at a time (+12 VGPRs)
        int j = (int)__builtin_ctzll(todo);
        float4 n0 = my[j * 3 + 0], n1 = my[j * 3 + 1], n2 = my[j * 3 + 2];
#endif
#pragma unroll 1
        do {
#if GSR_COMP_PIPE
            const float4 q0 = n0, q1 = n1, q2 = n2;
            todo &= ~(1ull << j);
            const int jn = todo ? (int)__builtin_ctzll(todo) : j;
            n0 = my[jn * 3 + 0];
            n1 = my[jn * 3 + 1];
            n2 = my[jn * 3 + 2];
#else
            const int j = (int)__builtin_ctzll(todo);
            todo &= ~(1ull << j);
            const float4 q0 = my[j * 3 + 0];  // cx cy opacity coverage
            const float4 q1 = my[j * 3 + 1];  // qa qb qc mid
            const float4 q2 = my[j * 3 + 2];  // r g b kT
#endif
#ifdef GSR_COMP_STATS
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((sb[k] >> j) & 1ull) {
                    st_evals += 1;
                    if (!__any(bt[k].y >= t_min)) st_wasted += 1;
                }
            st_records += 1;
#endif
#ifdef GSR_COMP_TRACE
#pragma unroll
            for (int k = 0; k < 4; ++k) tr_evals += (uint32_t)((sb[k] >> j) & 1ull);
#endif
#ifdef GSR_COMP_DENSE
            if (FRAG == kFragGauss) {
                // Dense evaluation (an experiment build, profiles/r3_s13): the
                // record's covered pixels of the tile are packed onto the wave's
                // lanes, one evaluation per 64 of them instead of one 64-lane
                // evaluation per touched 16x4 slice, and each alpha is handed to
                // the lane that owns its pixel by ds_bpermute.  The falloff, keep
                // test and blend are the expressions below, so the alphas and
                // the image are the same bit for bit.  The record's rectangle
                // terms are wave-uniform (scalar registers).
                const uint32_t cov = (uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(q0.w));
                const uint32_t covx = cov & 0xffffu, covy = cov >> 16;
                const int x0 = (int)__builtin_ctz(covx), x1 = 31 - (int)__builtin_clz(covx);
                const int y0 = (int)__builtin_ctz(covy), y1 = 31 - (int)__builtin_clz(covy);
                const int rw = x1 - x0 + 1, rh = y1 - y0 + 1;
                const int cnt = rw * rh;
                const float inv_w = __builtin_amdgcn_rcpf((float)rw);
                const float mid = q1.w;
                const float km = -mid * kKeepScaleWide;
                const f32x2 c_rg = f32x2{q2.x, q2.y};
                const f32x2 c_bt = f32x2{q2.z, q2.w};
                // this lane's pixel of slice k sits at rect index lidx + (4k - y0) rw (if covered)
                const uint32_t cc = (uint32_t)(lcol - x0);
                const bool col_in = cc < (uint32_t)rw;
                const int lidx = lrow * rw + (int)cc;
                const float pxe0 = (float)(col_base + x0) + 0.5f;
                const float pye0 = (float)(a.height - 1 - (row_base + y0)) + 0.5f;
                for (int e0 = 0; e0 < cnt; e0 += 64) {
                    const int qq = e0 + lane;
                    const int row = (int)(((float)qq + 0.5f) * inv_w);  // exact: qq < 256, rw <= 16
                    const int col = qq - row * rw;
                    const float dx = (pxe0 + (float)col) - q0.x;
                    const float p0 = fmaf(q1.x * dx, dx, -mid);
                    const float p1 = q1.y * dx;
                    const float dy = (pye0 - (float)row) - q0.y;
                    const float pw = (q1.z * dy + p1) * dy + p0;
                    const float ee = __builtin_amdgcn_exp2f(pw);
                    const float a1 = __builtin_amdgcn_fmed3f(q0.z * ee, 0.f, 1.f);
                    const float al = __builtin_amdgcn_fmed3f(fmaf(-kKeepScale, fabsf(pw), km), 0.f, a1);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (!((sb[k] >> j) & 1ull)) continue;
                        const int rk = 4 * k - y0;                       // uniform
                        const uint32_t r = (uint32_t)(lrow + rk);        // row within the rect
                        const uint32_t src = (uint32_t)(lidx + rk * rw - e0);
                        const bool mine = col_in & (r < (uint32_t)rh) & (src < 64u);
                        const float ak =
                            __int_as_float(__builtin_amdgcn_ds_bpermute((int)(src << 2), __float_as_int(al)));
                        const float wgt = (mine ? ak : 0.f) * bt[k].y;
                        const f32x2 ww = f32x2{wgt, wgt};
                        rg[k] = __builtin_elementwise_fma(c_rg, ww, rg[k]);
                        bt[k] = __builtin_elementwise_fma(c_bt, ww, bt[k]);
                    }
                }
                continue;
            }
#endif
            // lane coverage: bit 4k = this lane's pixel of slice k is inside the splat's quad
            // (all-zero when the column is not: bfe_i32 gives 0 or ~0)
            const uint32_t cov = __float_as_uint(q0.w);
            const uint32_t rb = (cov >> (16 + lrow)) & (uint32_t)__builtin_amdgcn_sbfe((int)cov, lcol, 1);
            // power*log2(e) = qa dx^2 + qb dx dy + qc dy^2 in pixel units
            // (gau_frag.glsl:37 with coordxy's scale folded in by the preprocess)
            const float dx = px - q0.x;
            // kFragGauss: q1.w = mid, and p0 is shifted by it (interval form, SplatRec)
            const float mid = FRAG == kFragGauss ? q1.w : 0.f;
            const float p0 = FRAG == kFragGauss ? fmaf(q1.x * dx, dx, -mid) : q1.x * dx * dx;
            const float p1 = q1.y * dx;
            const float c2 = q1.z;
            // K m (1 + 2^-22) of the keep test (kKeepScale)
            const float km = FRAG == kFragGauss ? -mid * kKeepScaleWide : 0.f;
            const f32x2 c_rg = f32x2{q2.x, q2.y};
            const f32x2 c_bt = f32x2{q2.z, q2.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!((sb[k] >> j) & 1ull)) continue;
                // opacity where the pixel is covered, +0 elsewhere (bit mask, no compare)
                const uint32_t covk = (uint32_t)__builtin_amdgcn_sbfe((int)rb, 4 * k, 1);
                float alpha;
                f32x2 crg = c_rg, cbt = c_bt;
                if (FRAG == kFragGauss) {
                    // pw' = pw - mid; keep <=> |pw'| <= -mid; alpha / 0.99 = clamp(s * 2^pw')
                    const float dy = pyw[k] - q0.y;
                    const float pw = (c2 * dy + p1) * dy + p0;
                    const float u = fmaf(-kKeepScale, fabsf(pw), km);  // >= 0 exactly where the fragment is kept
                    const float e = __builtin_amdgcn_exp2f(pw);
                    const float a1 = __builtin_amdgcn_fmed3f(__uint_as_float(covk & __float_as_uint(q0.z)) * e, 0.f, 1.f);
                    alpha = __builtin_amdgcn_fmed3f(u, 0.f, a1);
                } else if (FRAG == kFragBillboard) {
                    alpha = __uint_as_float(covk & 0x3f800000u);  // 1.0 or 0.0
                } else {
                    const float dy = pyw[k] - q0.y;
                    const float pw = (c2 * dy + p1) * dy + p0;  // power * log2(e)
                    const float e = __builtin_amdgcn_exp2f(pw);  // exp(power)
                    alpha = fminf(0.99f, __uint_as_float(covk & __float_as_uint(q0.z)) * e);
                    // discards: power > 0, alpha < 1/255
                    alpha = ((pw > 0.0f) | (alpha < (1.0f / 255.0f))) ? 0.0f : alpha;
                    if (FRAG == kFragFlatBall || FRAG == kFragGaussBall) alpha = (alpha > 0.22f) ? 1.0f : 0.0f;
                    if (FRAG == kFragGaussBall) {
                        crg = f32x2{fminf(fmaxf(q2.x * e, 0.f), 1.f), fminf(fmaxf(q2.y * e, 0.f), 1.f)};
                        cbt = f32x2{fminf(fmaxf(q2.z * e, 0.f), 1.f), q2.w};
                    }
                }
                // alpha == 0 leaves (C, T) bit-identical: a discarded fragment.
                // C += c w, T += kT w with w = alpha T (kFragGauss: alpha =
                // 0.99 a1, the colour already carries its 0.99)
#ifdef GSR_COMP_STATS
                if (!__any(alpha > 0.f)) st_empty += 1;  // no lane keeps a fragment of this slice
#endif
                const float w = alpha * bt[k].y;
                const f32x2 ww = f32x2{w, w};
                rg[k] = __builtin_elementwise_fma(crg, ww, rg[k]);
                bt[k] = __builtin_elementwise_fma(cbt, ww, bt[k]);
            }
#if GSR_COMP_PIPE
            j = jn;
#endif
        } while (todo);
        }
        if (t_min > 0.f) {
            uint32_t still = 0;
            if (kBound && track) {
                // publish this chunk's slice maxima, then test bound * max against t_min
                float m[4], B[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
                for (int k = 0; k < 4; ++k) m[k] = uniform_f(wave_max(bt[k].y));
                if (lane < 4) {
                    const float mine = lane == 0 ? m[0] : lane == 1 ? m[1] : lane == 2 ? m[2] : m[3];
                    __hip_atomic_store(my_tmax + lane, __float_as_uint(mine), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
                if (poll) prior_bound(tmax, (uint32_t)tile, base, kk, prior, B);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (B[k] * m[k] >= t_min) still |= 1u << k;
            } else {
                // stop a slice when every pixel's chunk-local T is below t_min
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (__any(bt[k].y >= t_min)) still |= 1u << k;
            }
            const uint32_t newly = live & ~still;
            if (track && newly && lane == 0) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (newly & (1u << k)) atomicMax(my_sat + k, 0xffffffffu - kk);
            }
            live &= still;
            if (!kBound && poll && live) {
                uint32_t dead = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (0xffffffffu - satw[k] < kk) dead |= 1u << k;
                live &= ~__builtin_amdgcn_readfirstlane(dead);
            }
        }
    }

#ifdef GSR_COMP_TRACE
    if (trace_evals) *trace_evals = tr_evals;
#endif
#ifdef GSR_COMP_STATS
    if (lane == 0) {
        atomicAdd(&g_comp_stats[0], (unsigned long long)st_evals);
        atomicAdd(&g_comp_stats[1], (unsigned long long)st_wasted);
        atomicAdd(&g_comp_stats[2], (unsigned long long)st_records);
        atomicAdd(&g_comp_stats[3], (unsigned long long)(end - begin));
        atomicAdd(&g_comp_stats[4], (unsigned long long)st_empty);
    }
#endif
    if (nchunks > 1) {
        // partial (C, T) per pixel, folded by k_merge or by the tile's last
        // chunk to finish (tail merge); layout [slot][k][lane]
        float4* p = partial + (size_t)slot * 256;
        if (!a.tail_merge) {
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k * 64 + lane] = make_float4(rg[k].x, rg[k].y, bt[k].x, bt[k].y);
            return;
        }
        // Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, hand-off
        // table row 1): the partials are stored `sc1` (16-B vector stores that
        // write through past the XCD's L2, so no release fence: an agent
        // release writes back the whole L2's dirty lines, and thousands of them
        // serialised the launch), the wave waits for them, then one
        // agent-scope add to the tile's counter (zeroed with the frame's other
        // zero words by the cull / preprocess).  The wave whose add returns
        // nchunks - 1 is the last: it reads every other chunk's partial with
        // `sc1` loads and folds the tile in chunk order.
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4 v = f32x4{rg[k].x, rg[k].y, bt[k].x, bt[k].y};
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + k * 64 + lane), "v"(v) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t old = 0;
        if ((a.debug_handoff & 1u) && kk == 0 && lane == 0) {
            // test knob: chunk 0 adds last (waits for the other chunks' adds; 0.2 s bound)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_atomic(sat + 4 * (size_t)a.num_tiles + tile) < nchunks - 1u &&
                   __builtin_amdgcn_s_memrealtime() - t0 < 20000000ull)
                __builtin_amdgcn_s_sleep(4);
        }
        if (lane == 0)
            old = __hip_atomic_fetch_add(sat + 4 * (size_t)a.num_tiles + tile, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        old = (uint32_t)__builtin_amdgcn_readlane((int)old, 0);
        if (old != nchunks - 1u) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t cbase = kk > 0 ? slot - kk + 1 : chunk_base[tile];  // slot of chunk c >= 1: cbase + c - 1
        // the slices' first saturating chunks, final now (every chunk's atomics
        // completed before its counter add), read coherently (ld_atomic)
        uint32_t satv = 0;
#ifdef GSR_TAIL_REVERT_SAT_ATOMIC  // verification build: the pre-8352f97 read (tests/test_gpu_handoff.py)
        if (lane < 4) satv = ld_relaxed(sat + (size_t)tile * 4 + lane);
#else
        if (lane < 4) satv = ld_atomic(sat + (size_t)tile * 4 + lane);
#endif
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // chunks past the first one to saturate the slice add < t_min: k_merge's bound
            const uint32_t last =
                min(nchunks - 1u, 0xffffffffu - (uint32_t)__builtin_amdgcn_readlane((int)satv, k));
            float r = 0.f, g = 0.f, b = 0.f, T = 1.f;
            for (uint32_t c0 = 0; c0 <= last; c0 += 4) {
                // other chunks' partials, stored `sc1` (write-through) by their
                // waves, are read with 16-B `sc1` loads (MI355X_MICROARCH.md,
                // inter-workgroup visibility, hand-off table row 1: sc1 stores,
                // last adder, sc1 loads).  Plain loads after the acquire can be
                // served by a stale line in this XCD's L2; they made a group's
                // images differ from run to run in a few pixels.  Slots this wave
                // does not need (past `last`, or its own chunk, in registers) load
                // its own partial instead, then are replaced.
                const float4* src[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = c0 + j;
                    const uint32_t cs = (c > last || c == kk) ? slot : c == 0 ? (uint32_t)tile : cbase + c - 1;
                    src[j] = partial + (size_t)cs * 256 + k * 64 + lane;
                }
                f32x4 u0, u1, u2, u3;
#ifdef GSR_TAIL_REVERT_SC1_LOADS  // verification build: the pre-f4e3b53 plain loads (tests/test_gpu_handoff.py)
                u0 = *reinterpret_cast<const f32x4*>(src[0]);
                u1 = *reinterpret_cast<const f32x4*>(src[1]);
                u2 = *reinterpret_cast<const f32x4*>(src[2]);
                u3 = *reinterpret_cast<const f32x4*>(src[3]);
#else
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(u0) : "v"(src[0]) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(u1) : "v"(src[1]) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(u2) : "v"(src[2]) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(u3) : "v"(src[3]) : "memory");
                // the loads' results are read only after this wait (they are its operands)
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : : "memory");
#endif
                const f32x4 u[4] = {u0, u1, u2, u3};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t c = c0 + j;
                    if (c > last) continue;
                    const f32x4 v = c == kk ? f32x4{rg[k].x, rg[k].y, bt[k].x, bt[k].y} : u[j];
                    r += T * v[0];
                    g += T * v[1];
                    b += T * v[2];
                    T *= v[3];
                }
            }
            rg[k] = f32x2{r, g};
            bt[k] = f32x2{b, T};
        }
    }
    if (x >= a.width) return;
    const size_t plane = (size_t)a.width * a.height;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = row_base + 4 * k + lrow;
        if (row >= a.height) continue;
        const float T = bt[k].y;
        const float r = rg[k].x + T * a.bg[0];
        const float g = rg[k].y + T * a.bg[1];
        const float b = bt[k].x + T * a.bg[2];
        const size_t pidx = (size_t)row * a.width + x;
        if (a.out_layout == 0) {
            st_out(out + pidx, r);
            st_out(out + plane + pidx, g);
            st_out(out + 2 * plane + pidx, b);
        } else {
            st_out(out + 3 * pidx, r);
            st_out(out + 3 * pidx + 1, g);
            st_out(out + 3 * pidx + 2, b);
        }
    }
}

#ifdef GSR_COMP_TRACE
// Tooling build only (tools/comp_trace.py): per-wave shader-clock stamps.
__device__ uint4 g_comp_trace[2 * kTraceMax];
#endif

// 8 waves per SIMD: the compiler's own choice is 65 VGPRs (7 waves); held to
// 64 it spills one 8-byte value outside the record loop
#ifndef GSR_COMP_WPE
#define GSR_COMP_WPE 8
#endif
#define GSR_COMP_OCC __attribute__((amdgpu_waves_per_eu(GSR_COMP_WPE, 8)))
// compositing waves per block (each wave takes its own chunk; no block barrier)
#ifndef GSR_COMP_THREADS
#define GSR_COMP_THREADS 256
#endif
constexpr int kCompThreads = GSR_COMP_THREADS;
constexpr int kCompWaves = kCompThreads / 64;

// A frame alone's compositing (k_composite): blocks are dealt round-robin to
// the 8 XCDs; each XCD gets R = 8 consecutive logical blocks (32 consecutive
// chunks, mostly neighbouring tiles) per window of 64, and the dispatch order
// changes only within a window.  Measured (profiles/r4_s23, r4_s24): 120.2 ->
// 117.0 us per launch, HBM fetch -1 %; R = 16 or 32 the same.  A group's
// launch (k_composite_views) keeps the plain order: remapped it ran no faster
// in flight (its class-major, first-major order matters more there).
#ifndef GSR_COMP_XCD_RUN
#define GSR_COMP_XCD_RUN 8
#endif
__device__ __forceinline__ uint32_t comp_block() {
    const uint32_t b = blockIdx.x;
    if (GSR_COMP_XCD_RUN <= 1) return b;
    constexpr uint32_t R = GSR_COMP_XCD_RUN, W = 8u * R;
    const uint32_t w = b / W;
    if ((w + 1) * W > gridDim.x) return b;  // the last partial window keeps the plain order
    const uint32_t r = b - w * W;
    return w * W + (r & 7u) * R + (r >> 3);
}

// Experiment (GSR_COMP_PERSIST = resident blocks per CU, 0 = off): a frame
// alone's compositing as a resident grid whose waves take the dispatch order
// (longest chunks first) in a snake, wave g positions g, 2G-1-g, 2G+g, ...,
// so every wave's chunks sum to about the same work instead of the
// dispatcher's greedy block placement.
#ifndef GSR_COMP_PERSIST
#define GSR_COMP_PERSIST 0
#endif

template <int FRAG, bool kBound>
__global__ __launch_bounds__(kCompThreads) GSR_COMP_OCC void k_composite(const uint4* __restrict__ desc,
                                                        const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ n_chunks_dev,
                                                        const uint32_t* __restrict__ list,
                                                        const SplatRec* __restrict__ recs, CompositeArgs a,
                                                        float* __restrict__ out, float4* __restrict__ partial,
                                                        uint32_t* __restrict__ sat, float4* __restrict__ tmax,
                                                        const uint32_t* __restrict__ chunk_base) {
    __shared__ float4 lds[kCompWaves][kBatch * 3];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (GSR_COMP_PERSIST > 0) {
        const uint32_t total = (uint32_t)a.num_tiles + n_chunks_dev[0];
        const uint32_t G = gridDim.x * kCompWaves, g = comp_block() * kCompWaves + wave;
        for (uint32_t r = 0;; ++r) {  // (a wave's positions increase with r: the first past the end ends it)
            const uint32_t pos = r * G + ((r & 1u) ? G - 1u - g : g);
            if (pos >= total) break;
            const uint32_t slot = order[pos];
            composite_chunk<FRAG, kBound, (GSR_COMP_PRIO & 1) != 0>(desc[slot], slot, lds[wave], list, recs, a, out, partial, sat, tmax,
                                          chunk_base);
        }
        return;
    }
    const uint32_t pos = comp_block() * kCompWaves + wave;
    if (pos >= (uint32_t)a.num_tiles + n_chunks_dev[0]) return;  // device count of extra chunks
    const uint32_t slot = order[pos];
#ifdef GSR_COMP_TRACE
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint4 d = desc[slot];
#ifdef GSR_COMP_TRACE
    uint32_t evals = 0;
    composite_chunk<FRAG, kBound, (GSR_COMP_PRIO & 1) != 0>(d, slot, lds[wave], list, recs, a, out, partial, sat, tmax, chunk_base, &evals);
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (__lane_id() == 0 && slot < kTraceMax) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));     // HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // XCC_ID
        // .w: the XCC in bits 0-3, the chunk's (record, slice) evaluations above
        g_comp_trace[2 * slot] = make_uint4(slot, hw, d.z - d.y, (xcc & 15u) | (evals << 4));
        g_comp_trace[2 * slot + 1] = make_uint4((uint32_t)t0, (uint32_t)t1, (uint32_t)r0, (uint32_t)r1);
    }
#else
    composite_chunk<FRAG, kBound, (GSR_COMP_PRIO & 1) != 0>(d, slot, lds[wave], list, recs, a, out, partial, sat, tmax, chunk_base);
#endif
}

// The composite of a group of views, one wave per chunk of any view.  By
// default (interleaved) the group's dispatch runs class-major over the views:
// every view's full chunks, then every view's longest partials, and so on
// (each view's chunks of one class in its own dispatch order), so the last
// waves of the launch are short chunks of all views.  View-major (interleave
// off: all of view 0, then view 1, ...) left the last view's long chunks to
// run alone at the end.  Waves past the group's chunk count exit.
struct CompView {
    const uint4* desc;
    const uint32_t* order;
    const uint32_t* n_chunks_dev;
    const uint32_t* cls_tot;  // the view's chunks per length class (chunk_class_totals)
    const uint32_t* list;
    const SplatRec* recs;
    float* out;
    float4* partial;
    uint32_t* sat;
    float4* tmax;
    const uint32_t* chunk_base;
};
struct CompViews {
    CompView v[kMaxViews];
    uint32_t k, classes;      // views; length classes (k * classes <= 64 when interleaved)
    uint32_t view_blocks;     // view-major: blocks per view
    uint32_t interleave;
    uint64_t* stamps;         // profiling (else null): [grid] block starts, then [grid * waves] wave ends
};

// Interleaved dispatch: the (view, position) of the group's p-th chunk, or
// view -1 past the end.  Lane j = v * classes + c holds view v's count of
// class c; lane q = c * k + v takes it in dispatch (class-major) order.
__device__ __forceinline__ int interleaved_chunk(const CompViews& vs, uint32_t p, uint32_t& pos) {
    const uint32_t lane = __lane_id();
    const uint32_t kc = vs.k * vs.classes;
    uint32_t n = 0;
    for (uint32_t v = 0; v < vs.k; ++v)  // independent loads, one view's classes each
        if (lane >= v * vs.classes && lane < (v + 1) * vs.classes) n = vs.v[v].cls_tot[lane - v * vs.classes];
    const uint32_t vm_incl = wave_inclusive_scan(n);  // view-major
    const uint32_t qc = lane / vs.k, qv = lane - qc * vs.k;
    const uint32_t nq = __shfl(n, (int)(lane < kc ? qv * vs.classes + qc : 0u), 64);
    const uint32_t q_incl = wave_inclusive_scan(lane < kc ? nq : 0u);  // class-major
    const uint64_t hit = __ballot(lane < kc && p < q_incl);
    if (hit == 0) return -1;
    const int q = (int)__builtin_ctzll(hit);
    const uint32_t c = (uint32_t)q / vs.k, v = (uint32_t)q - c * vs.k;
    // (q, v, c are wave-uniform: readlane, not an LDS permute)
    const uint32_t q_excl = (uint32_t)__builtin_amdgcn_readlane((int)(q_incl - nq), q);
    // the view's own dispatch position: its chunks of the earlier classes first
    const uint32_t vm_excl = vm_incl - n;
    const uint32_t cls_base = (uint32_t)__builtin_amdgcn_readlane((int)vm_excl, (int)(v * vs.classes + c)) -
                              (uint32_t)__builtin_amdgcn_readlane((int)vm_excl, (int)(v * vs.classes));
    pos = cls_base + (p - q_excl);
    return (int)v;
}

template <int FRAG>
__device__ __forceinline__ void composite_views_wave(const CompViews& vs, const CompositeArgs& a, float4* lds,
                                                     int wave) {
    int view;
    uint32_t pos;
    if (vs.interleave) {
        view = __builtin_amdgcn_readfirstlane(interleaved_chunk(vs, blockIdx.x * kCompWaves + wave, pos));
        pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)pos);
        if (view < 0) return;
    } else {
        view = (int)(blockIdx.x / vs.view_blocks);
        pos = (blockIdx.x - (uint32_t)view * vs.view_blocks) * kCompWaves + wave;
    }
    const CompView& v = vs.v[view];
    if (pos >= (uint32_t)a.num_tiles + v.n_chunks_dev[0]) return;
    const uint32_t slot = v.order[pos];
    const uint4 d = v.desc[slot];
    composite_chunk<FRAG, kBoundViews, (GSR_COMP_PRIO & 2) != 0>(d, slot, lds, v.list, v.recs, a, v.out, v.partial, v.sat, v.tmax, v.chunk_base);
}

template <int FRAG>
__global__ __launch_bounds__(kCompThreads) GSR_COMP_OCC void k_composite_views(CompViews vs, CompositeArgs a) {
    __shared__ float4 lds[kCompWaves][kBatch * 3];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (vs.stamps && threadIdx.x == 0) vs.stamps[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    composite_views_wave<FRAG>(vs, a, lds[wave], wave);
    if (vs.stamps && __lane_id() == 0)
        vs.stamps[gridDim.x + blockIdx.x * kCompWaves + wave] = __builtin_amdgcn_s_memrealtime();
}


// Fold the partial results of multi-chunk tiles in depth order: one block per
// tile of 4 x P waves (P = kMergeParts); wave w folds slice (w & 3) over the
// (w >> 2)-th of P parts of the tile's chunks (up to the saturating chunk, if
// any) with 16 partial loads in flight, and the parts are combined in order
// through LDS.  Default P = 1 (256 threads): with P = 4 (1024 threads) the
// deepest tiles' fold was spread over 4 waves, but a 16-wave block waits for
// a whole CU's worth of free slots while other views' compositors hold the
// chip: 0.2124 / 0.2126 -> 0.207 / 0.2074 ms per frame in flight with P = 1,
// and 17.4 -> 14.8 us alone (r1_s10 box).
#ifndef GSR_MERGE_THREADS
#define GSR_MERGE_THREADS 256
#endif
constexpr int kMergeThreads = GSR_MERGE_THREADS;
constexpr int kMergeParts = kMergeThreads / 64 / 4;  // 4
#ifndef GSR_MERGE_DEPTH
#define GSR_MERGE_DEPTH 16
#endif
constexpr int kMergeDepth = GSR_MERGE_DEPTH;  // partial loads in flight per lane

__device__ __forceinline__ void merge_tile(const uint32_t* __restrict__ chunk_cnt,
                                           const uint32_t* __restrict__ chunk_base,
                                           const float4* __restrict__ partial, const uint32_t* __restrict__ sat,
                                           const CompositeArgs& a, float* __restrict__ out,
                                           float4 (*part)[4][64]) {
    const int tile = blockIdx.x;
    const uint32_t cnt = chunk_cnt[tile];
    if (cnt <= 1) return;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k = w & 3, q = w >> 2;
    const int lane = __lane_id();
    const uint32_t last = min(cnt - 1, 0xffffffffu - ld_relaxed(sat + tile * 4 + k));  // written by atomics
    const uint32_t nfold = last + 1;
    const uint32_t per = (nfold + kMergeParts - 1) / kMergeParts;
    const uint32_t c_begin = min(nfold, q * per), c_end = min(nfold, c_begin + per);
    const uint32_t base = chunk_base[tile];
    float r = 0.f, g = 0.f, b = 0.f, T = 1.f;
    for (uint32_t c0 = c_begin; c0 < c_end; c0 += kMergeDepth) {
        float4 v[kMergeDepth];
#pragma unroll
        for (int j = 0; j < kMergeDepth; ++j) {
            const uint32_t c = c0 + j;
            if (c < c_end) {
                const uint32_t slot = c == 0 ? (uint32_t)tile : base + c - 1;
                v[j] = partial[(size_t)slot * 256 + k * 64 + lane];
            } else {
                v[j] = make_float4(0.f, 0.f, 0.f, 1.f);
            }
        }
#pragma unroll
        for (int j = 0; j < kMergeDepth; ++j) {
            r += T * v[j].x;
            g += T * v[j].y;
            b += T * v[j].z;
            T *= v[j].w;
        }
    }
    part[q][k][lane] = make_float4(r, g, b, T);
    __syncthreads();
    if (q != 0) return;
    // (C1, T1) then (C2, T2) == (C1 + T1*C2, T1*T2), quarters in depth order
#pragma unroll
    for (int p = 1; p < kMergeParts; ++p) {
        const float4 v = part[p][k][lane];
        r += T * v.x;
        g += T * v.y;
        b += T * v.z;
        T *= v.w;
    }
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int x = tx * kTile + (lane & 15);
    const int row = ty * kTile + 4 * k + (lane >> 4);
    if (x >= a.width || row >= a.height) return;
    r += T * a.bg[0];
    g += T * a.bg[1];
    b += T * a.bg[2];
    const size_t plane = (size_t)a.width * a.height;
    const size_t pidx = (size_t)row * a.width + x;
    if (a.out_layout == 0) {
        st_out(out + pidx, r);
        st_out(out + plane + pidx, g);
        st_out(out + 2 * plane + pidx, b);
    } else {
        st_out(out + 3 * pidx, r);
        st_out(out + 3 * pidx + 1, g);
        st_out(out + 3 * pidx + 2, b);
    }
}

__global__ __launch_bounds__(kMergeThreads) void k_merge(const uint32_t* __restrict__ chunk_cnt,
                                                         const uint32_t* __restrict__ chunk_base,
                                                         const float4* __restrict__ partial,
                                                         const uint32_t* __restrict__ sat, CompositeArgs a,
                                                         float* __restrict__ out) {
    __shared__ float4 part[kMergeParts][4][64];
    merge_tile(chunk_cnt, chunk_base, partial, sat, a, out, part);
}

struct MergeView {
    const uint32_t* chunk_cnt;
    const uint32_t* chunk_base;
    const float4* partial;
    const uint32_t* sat;
    float* out;
};
struct MergeViews {
    MergeView v[kMaxViews];
};

__global__ __launch_bounds__(kMergeThreads) void k_merge_views(MergeViews vs, CompositeArgs a) {
    __shared__ float4 part[kMergeParts][4][64];
    const MergeView& v = vs.v[blockIdx.y];
    merge_tile(v.chunk_cnt, v.chunk_base, v.partial, v.sat, a, v.out, part);
}

// ---------------------------------------------------------------- unorm8 blend
// GSR_BLEND_UNORM8: what the reference viewer's RGBA8 framebuffer holds.  GL
// blends every fragment in draw order (back to front) with SRC_ALPHA /
// ONE_MINUS_SRC_ALPHA into unorm8 storage (renderer_ogl.py:178-180,
// main.py:197-198).  That is not associative, so there are no chunks, no early
// termination and no merge: one wave per tile walks the tile's list backwards
// (its lists are front to back), 4 pixels per lane as in composite_chunk.
// Records are in plain form (u.plain_rec: plain opacity and colour, mid = 0).
// The per-fragment arithmetic is the fragment stage's (gau_frag.glsl:30-53);
// the blend is the RGBA8 target's fixed-point arithmetic as Mesa llvmpipe runs
// it on the reference's own shaders (tests/golden/llvmpipe_golden.npz,
// oracle/gl_oracle.py blend8): colour and alpha to unorm8 by
// rint(fl32(v * 255/256) * 256), then dst = min(255, mul8(c, a) +
// mul8(dst, 255 - a)) with llvmpipe's approximation of x y / 255,
// mul8(x, y) = (t + (t >> 8) + 128) >> 8, t = x y (lp_build_mul_norm; it
// differs from round(x y / 255) on 24 of the 65536 pairs).  The
// falloff is the record's log2-scaled quadratic, so alpha can differ from the
// oracle's expf(power) by an ulp, which moves it across an 8-bit rounding
// boundary rarely.
__device__ __forceinline__ float clamp01f(float v) { return fminf(fmaxf(v, 0.f), 1.f); }

__device__ __forceinline__ uint32_t to_unorm8(float v) {
#pragma clang fp contract(off)
    return (uint32_t)rintf((clamp01f(v) * (255.0f / 256.0f)) * 256.0f);
}

__device__ __forceinline__ uint32_t mul8(uint32_t x, uint32_t y) {
    const uint32_t t = x * y;
    return (t + (t >> 8) + 128u) >> 8;
}

__device__ __forceinline__ uint32_t blend8(uint32_t c, uint32_t a, uint32_t d) {
    return min(255u, mul8(c, a) + mul8(d, 255u - a));
}

template <int FRAG>
__device__ __forceinline__ void composite_tile_unorm8(const int tile, const uint2 range, float4* __restrict__ my,
                                                      const uint32_t* __restrict__ list,
                                                      const SplatRec* __restrict__ recs, const CompositeArgs& a,
                                                      float* __restrict__ out) {
    const int lane = __lane_id();
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int lcol = lane & 15, lrow = lane >> 4;
    const int col_base = tx * kTile, row_base = ty * kTile;
    const int x = col_base + lcol;
    const float px = (float)x + 0.5f;
    float pyw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) pyw[k] = (float)(a.height - 1 - (row_base + 4 * k + lrow)) + 0.5f;
    uint32_t pr[4], pg[4], pb[4];  // the framebuffer (unorm8), cleared to the background
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        pr[k] = to_unorm8(a.bg[0]);
        pg[k] = to_unorm8(a.bg[1]);
        pb[k] = to_unorm8(a.bg[2]);
    }
    // batches of up to 64 records, last (backmost) first
    for (uint32_t top = range.y; top > range.x; top -= min((uint32_t)kBatch, top - range.x)) {
        const uint32_t nb = min((uint32_t)kBatch, top - range.x);
        __builtin_amdgcn_wave_barrier();
        uint64_t sb[4];
        {
            float4 f0 = make_float4(0.f, 0.f, 0.f, 0.f), f1 = f0, f2 = f0;
            uint32_t covx = 0, covy = 0;
            if ((uint32_t)lane < nb) {  // batch record `lane` = list position top - 1 - lane (draw order)
                const float4* r = reinterpret_cast<const float4*>(recs + list[top - 1 - lane]);
                f0 = r[0]; f1 = r[1]; f2 = r[2];
                const uint32_t xs = __float_as_uint(f0.w), ys = __float_as_uint(f1.w);
                covx = span_bits16((int)(xs & 0xffffu) - col_base, (int)(xs >> 16) - col_base);
                covy = span_bits16((int)(ys & 0xffffu) - row_base, (int)(ys >> 16) - row_base);
            }
            my[lane * 3 + 0] = make_float4(f0.x, f0.y, f0.z, __uint_as_float(covx | (covy << 16)));
            my[lane * 3 + 1] = make_float4(f1.x, f1.y, f1.z, 0.f);
            my[lane * 3 + 2] = make_float4(f2.x, f2.y, f2.z, 0.f);
#pragma unroll
            for (int k = 0; k < 4; ++k) sb[k] = (uint64_t)__ballot(((covy >> (4 * k)) & 0xfu) != 0u && covx != 0u);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll 1
        for (int j = 0; j < (int)nb; ++j) {
            const float4 q0 = my[j * 3 + 0];  // cx cy opacity coverage
            const float4 q1 = my[j * 3 + 1];  // qa qb qc -
            const float4 q2 = my[j * 3 + 2];  // r g b -
            const uint32_t cov = __float_as_uint(q0.w);
            const bool colin = (cov >> lcol) & 1u;
            const float dx = px - q0.x;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (!((sb[k] >> j) & 1ull)) continue;
                const bool covered = colin && ((cov >> (16 + 4 * k + lrow)) & 1u);
                float al = 1.0f, cr = q2.x, cg = q2.y, cbl = q2.z;
                bool keep = covered;
                if (FRAG != kFragBillboard) {
                    const float dy = pyw[k] - q0.y;
                    const float pw = (q1.z * dy + q1.y * dx) * dy + q1.x * dx * dx;  // power * log2(e)
                    const float e = __builtin_amdgcn_exp2f(pw);
                    al = fminf(0.99f, q0.z * e);
                    keep = keep && !(pw > 0.0f) && !(al < 1.0f / 255.0f);
                    if (FRAG == kFragFlatBall || FRAG == kFragGaussBall) al = al > 0.22f ? 1.0f : 0.0f;
                    if (FRAG == kFragGaussBall) {
                        cr = q2.x * e;
                        cg = q2.y * e;
                        cbl = q2.z * e;
                    }
                }
                if (keep) {
                    const uint32_t a8 = to_unorm8(al);
                    pr[k] = blend8(to_unorm8(cr), a8, pr[k]);
                    pg[k] = blend8(to_unorm8(cg), a8, pg[k]);
                    pb[k] = blend8(to_unorm8(cbl), a8, pb[k]);
                }
            }
        }
    }
    if (x >= a.width) return;
    const size_t plane = (size_t)a.width * a.height;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = row_base + 4 * k + lrow;
        if (row >= a.height) continue;
        const size_t pidx = (size_t)row * a.width + x;
        const float vr = (float)pr[k] / 255.0f, vg = (float)pg[k] / 255.0f, vb = (float)pb[k] / 255.0f;
        if (a.out_layout == 0) {
            out[pidx] = vr;
            out[plane + pidx] = vg;
            out[2 * plane + pidx] = vb;
        } else {
            out[3 * pidx] = vr;
            out[3 * pidx + 1] = vg;
            out[3 * pidx + 2] = vb;
        }
    }
}

template <int FRAG>
__global__ __launch_bounds__(256) void k_composite_unorm8(const uint2* __restrict__ ranges,
                                                          const uint32_t* __restrict__ list,
                                                          const SplatRec* __restrict__ recs, CompositeArgs a,
                                                          float* __restrict__ out) {
    __shared__ float4 lds[4][kBatch * 3];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.x * 4 + wave;
    if (tile >= a.num_tiles) return;
    composite_tile_unorm8<FRAG>(tile, ranges[tile], lds[wave], list, recs, a, out);
}

}  // namespace

#ifdef GSR_COMP_STATS
// host5: slice evaluations, those on saturated slices, records, instances, slices where no lane keeps a fragment
extern "C" int gsr_debug_comp_stats(unsigned long long* host5) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(host5, HIP_SYMBOL(gsr::g_comp_stats), 40, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    static const unsigned long long zeros[5] = {0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_comp_stats), zeros, 40, 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif

#ifdef GSR_COMP_TRACE
// Copies the last composite launch's per-wave stamps to host memory (tooling).
extern "C" int64_t gsr_debug_comp_trace(void* host_dst, int64_t max_entries) {
    const int64_t n = max_entries < (int64_t)kTraceMax ? max_entries : (int64_t)kTraceMax;
    if (hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(g_comp_trace), (size_t)n * 32, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}
#endif

uint32_t clamp_stage_limit(long v) { return (v >= 0 && v < kBinStage) ? (uint32_t)v : (uint32_t)kBinStage; }

size_t bin_tmp_elems(size_t n_vis) { return (n_vis + kBinBlock - 1) / kBinBlock + 1; }

int launch_binning(const uint32_t* sorted_ids, const uint2* trect, const uint32_t* rect4_sorted, uint32_t n_vis,
                   int tiles_x, uint32_t* tmp, uint2* trect_sorted, uint32_t* tile_keys, uint32_t* tile_vals,
                   uint32_t stage_limit, hipStream_t s) {
    stage_limit = std::min(stage_limit, (uint32_t)kBinStage);
    if (n_vis == 0) return GSR_OK;
    const uint32_t nb = (n_vis + kBinBlock - 1) / kBinBlock;
    if (rect4_sorted)
        k_bin_reduce<true><<<nb, kThreads, 0, s>>>(sorted_ids, trect, rect4_sorted, n_vis, tmp, trect_sorted);
    else
        k_bin_reduce<false><<<nb, kThreads, 0, s>>>(sorted_ids, trect, rect4_sorted, n_vis, tmp, trect_sorted);
    GSR_LAUNCH_CHECK("bin_reduce");
    if (rect4_sorted)
        k_bin_write<true><<<nb, kThreads, 0, s>>>(sorted_ids, trect_sorted, rect4_sorted, n_vis, tmp, tiles_x,
                                                  tile_keys, tile_vals, stage_limit);
    else
        k_bin_write<false><<<nb, kThreads, 0, s>>>(sorted_ids, trect_sorted, rect4_sorted, n_vis, tmp, tiles_x,
                                                   tile_keys, tile_vals, stage_limit);
    GSR_LAUNCH_CHECK("bin_write");
    return GSR_OK;
}

size_t bin_hist_elems(size_t n_vis, int tbits, int passes) {
    if (tbits <= 0 || passes <= 0) return 0;
    return ((n_vis + kBinBlock - 1) / kBinBlock) * ((size_t)1 << ((tbits + passes - 1) / passes));
}

int launch_binning_sorted(const uint32_t* sorted_ids, const uint2* trect, const uint32_t* rect4_sorted,
                          uint32_t n_vis, int tiles_x, int tbits, int passes, uint32_t* hist, uint32_t* totals,
                          uint2* trect_sorted, uint32_t* tile_keys, uint32_t* tile_vals, hipStream_t s,
                          const uint32_t* sorted_keys, uint32_t* inst_keys) {
    if (n_vis == 0) return GSR_OK;
    const int tb = tbits > 0 ? tbits : 1;  // one tile: a single digit value, generation order kept
    const int ps = passes > 0 ? passes : 1;
    const int w = (tb + ps - 1) / ps;
    if (w > 11) return set_error(GSR_ERR_INVALID, "binning: tile digit wider than 11 bits");
    const uint32_t nbb = (n_vis + kBinBlock - 1) / kBinBlock;
    const PassArgs pa{nullptr, (uint32_t)tb, (uint32_t)ps, 0u};
    const bool packed = rect4_sorted != nullptr;
#define GSR_BIN_HIST(P, CB)                                                                                 \
    k_bin_hist<P, CB><<<nbb, kThreads, 0, s>>>(sorted_ids, trect, rect4_sorted, n_vis, tiles_x, pa, hist, nbb, \
                                               trect_sorted)
#define GSR_BIN_SCATTER(P, CB)                                                                                  \
    do {                                                                                                        \
        if (inst_keys)                                                                                          \
            k_bin_scatter<P, CB, true><<<nbb, kThreads, 0, s>>>(sorted_ids, trect_sorted, rect4_sorted, n_vis,     \
                                                                tiles_x, pa, hist, totals, nbb, tile_keys,         \
                                                                tile_vals, sorted_keys, inst_keys);                \
        else                                                                                                    \
            k_bin_scatter<P, CB, false><<<nbb, kThreads, 0, s>>>(sorted_ids, trect_sorted, rect4_sorted, n_vis,    \
                                                                 tiles_x, pa, hist, totals, nbb, tile_keys,        \
                                                                 tile_vals, nullptr, nullptr);                     \
    } while (0)
    if (w <= 8) {
        if (packed) GSR_BIN_HIST(true, 8); else GSR_BIN_HIST(false, 8);
    } else {
        if (packed) GSR_BIN_HIST(true, 11); else GSR_BIN_HIST(false, 11);
    }
    GSR_LAUNCH_CHECK("bin_hist");
    int rc;
    if ((rc = radix_offsets(hist, nbb, tb, ps, 0, totals, s))) return rc;
    if (w <= 8) {
        if (packed) GSR_BIN_SCATTER(true, 8); else GSR_BIN_SCATTER(false, 8);
    } else {
        if (packed) GSR_BIN_SCATTER(true, 11); else GSR_BIN_SCATTER(false, 11);
    }
    GSR_LAUNCH_CHECK("bin_scatter");
#undef GSR_BIN_HIST
#undef GSR_BIN_SCATTER
    return GSR_OK;
}

int launch_tile_ranges(const uint32_t* tile_keys, uint32_t n_dup, uint2* ranges, const RunFix& fix, hipStream_t s) {
    if (n_dup == 0) return GSR_OK;
    const uint32_t per_block = kThreads * (fix.coarse ? kFixItems : kRangeItems);
    if (fix.coarse)
        k_tile_ranges<true><<<(n_dup + per_block - 1) / per_block, kThreads, 0, s>>>(tile_keys, n_dup, ranges, fix);
    else
        k_tile_ranges<false><<<(n_dup + per_block - 1) / per_block, kThreads, 0, s>>>(tile_keys, n_dup, ranges, fix);
    GSR_LAUNCH_CHECK("tile_ranges");
    return GSR_OK;
}

// Multi-chunk tiles folded by their last chunk inside the compositing launch
// (tail_merge): a group's frames (3072-instance chunks: few multi-chunk tiles)
// do it by default, which drops one launch per group (the context's
// GSR_TAIL_MERGE=0: k_merge_views).  A frame alone (192-instance chunks: ~2500
// multi-chunk tiles at C2) keeps k_merge: a deep tile's last chunk folding ~40
// partials alone put the fold on the launch's tail, composite 120 -> 170 us
// (profiles/r3_s9); its four waves per tile in k_merge take 15
// (GSR_TAIL_MERGE_ALONE=1 to A/B).  The flags are read once, at context
// creation, and the compositing and merge launches of a frame get the same one.
static CompositeArgs make_args(const FrameUniforms& u, float t_min, const float* bg, int out_layout,
                               bool tail_merge = false, uint32_t debug_handoff = 0) {
    CompositeArgs a;
    a.width = u.width;
    a.height = u.height;
    a.tiles_x = u.tiles_x;
    a.num_tiles = u.tiles_x * u.tiles_y;
    a.t_min = t_min;
    a.bg[0] = bg[0];
    a.bg[1] = bg[1];
    a.bg[2] = bg[2];
    a.out_layout = out_layout;
    a.tail_merge = tail_merge ? 1 : 0;
    a.debug_handoff = tail_merge ? debug_handoff : 0u;
    return a;
}

size_t chunk_cnt_elems(int num_tiles) {
    return (size_t)num_tiles + (1 + kMaxLenClasses) * ((size_t)num_tiles / kThreads + 1) + kMaxLenClasses + 1;
}

const uint32_t* chunk_class_totals(const uint32_t* chunk_cnt, int num_tiles, uint32_t classes) {
    const size_t g = ((size_t)num_tiles + kThreads - 1) / kThreads;
    return chunk_cnt + num_tiles + (1 + classes) * g;
}

int launch_chunks(const uint2* ranges, int num_tiles, uint32_t chunk, uint32_t classes, uint32_t* chunk_cnt,
                  uint32_t* chunk_base, uint32_t* n_extra_dev, uint4* desc, uint32_t* order, float4* tmax,
                  hipStream_t s, bool first_major, const LongRuns* long_runs, uint32_t max_extra) {
    if (classes < 2 || classes > (uint32_t)kMaxLenClasses) return set_error(GSR_ERR_INVALID, "chunk length classes");
    const unsigned g = (unsigned)((num_tiles + kThreads - 1) / kThreads);
    // the per-block totals live in chunk_cnt past its num_tiles entries
    uint32_t* tot = chunk_cnt + num_tiles;
    // one block for the whole frame when it fits (k_chunk_single); the long runs as its blocks 1..
    if ((uint32_t)num_tiles <= kCsMaxTiles && max_extra <= kCsMaxExtra &&
        classes <= (uint32_t)kCsClasses) {
        const bool runs = long_runs && long_runs->n_dup > 0 && long_runs->fix.coarse;
        LongRunArgs la{};
        if (runs)
            if (int rc = long_run_args(long_runs->tile_keys, long_runs->n_dup, ranges, long_runs->fix, la)) return rc;
        k_chunk_single<<<1 + (runs ? kLongGrid : 0), kCsThreads, 0, s>>>(
            ranges, num_tiles, chunk, classes, first_major ? 1u : 0u, chunk_cnt, chunk_base, n_extra_dev, desc, order,
            tmax, const_cast<uint32_t*>(chunk_class_totals(chunk_cnt, num_tiles, classes)), la);
        GSR_LAUNCH_CHECK("chunk_single");
        return GSR_OK;
    }
    if (long_runs && long_runs->n_dup > 0 && long_runs->fix.coarse) {
        LongRunArgs la;
        if (int rc = long_run_args(long_runs->tile_keys, long_runs->n_dup, ranges, long_runs->fix, la)) return rc;
        const unsigned n_cc = (g + kCountGroups - 1) / kCountGroups;
        k_chunk_count_long<<<n_cc + kLongGrid, kTdsThreads, 0, s>>>(ranges, num_tiles, chunk, classes, tot,
                                                                    first_major ? 1u : 0u, n_cc, la);
        GSR_LAUNCH_CHECK("chunk_count_long");
    } else {
        k_chunk_count<<<g, kThreads, 0, s>>>(ranges, num_tiles, chunk, classes, tot, first_major ? 1u : 0u);
        GSR_LAUNCH_CHECK("chunk_count");
    }
    k_chunk_write<<<g, kThreads, 0, s>>>(ranges, num_tiles, chunk, classes, tot, chunk_cnt, chunk_base, n_extra_dev,
                                         desc, order, tmax, first_major ? 1u : 0u);
    GSR_LAUNCH_CHECK("chunk_write");
    return GSR_OK;
}

int launch_long_runs(const uint32_t* tile_keys, uint32_t n_dup, const uint2* ranges, const RunFix& fix,
                     hipStream_t s) {
    if (n_dup == 0 || fix.coarse == 0) return GSR_OK;
    LongRunArgs a;
    if (int rc = long_run_args(tile_keys, n_dup, ranges, fix, a)) return rc;
    k_long_runs<<<kLongGrid, kTdsThreads, 0, s>>>(a);
    GSR_LAUNCH_CHECK("long_runs");
    return GSR_OK;
}

template <int FRAG>
static void composite_launch(unsigned grid, bool bound, hipStream_t s, const uint4* desc, const uint32_t* order,
                             const uint32_t* n_chunks_dev, const uint32_t* tile_vals, const SplatRec* recs,
                             const CompositeArgs& a, float* out, float4* partial, uint32_t* sat, float4* tmax,
                             const uint32_t* chunk_base) {
    if (bound)
        k_composite<FRAG, true><<<grid, kCompThreads, 0, s>>>(desc, order, n_chunks_dev, tile_vals, recs, a, out, partial,
                                                              sat, tmax, chunk_base);
    else
        k_composite<FRAG, false><<<grid, kCompThreads, 0, s>>>(desc, order, n_chunks_dev, tile_vals, recs, a, out, partial,
                                                               sat, tmax, chunk_base);
}

int launch_composite(const uint4* desc, const uint32_t* order, const uint32_t* n_chunks_dev, uint32_t max_chunks,
                     const uint32_t* chunk_cnt,
                     const uint32_t* chunk_base, uint32_t* sat, const uint32_t* tile_vals, const SplatRec* recs,
                     const FrameUniforms& u, int frag_class, float t_min, const float* bg, int out_layout, float* out,
                     float4* partial, float4* tmax, bool tail_merge, hipStream_t s) {
    const CompositeArgs a = make_args(u, t_min, bg, out_layout, tail_merge);
    if (max_chunks == 0) return GSR_OK;
    unsigned grid = (unsigned)((max_chunks + kCompWaves - 1) / kCompWaves);
    if (GSR_COMP_PERSIST > 0) {  // experiment: a resident grid (k_composite)
        static int cus = 0;
        if (!cus) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
                cus = 256;
        }
        grid = std::min(grid, (unsigned)(cus * GSR_COMP_PERSIST));
    }
    const bool bound = tmax != nullptr;  // the cross-chunk transmittance bound (launch_chunks initialised tmax)
    switch (frag_class) {
        case kFragGauss:
            composite_launch<kFragGauss>(grid, bound, s, desc, order, n_chunks_dev, tile_vals, recs, a, out, partial,
                                         sat, tmax, chunk_base);
            break;
        case kFragBillboard:
            composite_launch<kFragBillboard>(grid, bound, s, desc, order, n_chunks_dev, tile_vals, recs, a, out,
                                             partial, sat, tmax, chunk_base);
            break;
        case kFragFlatBall:
            composite_launch<kFragFlatBall>(grid, bound, s, desc, order, n_chunks_dev, tile_vals, recs, a, out,
                                            partial, sat, tmax, chunk_base);
            break;
        default:
            composite_launch<kFragGaussBall>(grid, bound, s, desc, order, n_chunks_dev, tile_vals, recs, a, out,
                                             partial, sat, tmax, chunk_base);
            break;
    }
    GSR_LAUNCH_CHECK("composite");
    return GSR_OK;
}

int launch_composite_unorm8(const uint2* ranges, const uint32_t* tile_list, const SplatRec* recs,
                            const FrameUniforms& u, int frag_class, const float* bg, int out_layout, float* out,
                            hipStream_t s) {
    const CompositeArgs a = make_args(u, 0.f, bg, out_layout);
    const unsigned grid = (unsigned)((a.num_tiles + 3) / 4);
    switch (frag_class) {
        case kFragGauss: k_composite_unorm8<kFragGauss><<<grid, 256, 0, s>>>(ranges, tile_list, recs, a, out); break;
        case kFragBillboard:
            k_composite_unorm8<kFragBillboard><<<grid, 256, 0, s>>>(ranges, tile_list, recs, a, out);
            break;
        case kFragFlatBall:
            k_composite_unorm8<kFragFlatBall><<<grid, 256, 0, s>>>(ranges, tile_list, recs, a, out);
            break;
        default: k_composite_unorm8<kFragGaussBall><<<grid, 256, 0, s>>>(ranges, tile_list, recs, a, out); break;
    }
    GSR_LAUNCH_CHECK("composite_unorm8");
    return GSR_OK;
}

int launch_merge(const uint32_t* chunk_cnt, const uint32_t* chunk_base, const float4* partial, const uint32_t* sat,
                 const FrameUniforms& u, float t_min, const float* bg, int out_layout, float* out, bool tail_merge,
                 hipStream_t s) {
    if (tail_merge) return GSR_OK;  // the compositing launch folded its multi-chunk tiles
    const CompositeArgs a = make_args(u, t_min, bg, out_layout);
    k_merge<<<(unsigned)a.num_tiles, kMergeThreads, 0, s>>>(chunk_cnt, chunk_base, partial, sat, a, out);
    GSR_LAUNCH_CHECK("merge");
    return GSR_OK;
}

// ------------------------------------------------------------ groups of views
int launch_binning_views(FinishView* views, int k, int tiles_x, uint32_t stage_limit, hipStream_t s) {
    stage_limit = std::min(stage_limit, (uint32_t)kBinStage);
    BinViews bv{};
    uint32_t nb[kMaxViews];
    uint32_t nb_max = 0;
    for (int i = 0; i < k; ++i) {
        const FinishView& f = views[i];
        bv.v[i] = BinView{f.sorted_ids, f.trect, f.rect4_sorted, f.trect_sorted, f.bin_tmp, f.tile_keys, f.tile_vals,
                          f.n_vis};
        if ((f.rect4_sorted != nullptr) != (views[0].rect4_sorted != nullptr))
            return set_error(GSR_ERR_INVALID, "binning: packed rectangles on some views only");
        nb[i] = (f.n_vis + kBinBlock - 1) / kBinBlock;
        nb_max = std::max(nb_max, nb[i]);
    }
    if (nb_max == 0) return GSR_OK;
    const bool packed = views[0].rect4_sorted != nullptr;
    if (packed)
        k_bin_reduce_views<true><<<dim3(nb_max, (unsigned)k), kThreads, 0, s>>>(bv);
    else
        k_bin_reduce_views<false><<<dim3(nb_max, (unsigned)k), kThreads, 0, s>>>(bv);
    GSR_LAUNCH_CHECK("bin_reduce_views");
    if (packed)
        k_bin_write_views<true><<<dim3(nb_max, (unsigned)k), kThreads, 0, s>>>(bv, tiles_x, stage_limit);
    else
        k_bin_write_views<false><<<dim3(nb_max, (unsigned)k), kThreads, 0, s>>>(bv, tiles_x, stage_limit);
    GSR_LAUNCH_CHECK("bin_write_views");
    return GSR_OK;
}

int launch_binning_sorted_views(FinishView* views, uint32_t* const* hist, uint32_t* const* totals, int k, int tiles_x,
                                int tbits, int passes, hipStream_t s) {
    BinSortViews bv{};
    uint32_t nbb = 0;
    for (int i = 0; i < k; ++i) {
        const FinishView& f = views[i];
        bv.v[i] = BinView{f.sorted_ids, f.trect, f.rect4_sorted, f.trect_sorted, f.bin_tmp, f.tile_keys, f.tile_vals,
                          f.n_vis};
        bv.hist[i] = hist[i];
        bv.totals[i] = totals[i];
        if ((f.rect4_sorted != nullptr) != (views[0].rect4_sorted != nullptr))
            return set_error(GSR_ERR_INVALID, "binning: packed rectangles on some views only");
        nbb = std::max(nbb, (f.n_vis + kBinBlock - 1) / kBinBlock);
    }
    if (nbb == 0) return GSR_OK;
    const int tb = tbits > 0 ? tbits : 1;
    const int ps = passes > 0 ? passes : 1;
    const int w = (tb + ps - 1) / ps;
    if (w > 11) return set_error(GSR_ERR_INVALID, "binning: tile digit wider than 11 bits");
    const PassArgs pa{nullptr, (uint32_t)tb, (uint32_t)ps, 0u};
    const bool packed = views[0].rect4_sorted != nullptr;
    const dim3 grid(nbb, (unsigned)k);
    if (w <= 8) {
        if (packed) k_bin_hist_views<true, 8><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
        else k_bin_hist_views<false, 8><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
    } else {
        if (packed) k_bin_hist_views<true, 11><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
        else k_bin_hist_views<false, 11><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
    }
    GSR_LAUNCH_CHECK("bin_hist_views");
    int rc;
    if ((rc = radix_offsets_views(hist, totals, k, nbb, tb, ps, 0, s))) return rc;
    if (w <= 8) {
        if (packed) k_bin_scatter_views<true, 8><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
        else k_bin_scatter_views<false, 8><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
    } else {
        if (packed) k_bin_scatter_views<true, 11><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
        else k_bin_scatter_views<false, 11><<<grid, kThreads, 0, s>>>(bv, tiles_x, pa, nbb);
    }
    GSR_LAUNCH_CHECK("bin_scatter_views");
    return GSR_OK;
}

int launch_tile_ranges_views(FinishView* views, int k, hipStream_t s) {
    RangeViews rv{};
    uint32_t n_max = 0;
    bool fix = false;
    for (int i = 0; i < k; ++i) {
        rv.keys[i] = views[i].tile_keys;
        rv.ranges[i] = views[i].ranges;
        rv.n[i] = views[i].n_dup;
        rv.fix[i] = views[i].fix;
        fix |= views[i].fix.coarse != 0;
        n_max = std::max(n_max, views[i].n_dup);
    }
    if (n_max == 0) return GSR_OK;
    const uint32_t per_block = kThreads * (fix ? kFixItems : kRangeItems);
    if (fix)
        k_tile_ranges_views<true><<<dim3((n_max + per_block - 1) / per_block, (unsigned)k), kThreads, 0, s>>>(rv);
    else
        k_tile_ranges_views<false><<<dim3((n_max + per_block - 1) / per_block, (unsigned)k), kThreads, 0, s>>>(rv);
    GSR_LAUNCH_CHECK("tile_ranges_views");
    return GSR_OK;
}

int launch_chunks_views(FinishView* views, int k, int num_tiles, uint32_t chunk, uint32_t classes, bool first_major,
                        hipStream_t s) {
    if (classes < 2 || classes > (uint32_t)kMaxLenClasses) return set_error(GSR_ERR_INVALID, "chunk length classes");
    ChunkViews cv{};
    for (int i = 0; i < k; ++i) {
        const FinishView& f = views[i];
        float4* tmax = kBoundViews ? f.tmax : nullptr;  // the published maxima are only read by the bound form
        cv.v[i] = ChunkView{f.ranges, f.chunk_cnt, f.chunk_base, f.n_extra_dev, f.desc, f.order, tmax};
    }
    const dim3 grid((unsigned)((num_tiles + kThreads - 1) / kThreads), (unsigned)k);
    k_chunk_count_views<<<grid, kThreads, 0, s>>>(cv, num_tiles, chunk, classes, first_major ? 1u : 0u);
    GSR_LAUNCH_CHECK("chunk_count_views");
    k_chunk_write_views<<<grid, kThreads, 0, s>>>(cv, num_tiles, chunk, classes, first_major ? 1u : 0u);
    GSR_LAUNCH_CHECK("chunk_write_views");
    return GSR_OK;
}

int launch_composite_views(FinishView* views, int k, uint32_t max_chunks, uint32_t classes, bool first_major,
                           bool interleave, const FrameUniforms& u, int frag_class, float t_min, const float* bg,
                           int out_layout, bool tail_merge, uint32_t debug_handoff, hipStream_t s, uint64_t* stamps) {
    const CompositeArgs a = make_args(u, t_min, bg, out_layout, tail_merge, debug_handoff);
    CompViews cv{};
    for (int i = 0; i < k; ++i) {
        const FinishView& f = views[i];
        cv.v[i] = CompView{f.desc, f.order, f.n_extra_dev, chunk_class_totals(f.chunk_cnt, a.num_tiles, classes),
                           f.tile_vals, f.recs, f.out, f.partial, f.sat, f.tmax, f.chunk_base};
    }
    cv.k = (uint32_t)k;
    cv.classes = classes + (first_major ? 1u : 0u);  // first-major: the later chunks as one more class
    cv.view_blocks = (max_chunks + kCompWaves - 1) / kCompWaves;
    cv.interleave = interleave && (uint32_t)k * cv.classes <= 64u;
    cv.stamps = stamps;
    const dim3 grid(cv.view_blocks * (unsigned)k);
    switch (frag_class) {
        case kFragGauss: k_composite_views<kFragGauss><<<grid, kCompThreads, 0, s>>>(cv, a); break;
        case kFragBillboard: k_composite_views<kFragBillboard><<<grid, kCompThreads, 0, s>>>(cv, a); break;
        case kFragFlatBall: k_composite_views<kFragFlatBall><<<grid, kCompThreads, 0, s>>>(cv, a); break;
        default: k_composite_views<kFragGaussBall><<<grid, kCompThreads, 0, s>>>(cv, a); break;
    }
    GSR_LAUNCH_CHECK("composite_views");
    return GSR_OK;
}

size_t composite_views_blocks(uint32_t max_chunks, int k) {
    return (size_t)((max_chunks + kCompWaves - 1) / kCompWaves) * (size_t)k;
}

int composite_views_waves_per_block() { return kCompWaves; }

int launch_merge_views(FinishView* views, int k, const FrameUniforms& u, float t_min, const float* bg,
                       int out_layout, bool tail_merge, hipStream_t s) {
    if (tail_merge) return GSR_OK;  // the compositing launch folded its multi-chunk tiles
    const CompositeArgs a = make_args(u, t_min, bg, out_layout);
    MergeViews mv{};
    for (int i = 0; i < k; ++i) {
        const FinishView& f = views[i];
        mv.v[i] = MergeView{f.chunk_cnt, f.chunk_base, f.partial, f.sat, f.out};
    }
    k_merge_views<<<dim3((unsigned)a.num_tiles, (unsigned)k), kMergeThreads, 0, s>>>(mv, a);
    GSR_LAUNCH_CHECK("merge_views");
    return GSR_OK;
}

}  // namespace gsr

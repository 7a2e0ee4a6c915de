// Internal definitions shared by the gsr HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "gsr.h"

namespace gsr {

constexpr int kTile = 16;              // composite tile edge (pixels)
constexpr int kMaxViews = GSR_MAX_VIEWS;  // views of one scene begun together (gsr_render_begin_views)
constexpr int kMaxLenClasses = 16;        // compositing dispatch: full chunks + partial-length classes
constexpr int kWave = 64;              // CDNA wavefront

// One visible splat after preprocess: 48 bytes = exactly three float4, so the
// compositor reads a record with three broadcast ds_read_b128 (12 LDS cycles).
// The fragment falloff is stored as the quadratic form of power*log2(e) in
// PIXEL offsets (gau_frag.glsl:37 with coordxy = (pixel - centre) * s):
//   power*log2e = qa*dx^2 + qb*dx*dy + qc*dy^2,  dx = px - cx, dy = pyw - cy
//   qa = -0.5*log2e*A*sx*sx,  qb = -log2e*B*sx*sy,  qc = -0.5*log2e*C*sy*sy
struct alignas(16) SplatRec {
    float cx, cy;       // quad centre, window coords (origin bottom-left)
    float opacity;      // alpha varying
    uint32_t xspan;     // covered pixel columns x0 | x1 << 16, inclusive (image coords)
    float qa, qb, qc;   // falloff quadratic form (see above)
    uint32_t yspan;     // covered pixel rows r0 | r1 << 16, inclusive (image coords, row 0 = top)
    float r, g, b;      // colour varying (clamped to [0,1] unless mode -6)
    float mid;          // kFragGauss only (else 0): see below
};
// kFragGauss records carry the fragment's alpha in "interval form", so the
// compositor tests both discards of gau_frag.glsl:38-42 with ONE compare and
// gets min(0.99, .) from the clamp output modifier:
//   a = opacity * 2^pw,  keep  <=>  pw <= 0  and  a >= 1/255
//                              <=>  thr <= pw <= 0,  thr = -log2(255 * opacity)
//   mid = thr / 2:         keep  <=>  |pw - mid| <= -mid
//   min(0.99, a) = 0.99 * clamp(s * 2^(pw - mid), 0, 1),  s = sqrt(opacity / 255) / 0.99
// so `opacity` holds s and r, g, b hold 0.99 * colour (the 0.99 of the alpha
// is folded into the colour and into the transmittance update).  Other
// fragment classes keep the plain opacity and colour, and mid = 0.
static_assert(sizeof(SplatRec) == 48, "SplatRec must be 48 bytes");
constexpr float kLog2e = 1.4426950408889634f;

// Render-mode classes of the fragment stage (gau_frag.glsl:16-52).
enum FragClass : int { kFragGauss = 0, kFragBillboard = 1, kFragFlatBall = 2, kFragGaussBall = 3 };

__host__ __device__ constexpr int frag_class_of(int mode) {
    return (mode == -4 || mode == -1) ? kFragBillboard
           : mode == -5              ? kFragFlatBall
           : mode == -6              ? kFragGaussBall
                                     : kFragGauss;
}

// Everything the per-Gaussian stage needs, passed by value (kernarg).
struct FrameUniforms {
    float V[16];            // row-major view
    float P[16];            // row-major projection
    float hfov[3];          // tan(fovx/2), tan(fovy/2), focal
    float campos[3];
    float gsf;              // gaussian_scale_factor
    float sdsf;             // screen_display_scale_factor
    float dc_factor, extra_factor;
    float cscale[3];
    float rotmod[4];        // (x,y,z,w)
    float lcos[3], lsin[3]; // light rotation cos/sin per axis
    float pcenter[3];
    float obb_inv[9];       // row-major inverse(cube_rotation)
    float cmin[3], cmax[3];
    int32_t enable_aabb, enable_obb;
    int32_t render_mod;
    int32_t sh_dim;         // floats of SH per Gaussian (3, 12, 27, 48)
    int32_t width, height;
    int32_t tiles_x, tiles_y;
    int32_t plain_rec;      // records in plain form (GSR_BLEND_UNORM8), not interval form (SplatRec)
};

struct SceneData {
    int64_t n = 0;
    int32_t sh_dim = 0;
    int32_t sh_planes = 0;      // ceil(sh_dim/4) float4 planes
    float4* pos_op = nullptr;   // (x, y, z, opacity)            [n]
    float4* rot = nullptr;      // (w, x, y, z)                  [n]
    float4* scale = nullptr;    // (sx, sy, sz, 0)               [n]
    float4* sh = nullptr;       // plane p at sh + p*n           [planes][n]
    void* block = nullptr;      // single allocation backing all of the above
};

// ---------------------------------------------------------------- helpers
std::string& last_error_ref();
int set_error(int code, const std::string& msg);

#define GSR_HIP_CHECK(expr)                                                      \
    do {                                                                         \
        hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess)                                                    \
            return ::gsr::set_error(GSR_ERR_HIP, std::string(#expr) + ": " +    \
                                                     hipGetErrorString(e_));     \
    } while (0)

#define GSR_LAUNCH_CHECK(what)                                                   \
    do {                                                                         \
        hipError_t e_ = hipGetLastError();                                       \
        if (e_ != hipSuccess)                                                    \
            return ::gsr::set_error(GSR_ERR_HIP, std::string("launch ") + what + \
                                                     ": " + hipGetErrorString(e_)); \
    } while (0)

// ---------------------------------------------------------------- device utils
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = __lane_id();
    return (l == 0) ? 0ull : (~0ull >> (64 - l));
}

// Lanes of the wave holding the same 8-bit digit (only `valid` lanes).
__device__ __forceinline__ uint64_t match_digit8(uint32_t digit, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const bool bit = (digit >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

// Inclusive wave scan (64 lanes) with DPP lane moves, no LDS round trips (a
// __shfl_up is a ds_bpermute: six dependent LDS trips per scan):
// row_shr:1/2/4/8 scan each 16-lane row, then row_bcast:15 adds row 0's total
// to row 1 and row 2's to row 3, and row_bcast:31 adds lane 31's (rows 0-1)
// to rows 2-3.  Lanes a DPP move has no source for (or rows it masks off)
// read `old` = 0.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_move0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    v += dpp_move0<0x111>(v);        // row_shr:1
    v += dpp_move0<0x112>(v);        // row_shr:2
    v += dpp_move0<0x114>(v);        // row_shr:4
    v += dpp_move0<0x118>(v);        // row_shr:8
    v += dpp_move0<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
    v += dpp_move0<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Unsigned max over the wave, in every lane: the same DPP prefix pattern with
// max (a lane with no DPP source reads 0, the identity of unsigned max).
__device__ __forceinline__ uint32_t wave_reduce_max(uint32_t v) {
    v = max(v, dpp_move0<0x111>(v));
    v = max(v, dpp_move0<0x112>(v));
    v = max(v, dpp_move0<0x114>(v));
    v = max(v, dpp_move0<0x118>(v));
    v = max(v, dpp_move0<0x142, 0xa>(v));
    v = max(v, dpp_move0<0x143, 0xc>(v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Sum over the wave, in every lane (the scan's last lane, broadcast).
__device__ __forceinline__ uint32_t wave_reduce_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_inclusive_scan(v), 63);
}

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

// ---------------------------------------------------------------- radix digits
// One pass of the LSD radix sort (radix_sort.hip; also the tile sort's pass 0
// fused into the binning, composite.hip).
struct PassArgs {
    const uint32_t* key_range;  // device {~kmin, kmax} or null (then kmin = 0 and B = bits)
    uint32_t bits;
    uint32_t passes;
    uint32_t pass;
    // the first pass over the fused cull's slots (launch_preprocess_fc): all n
    // keys are read (not the device count) and keys outside {kmin, kmax}
    // (culled slots, key 0xffffffff) are dropped; later passes see only V
    uint32_t drop = 0;
    // Coarse depth order (the frame's depth sort): only the top `coarse` bits
    // of the B-bit key range are sorted (0: all B).  Equal coarse keys keep
    // their input (slot) order; tile_ranges restores the exact order inside
    // each tile's list (RunFix).
    uint32_t coarse = 0;
};

struct Digit {
    uint32_t kmin, shift, w, mask;
    uint32_t lim;  // kept keys: key - kmin <= lim (PassArgs::drop)
    __device__ __forceinline__ uint32_t of(uint32_t key) const { return ((key - kmin) >> shift) & mask; }
    __device__ __forceinline__ bool keep(uint32_t key) const { return key - kmin <= lim; }
};

__device__ __forceinline__ Digit digit_params(const PassArgs& p) {
    Digit d;
    uint32_t B, s0 = 0;
    if (p.key_range) {
        d.kmin = ~p.key_range[0];
        const uint32_t kmax = p.key_range[1];
        B = kmax > d.kmin ? 32u - (uint32_t)__clz(kmax - d.kmin) : 0u;
        // an empty range ({0, 0}: nothing visible) keeps no key: every slot is then culled (0xffffffff)
        d.lim = kmax >= d.kmin ? kmax - d.kmin : 0xfffffffeu;
        if (kmax < d.kmin) d.kmin = 0u;
        if (p.coarse && B > p.coarse) {
            s0 = B - p.coarse;
            B = p.coarse;
        }
    } else {
        d.kmin = 0u;
        d.lim = 0xffffffffu;
        B = p.bits;
    }
    d.w = max(1u, (B + p.passes - 1u) / p.passes);
    d.shift = s0 + p.pass * d.w;
    d.mask = (1u << d.w) - 1u;
    return d;
}

// kmin and the coarse shift of the frame's depth sort (digit_params, PassArgs::coarse)
// (0 also for an exact sort, coarse == 0: nothing to repair)
__device__ __forceinline__ uint32_t coarse_shift(const uint32_t* key_range, uint32_t coarse, uint32_t& kmin) {
    kmin = ~key_range[0];
    const uint32_t kmax = key_range[1];
    const uint32_t B = kmax > kmin ? 32u - (uint32_t)__clz(kmax - kmin) : 0u;
    if (kmax < kmin) kmin = 0u;
    return coarse && B > coarse ? B - coarse : 0u;
}

// Lanes of the wave holding the same w-bit digit (only `valid` lanes).
// Per digit bit: the ballot m, then each lane keeps the lanes that agree with
// it: p &= ~(m ^ t), t = the lane's bit as 0 / all ones (a sign-extended bit
// field; one 3-input bit op per 32-bit half: 4 VALU per bit, against 8 for
// `p &= bit ? m : ~m` as the compiler emitted it).
__device__ __forceinline__ uint64_t match_digit(uint32_t digit, uint32_t w, bool valid) {
    const uint64_t v = __ballot(valid);
    uint32_t plo = (uint32_t)v, phi = (uint32_t)(v >> 32);
    for (uint32_t b = 0; b < w; ++b) {
        const uint32_t t = (uint32_t)__builtin_amdgcn_sbfe((int)digit, (int)b, 1);
        const uint64_t m = __ballot(t != 0u);
        plo &= ~((uint32_t)m ^ t);
        phi &= ~((uint32_t)(m >> 32) ^ t);
    }
    return ((uint64_t)phi << 32) | plo;
}

// ---------------------------------------------------------------- host launchers
// scan.hip: exclusive scan of n uint32 (in may equal out). Writes the total to
// *total_dev (device) when non-null. tmp must hold scan_tmp_elems(n) uint32.
// Optionally also reduces n_kr key ranges {~kmin, kmax} (componentwise max)
// into kr_out[0..1].
size_t scan_tmp_elems(size_t n);
int scan_exclusive(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp,
                   uint32_t* total_dev, hipStream_t s, const uint2* kr_in = nullptr,
                   size_t n_kr = 0, uint32_t* kr_out = nullptr);
// The same for k views' arrays of n elements each in one launch (n <= 16384:
// scan_views_fits), key ranges reduced alongside (kr_in/kr_out per view).
bool scan_views_fits(size_t n);
int scan_exclusive_views(const uint32_t* const* in, uint32_t* const* out, size_t n, uint32_t* const* total_dev,
                         const uint2* const* kr_in, size_t n_kr, uint32_t* const* kr_out, int k, hipStream_t s);

// radix_sort.hip: stable LSD sort of (key, val), `passes` passes of
// w = ceil(B / passes) <= 11 bits, where B = `bits` (keys < 2^bits) or, when
// key_range (device {~kmin, kmax}) is given, B = bits(kmax - kmin) chosen on
// the device (keys are then sorted as key - kmin).  Buffers are ping-ponged;
// the sorted result ends in (*keys_io, *vals_io) (pointers swapped as needed).
// identity_vals: vals = 0..n-1 (vals_io not read).  n_dev (nullable):
// device-side element count <= n (grids are sized by n).  tmp holds
// radix_tmp_elems(n) uint32, totals radix_totals_elems() uint32.
// The same sort for several views at once (one launch per step for all of
// them, view = blockIdx.y); every view sorts n_host keys (its device count
// n_dev bounds the work), same bits/passes; each has its own buffers.
struct RadixViewArgs {
    uint32_t** keys_io;
    uint32_t** vals_io;
    uint32_t** keys_alt;
    uint32_t** vals_alt;
    const uint32_t* n_dev;
    const uint32_t* key_range;
    uint32_t* tmp;
    uint32_t* totals;
    const uint2* rect_in = nullptr;  // payload (see radix_sort_pairs): on every view or none
    uint32_t** pay_io = nullptr;
    uint32_t** pay_alt = nullptr;
    bool drop_first = false;  // see radix_sort_pairs
    uint32_t coarse = 0;      // see PassArgs::coarse
    bool keys_last = true;    // the last pass writes the sorted keys (else keys_io keeps its input)
};
int radix_sort_pairs_views(RadixViewArgs* views, int k, bool identity_vals, size_t n, int bits, int passes,
                           hipStream_t s, int first_pass = 0);
// Pass p's digit offsets from a digit-major count matrix hist[d * ntiles + tile]
// produced by another kernel (the tile sort's pass 0 counted by the binning):
// exclusive per-digit prefix over tiles in place, digit totals to `totals`.
int radix_offsets(uint32_t* hist, uint32_t ntiles, int bits, int passes, int pass, uint32_t* totals,
                  hipStream_t s);
// The same for k views (hist[v], totals[v]; each view's ntiles rows).
int radix_offsets_views(uint32_t* const* hist, uint32_t* const* totals, int k, uint32_t ntiles, int bits,
                        int passes, int pass, hipStream_t s);
size_t radix_tmp_elems(size_t n);
size_t radix_totals_elems();
int radix_passes_for(int bits);
int radix_sort_pairs(uint32_t** keys_io, uint32_t** vals_io, uint32_t** keys_alt,
                     uint32_t** vals_alt, bool identity_vals, size_t n, const uint32_t* n_dev,
                     int bits, int passes, const uint32_t* key_range, uint32_t* tmp,
                     uint32_t* totals, hipStream_t s, const uint2* rect_in = nullptr,
                     uint32_t** pay_io = nullptr, uint32_t** pay_alt = nullptr, int first_pass = 0,
                     bool drop_first = false, uint32_t coarse = 0, bool keys_last = true);
// drop_first (needs key_range): the keys are the fused cull's n slots; the
// first pass reads all n and drops the culled ones (PassArgs::drop), later
// passes run over the device count n_dev = V.
// Payload (rect_in non-null): the tile rectangles rect_in[n] (uint2, in the
// input order) travel with the pairs packed to 32 bits (pack_rect: frames of
// at most 256 x 256 tiles); the sorted packed rectangles end in *pay_io.
constexpr int kPackedRectTiles = 256;

// scene.hip
int scene_repack_from_fields(SceneData& sd, const float* xyz, const float* rot,
                             const float* scale, const float* opacity, const float* sh,
                             hipStream_t s);
int scene_repack_from_flat(SceneData& sd, const float* flat, hipStream_t s);
// the SoA planes back to a flat [n, 11 + sh_dim] device array
int scene_unpack_flat(const SceneData& sd, float* flat, hipStream_t s);
// PLY load (gsr_scene_load_ply): load_ply's activations on raw flat rows, then
// (interval > 0) scale_data: keys = 6 uint32 scratch, out4 = (centre, factor)
// device floats; xyz [n,3] receives the final positions (for points_center).
int ply_activate_flat(float* flat, int64_t n, int sh_dim, float interval, uint32_t* keys, float* out4, float* xyz,
                      hipStream_t s);
// export.hip: points_center = np.mean(xyz, axis=0), bit-exact, into out3 (device)
int launch_points_center(const float* xyz, int64_t n, float* out3, hipStream_t s);
// ply.cpp: the raw (pre-activation) vertex rows of a PLY streamed into a new
// device array flat [n, 11 + sh_dim] (hipMalloc'd; the caller frees it):
// chunks parsed by host threads into pinned buffers, copied while the next
// chunk is parsed.
int ply_stream_flat(const char* path, int32_t n_threads, hipStream_t s, float** flat_dev, int64_t* n, int32_t* sh_dim);

// preprocess.hip
// k_cull also zeroes n_zero words at zero_words (the frame's zero block) and
// writes per block of kCullBlock Gaussians the depth-key range {~kmin, kmax}
// of its visible ones ({0, 0} if none) to block_ranges.
constexpr int kCullBlock = 256;
int launch_cull(const SceneData& sd, const FrameUniforms& u, uint64_t* vis_mask,
                uint32_t* wave_counts, uint2* block_ranges, uint32_t* zero_words, uint32_t n_zero,
                hipStream_t s);
// counters[0] = V (input), counters[1] = D (written by the last block, which
// also stores (V, D, seq) to host-mapped host_counters and re-arms done_ctr).
int launch_preprocess(const SceneData& sd, const FrameUniforms& u, const uint64_t* vis_mask,
                      const uint32_t* wave_off, const uint32_t* n_vis_dev, SplatRec* recs,
                      uint32_t* depth_keys, uint2* trect, uint32_t* counters,
                      unsigned long long* done_ctr, uint32_t* host_counters, uint32_t seq,
                      int32_t* radii, hipStream_t s);
int launch_depth_keys_all(const SceneData& sd, const float* V, uint32_t* keys, hipStream_t s);

// Several views of one scene (gsr_render_begin_views): one pass over the scene.
struct ViewCullArgs {
    const FrameUniforms* u;
    uint64_t* vis_mask;
    uint32_t* wave_counts;
    uint2* block_ranges;
    uint32_t* zero_words;
    uint32_t n_zero;
};
struct ViewPreArgs {
    const FrameUniforms* u;
    const uint64_t* vis_mask;
    const uint32_t* wave_off;
    const uint32_t* n_vis_dev;
    SplatRec* recs;
    uint32_t* depth_keys;
    uint2* trect;
    uint32_t* counters;
    unsigned long long* done_ctr;
    uint32_t* host_counters;
    int32_t* radii;
    uint32_t seq;
};
int launch_cull_views(const SceneData& sd, const ViewCullArgs* views, int k, hipStream_t s);
int launch_preprocess_views(const SceneData& sd, const ViewPreArgs* views, int k, hipStream_t s);

// Culling fused into the preprocess (no k_cull, no scan): Gaussian i owns
// slot n-1-i (a culled slot: key 0xffffffff, empty rect); the last block
// writes counters[0] = V, counters[1] = D and key_range {~kmin, kmax} of the
// visible keys, publishes (V, D, seq) to host_counters and re-arms done_ctr
// (kDoneCtrWords words: completion, then key-range and count shards).
// Every block also clears zero_words[0, n_zero) (sc1 stores).
constexpr size_t kDoneCtrWords = 1 + 3 * 64;
int launch_preprocess_fc(const SceneData& sd, const FrameUniforms& u, SplatRec* recs, uint32_t* depth_keys,
                         uint2* trect, uint32_t* counters, uint32_t* key_range, uint32_t* zero_words, uint32_t n_zero,
                         unsigned long long* done_ctr, uint32_t* host_counters, uint32_t seq, int32_t* radii,
                         hipStream_t s);
struct ViewPreFcArgs {
    const FrameUniforms* u;
    SplatRec* recs;
    uint32_t* depth_keys;
    uint2* trect;
    uint32_t* counters;
    uint32_t* key_range;
    uint32_t* zero_words;
    unsigned long long* done_ctr;
    uint32_t* host_counters;
    int32_t* radii;
    uint32_t n_zero;
    uint32_t seq;
};
int launch_preprocess_fc_views(const SceneData& sd, const ViewPreFcArgs* views, int k, hipStream_t s);

// composite.hip
size_t bin_tmp_elems(size_t n_vis);
// trect_sorted: n_vis uint2 of scratch (the rects in depth order)
// rect4_sorted (nullable): the packed rects in depth order (the depth sort's
// payload); else the rects are gathered by id from trect
// stage_limit: blocks with at most this many instances stage them in LDS (capped at the build's kBinStage)
uint32_t clamp_stage_limit(long v);
int launch_binning(const uint32_t* sorted_ids, const uint2* trect, const uint32_t* rect4_sorted, uint32_t n_vis,
                   int tiles_x, uint32_t* tmp, uint2* trect_sorted, uint32_t* tile_keys, uint32_t* tile_vals,
                   uint32_t stage_limit, hipStream_t s);
// Repair of a coarse depth order inside the tile lists (k_tile_ranges): runs of
// one tile's instances with equal coarse depth keys are put in (full key, slot)
// order, in place.  coarse == 0 (an exact depth sort): nothing to repair.
// Runs longer than kFixRunMax that reach past a thread's register window are
// not repaired there: their starts go to long_starts (*long_count, zeroed per
// frame) and launch_long_runs sorts them (long_runs.h).
struct RunFix {
    uint32_t* vals;             // the tile list (slots), repaired in place
    const uint32_t* key_range;  // the frame's {~kmin, kmax}
    uint32_t coarse;
    uint32_t* scratch_keys;     // n_dup words each, free at this point (the tile sort's alternates): the long runs' global path
    uint32_t* scratch_vals;
    uint32_t* inst_keys = nullptr;     // each list position's depth key (binning + tile sort payload)
    uint32_t* long_starts = nullptr;   // long_runs_elems(n_dup) words: long_run_cap starts, then their lengths
    uint32_t* long_count = nullptr;
};
// runs repaired by one thread (O(L^2) steps, L + 1 serial scan loads) at most this long
constexpr uint32_t kFixRunMax = 16;
inline size_t long_run_cap(size_t n_dup) { return n_dup / (kFixRunMax + 1) + 1; }
inline size_t long_runs_elems(size_t n_dup) { return 2 * long_run_cap(n_dup); }
int launch_tile_ranges(const uint32_t* tile_keys, uint32_t n_dup, uint2* ranges, const RunFix& fix,
                       hipStream_t s);
// long_runs.h: the coarse order's long runs (RunFix::long_starts), each
// bounded by a 64-way search from its start (runs are stretches of one tile's
// list with equal coarse key, ranges[tile] bounds them) and sorted by (full
// key, slot) on chip: up to 1024 instances by one wave, up to 24576 by a
// 1024-thread block in registers, longer ones by a block through the scratch
// buffers.  A fixed grid takes the listed runs in turn and exits at once when
// there are none (a launch of its own; launch_chunks takes them as extra blocks).
int launch_long_runs(const uint32_t* tile_keys, uint32_t n_dup, const uint2* ranges, const RunFix& fix,
                     hipStream_t s);
// The binning with the tile sort's first radix pass fused in (composite.hip,
// k_bin_hist / k_bin_scatter): the instances end in (tile_keys, tile_vals)
// ordered by digit 0 of the tile sort (tbits bits in `passes` passes); the
// sort then continues from pass 1 (radix_sort_pairs first_pass = 1).  hist
// holds bin_hist_elems(n_vis, tbits, passes) uint32, totals
// radix_totals_elems().  tbits = 0 (one tile): generation order.
size_t bin_hist_elems(size_t n_vis, int tbits, int passes);
int launch_binning_sorted(const uint32_t* sorted_ids, const uint2* trect, const uint32_t* rect4_sorted,
                          uint32_t n_vis, int tiles_x, int tbits, int passes, uint32_t* hist, uint32_t* totals,
                          uint2* trect_sorted, uint32_t* tile_keys, uint32_t* tile_vals, hipStream_t s,
                          const uint32_t* sorted_keys = nullptr, uint32_t* inst_keys = nullptr);
// chunk_cnt must hold chunk_cnt_elems(num_tiles) entries (block totals after the tiles);
// order: one entry per chunk (dispatch position -> chunk slot)
size_t chunk_cnt_elems(int num_tiles);
// classes (2 .. kMaxLenClasses): dispatch order = full chunks, then the partial
// ones in classes - 1 length classes, longest first; the frame's chunk count
// of each class lands at chunk_class_totals(chunk_cnt, num_tiles, classes)
// long_runs (nullable): the frame's coarse-order long runs, sorted by extra
// blocks of the chunk-count launch (in place of launch_long_runs)
struct LongRuns {
    const uint32_t* tile_keys;
    uint32_t n_dup;
    RunFix fix;
};
int launch_chunks(const uint2* ranges, int num_tiles, uint32_t chunk, uint32_t classes, uint32_t* chunk_cnt,
                  uint32_t* chunk_base, uint32_t* n_extra_dev, uint4* desc, uint32_t* order, float4* tmax,
                  hipStream_t s, bool first_major = false, const LongRuns* long_runs = nullptr,
                  uint32_t max_extra = 0xffffffffu);  // (an upper bound of the extra chunks: n_dup / chunk)
const uint32_t* chunk_class_totals(const uint32_t* chunk_cnt, int num_tiles, uint32_t classes);
int launch_composite(const uint4* desc, const uint32_t* order, const uint32_t* n_chunks_dev, uint32_t max_chunks,
                     const uint32_t* chunk_cnt, const uint32_t* chunk_base, uint32_t* sat,
                     const uint32_t* tile_vals, const SplatRec* recs, const FrameUniforms& u,
                     int frag_class, float t_min, const float* bg, int out_layout, float* out,
                     float4* partial, float4* tmax, bool tail_merge, hipStream_t s);
// GSR_BLEND_UNORM8: one wave per tile, back to front, 8-bit rounding after every blend
int launch_composite_unorm8(const uint2* ranges, const uint32_t* tile_list, const SplatRec* recs,
                            const FrameUniforms& u, int frag_class, const float* bg, int out_layout, float* out,
                            hipStream_t s);
// k_merge: folds the partials of multi-chunk tiles into `out` (after launch_composite)
// (tail_merge: the compositing launch folded the tiles; nothing is launched)
int launch_merge(const uint32_t* chunk_cnt, const uint32_t* chunk_base, const float4* partial, const uint32_t* sat,
                 const FrameUniforms& u, float t_min, const float* bg, int out_layout, float* out, bool tail_merge,
                 hipStream_t s);

// The second half of a group of views' frames (gsr_render_finish_views): each
// stage is one launch for the whole group (view = blockIdx.y); grids cover the
// largest view and the blocks past a view's own size exit.  All views share
// the frame size, t_min, background, output layout and chunk length.
struct FinishView {
    // binning (n_vis, n_dup: this view's exact counts)
    const uint32_t* sorted_ids;
    const uint2* trect;
    const uint32_t* rect4_sorted;  // nullable, on every view or none (launch_binning)
    uint32_t n_vis, n_dup;
    uint32_t* bin_tmp;
    uint2* trect_sorted;
    uint32_t* tile_keys;  // tile-sorted (keys, vals) after the tile sort
    uint32_t* tile_vals;
    RunFix fix;           // coarse depth order repair (vals, scratch set after the tile sort)
    // chunks, composite, merge
    uint2* ranges;
    uint32_t* chunk_cnt;
    uint32_t* chunk_base;
    uint32_t* n_extra_dev;
    uint4* desc;
    uint32_t* order;
    float4* tmax;
    uint32_t* sat;
    const SplatRec* recs;
    float* out;
    float4* partial;
};
// binning: bin_tmp of each view holds its per-block instance counts
int launch_binning_views(FinishView* views, int k, int tiles_x, uint32_t stage_limit, hipStream_t s);
// ... and with the tile sort's pass 0 fused in (hist[v], totals[v] per view)
int launch_binning_sorted_views(FinishView* views, uint32_t* const* hist, uint32_t* const* totals, int k, int tiles_x,
                                int tbits, int passes, hipStream_t s);
int launch_tile_ranges_views(FinishView* views, int k, hipStream_t s);
// first_major: every tile's first chunk dispatched before any later chunk
int launch_chunks_views(FinishView* views, int k, int num_tiles, uint32_t chunk, uint32_t classes, bool first_major,
                        hipStream_t s);
// interleave: dispatch class-major over the views (k * classes <= 64), else view after view
// stamps (nullable, profiling): the launch writes, by plain stores, every
// block's start clock ([blocks]) and then every wave's end clock
// ([blocks * composite_views_waves_per_block()]) of the 100 MHz constant
// clock (s_memrealtime).  debug_handoff: the tail merge's test knob (0).
int launch_composite_views(FinishView* views, int k, uint32_t max_chunks, uint32_t classes, bool first_major,
                           bool interleave, const FrameUniforms& u, int frag_class, float t_min, const float* bg,
                           int out_layout, bool tail_merge, uint32_t debug_handoff, hipStream_t s,
                           uint64_t* stamps = nullptr);
// Blocks of one launch_composite_views launch, and its waves per block (the
// build's GSR_COMP_THREADS / 64): a launch's stamps take blocks * (1 + waves) words.
size_t composite_views_blocks(uint32_t max_chunks, int k);
int composite_views_waves_per_block();
int launch_merge_views(FinishView* views, int k, const FrameUniforms& u, float t_min, const float* bg,
                       int out_layout, bool tail_merge, hipStream_t s);

}  // namespace gsr

struct gsr_scene {
    gsr::SceneData d;
    int device = 0;
};

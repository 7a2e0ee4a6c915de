// C ABI (include/gsr.h): scene lifetime, frame workspace, render orchestration.
//
// Frame pipeline on one stream (N = Gaussians, V = visible, D = instances):
//   memset(per-frame zero block: counters, radix totals, tile ranges, saturation words)
//   k_cull(N) -> scan(N/64 wave counts; total = V on device)
//   k_preprocess(N): records, depth keys, tile rects; D accumulated on device
//   (the last preprocess block stores (V, D, seq) to host-mapped memory)
//   depth radix sort (grid sized by N, count V and key range read on device), 3 passes
//   [host polls for (V, D, seq) while the GPU runs the depth sort]
//   binning (reduce, scan, fused scan+write) -> stable tile radix sort over D
//   k_tile_ranges -> chunk count / scan / write -> k_composite(chunks) -> k_merge
// The only host wait overlaps GPU work, so no stage of the frame idles.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "gsr_internal.h"
#include "gsr_io.h"

namespace gsr {

std::string& last_error_ref() {
    static thread_local std::string s;
    return s;
}

int set_error(int code, const std::string& msg) {
    last_error_ref() = msg;
    return code;
}

// A caller-provided workspace (gsr_context_attach_workspace), or with
// `measure` set the sizing pass of gsr_workspace_size: a context's buffers are
// carved off it in order, 256-B aligned, and nothing is returned to it.
struct Arena {
    char* base = nullptr;
    size_t bytes = 0;
    size_t used = 0;
    bool measure = false;
    bool sealed = false;  // attached and sized: a buffer outgrowing its reservation fails instead of carving more
};
constexpr size_t kArenaAlign = 256;

namespace {

// A context-owned device array that grows on demand.  Growth never frees the
// old allocation: hipFree synchronises the whole device, which would stall
// every other view in flight, and the context's previous frame may still read
// the old block.  Retired blocks are freed with the context (release()).
// gsr_context_reserve sizes everything up front, so a steady state never grows.
// With an arena (caller workspace) the blocks come from it instead, and a
// buffer that outgrows it fails the call with GSR_ERR_NOMEM.
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;  // elements
    int64_t allocs = 0;  // allocations made (gsr_context_workspace)
    std::vector<void*> retired;
    Arena* arena = nullptr;
    int ensure(size_t n, const char* what) {
        if (n <= cap && p) return GSR_OK;
        size_t want = n < 64 ? 64 : n + n / 8;  // 12.5% headroom against regrowth
        T* q = nullptr;
        if (arena && arena->sealed)
            return set_error(GSR_ERR_NOMEM, std::string("context: ") + what +
                                                " exceeds the bounds the caller's workspace was attached for");
        if (arena) {
            const size_t off = (arena->used + kArenaAlign - 1) & ~(kArenaAlign - 1);
            const size_t end = off + want * sizeof(T);
            if (!arena->measure && end > arena->bytes)
                return set_error(GSR_ERR_NOMEM, std::string("context: the caller's workspace (") +
                                                    std::to_string(arena->bytes) + " B) is too small for " + what +
                                                    " (gsr_workspace_size gives the bytes a bound needs)");
            arena->used = end;
            // measuring: a stand-in address that is never dereferenced
            q = arena->measure ? reinterpret_cast<T*>((uintptr_t)(kArenaAlign + off))
                               : reinterpret_cast<T*>(arena->base + off);
        } else if (hipMalloc(&q, want * sizeof(T)) != hipSuccess) {
            return set_error(GSR_ERR_NOMEM, std::string("context: hipMalloc failed for ") + what);
        }
        if (p && !arena) retired.push_back(p);
        p = q;
        cap = want;
        ++allocs;
        return GSR_OK;
    }
    size_t bytes() const { return cap * sizeof(T); }
    void release() {
        if (arena) {  // the caller owns the memory
            p = nullptr;
            cap = 0;
            return;
        }
        if (p) (void)hipFree(p);
        for (void* r : retired) (void)hipFree(r);
        retired.clear();
        p = nullptr;
        cap = 0;
    }
};

}  // namespace
}  // namespace gsr

namespace gsr {
// A frame between gsr_render_begin and gsr_render_finish.
struct PendingFrame {
    bool active = false;
    uint32_t coarse = 0;  // its depth sort's coarse bits (0: exact), for the run repair
    FrameUniforms u{};
    float t_min = 0.f;
    float bg[3] = {0.f, 0.f, 0.f};
    int32_t out_layout = 0;
    int32_t blend = GSR_BLEND_FLOAT;
    float* out = nullptr;
    hipStream_t stream = nullptr;
    size_t n = 0;
    int slot = 0;
    uint32_t *ka = nullptr, *va = nullptr, *kb = nullptr, *vb = nullptr;  // depth sort buffers (result in ka/va)
    uint32_t *pa = nullptr, *pb = nullptr;  // packed tile rects carried by the depth sort (result in pa)
    bool packed = false;                    // the depth sort carries them (frames of <= 256 x 256 tiles)
    bool sort_ready = false;  // gsr_render_begin_views done, gsr_render_begin_sort not yet
};
}  // namespace gsr

// compositing launches whose in-kernel spans one profiling run can record
constexpr size_t kSpanLaunches = 64;

// depth sort passes of a frame rendered alone (gsr_render; see kDepthPasses)
constexpr int kDepthPassesAlone = 3;
// Coarse depth order (round 4): a frame alone's depth sort (gsr_render_begin)
// orders only the top 16 bits of its key range, 2 passes of 8 against 3 exact
// passes of <= 9 (depth sort 76 -> 51 us), and keeps equal coarse keys in slot
// order.  Only each tile's list needs the exact (key, slot) order: the
// binning and the tile sort carry each instance's full depth key, and
// k_tile_ranges restores the order run by run (RunFix; runs that outgrow its
// register window go to k_long_runs, long_runs.h).  Needs the fused binning
// (which carries the keys; GSR_BIN_FUSED=0 sorts exactly).  A group's frames
// (gsr_render_begin_views / _sorts / _finish_views) keep the exact sort (4
// passes of <= 8 bits): in flight the sort's VALU work is the same in 3 or 4
// passes and the repair only costs (0.1356-0.1365 vs 0.1332-0.1353 ms per frame
// with 3 passes of 8), and one depth order for the group's paths keeps each
// finish reading what its sort step left.  With a coarse sort the
// frame's global depth order (GSR_DEBUG_DEPTH_ORDER) is the coarse one;
// gsr_sort_depth stays exact.
constexpr uint32_t kDepthCoarseAlone = 16;
// ... for scenes of at most kCoarseMaxN Gaussians.  Above it the run repair and the keys the binning and the tile
// sort carry cost more (they scale with the instances) than the two passes save, and a frame alone sorts exactly in
// kDepthPassesBigAlone passes of <= 8 bits (round 6, profiles/r6_s11: C3 alone 1.244 -> 1.195 ms; 3 passes of <= 11
// bits: 1.259; c2h and C5, 1M Gaussians, within 1 % either way; C2 coarse 0.309 against 0.327 exact, r6_s12)
constexpr size_t kCoarseMaxN = (size_t)1 << 21;
constexpr int kDepthPassesBigAlone = 4;
constexpr uint32_t kDepthCoarseMax = 16;  // 2 passes of <= 8 bits: the last pass's keys are the carried ones

struct gsr_context {
    gsr::DevBuf<uint64_t> vis_mask;
    gsr::DevBuf<uint32_t> wave_counts;
    gsr::DevBuf<uint2> block_ranges;                        // per cull block: depth-key range
    gsr::DevBuf<uint32_t> scan_tmp;
    gsr::DevBuf<gsr::SplatRec> recs;
    gsr::DevBuf<uint32_t> keys_a, keys_b, vals_a, vals_b;   // depth sort (capacity N)
    gsr::DevBuf<uint2> trect;                               // per record: packed tile rectangle
    gsr::DevBuf<uint2> trect_sorted;                        // the same, in depth order (binning)
    gsr::DevBuf<uint32_t> rect4_a, rect4_b;                 // packed rects, depth sort payload
    gsr::DevBuf<uint32_t> bin_tmp;                          // binning block offsets
    gsr::DevBuf<uint32_t> tkeys_a, tkeys_b, tvals_a, tvals_b;  // tile sort (capacity D)
    gsr::DevBuf<uint32_t> radix_tmp;
    gsr::DevBuf<uint32_t> zero;                   // per-frame zeroed block (see zero_layout)
    gsr::DevBuf<uint32_t> chunk_cnt, chunk_base;  // per tile
    gsr::DevBuf<uint4> chunk_desc;                // per chunk
    gsr::DevBuf<uint32_t> chunk_order;            // per chunk: dispatch position -> chunk slot
    gsr::DevBuf<float4> partial;                  // per chunk x 256 px (multi-chunk tiles)
    gsr::DevBuf<float4> tmax;                     // per chunk: published slice maxima of local T
    uint32_t chunk = 192;                         // instances per compositing chunk of a frame finished alone
                                                  // (gsr_render / gsr_render_finish): latency (r2_s17 sweep)
    uint32_t chunk_target = 16384;                // a frame alone with many instances: chunks of at least
                                                  // n_dup / chunk_target (rounded up to 64; at most
                                                  // chunk_views), 0: `chunk` always (frame_chunk).  16384:
                                                  // C3 704-instance chunks (latency 1.56 -> 1.40 ms), c2h 320
                                                  // (0.80 -> 0.66), C2 / C5 unchanged (profiles/r5_s17, r5_s20)
    uint32_t chunk_views = 3072;                  // ... of a group's frames (gsr_render_finish_views): with
                                                  // views in flight the other views fill the chip while a
                                                  // deep tile's long chunk runs, so few chunks (fewer partials,
                                                  // merges, descriptors) win (r2_s28 sweep)
    uint32_t len_classes = 8;                     // compositing dispatch order: full chunks, then the partial
                                                  // ones in len_classes - 1 length classes, longest first
    bool views_interleave = true;                 // a group's compositing dispatch class-major over its views
    bool first_major = true;                      // ... every tile's first chunk before any later one
    bool first_major_alone = false;               // the same for a frame finished alone (gsr_render_finish)
    bool chunk_single = false;                    // a frame alone's chunk descriptors by one block when they fit
                                                  // (k_chunk_single; GSR_CHUNK_SINGLE=0: count + write launches)
    bool bound_alone = false;                     // every frame alone with t_min > 0 takes the deep form's
                                                  // first-major order and cross-chunk bound (GSR_BOUND_ALONE)
    bool bin_fused = true;                        // the tile sort's pass 0 fused into the binning (k_bin_scatter)
    bool tail_merge_group = true;                 // a group's multi-chunk tiles folded in the compositing launch
    bool tail_merge_alone = false;                // ... and a frame alone's (else k_merge)
    uint32_t bin_stage_limit = 0xffffffffu;       // blocks of at most this many instances stage them (build cap)
    uint32_t debug_handoff = 0;                   // tail-merge test knob (GSR_DEBUG_HANDOFF; 0 in production)
    bool fused_cull = true;                       // culling inside the preprocess (launch_preprocess_fc)
    int depth_passes_alone = kDepthPassesAlone;   // depth sort passes of gsr_render's frames
    int depth_passes_now = 0;                     // this frame's (0: kDepthPasses)
    // depth sort of a frame alone: the top bits of its key range, the exact order restored per tile list by
    // k_tile_ranges and k_long_runs (GSR_DEPTH_COARSE=0: every bit, depth_passes_alone)
    uint32_t depth_coarse_alone = kDepthCoarseAlone;
    gsr::DevBuf<uint32_t> tpay_a, tpay_b;  // the instances' depth keys through the tile sort (coarse order repair)
    gsr::DevBuf<uint32_t> long_runs;       // starts of the runs that outgrow the repair window (k_long_runs)
    bool rect_payload = true;              // the depth sort carries the packed tile rects (GSR_NO_RECT_PAYLOAD:
                                           // the binning gathers them by slot; A/B and test knob)
    // the forms the last finished frame took (gsr_context_knob "frame_*")
    bool last_packed = false, last_deep = false;
    uint32_t last_coarse = 0, last_chunk = 0;
    uint32_t* host_counters = nullptr;      // pinned, host-mapped: (V, D, seq) stored by the last preprocess block
    uint32_t seq = 0;                       // frame sequence number the host waits for
    uint32_t* host_counters_dev = nullptr;  // its device address
    gsr::DevBuf<unsigned long long> done_ctr;  // preprocess completion + instance count (self re-arming)
    bool done_armed = false;                   // done_ctr zeroed on a frame's stream (arm_done_ctr)
    gsr_frame_stats stats{};
    // last frame's result arrays (for gsr_debug_copy)
    const uint32_t* last_depth_order = nullptr;
    const uint32_t* last_tile_list = nullptr;
    int64_t last_tiles = 0;
    const uint2* last_ranges = nullptr;
    // profiling: 10 events per frame, two frames in flight
    bool prof_on = false;
    hipEvent_t ev[2][12] = {};
    bool ev_pending[2] = {false, false};
    int64_t frame_idx = 0;
    double acc_ms[GSR_NUM_STAGES] = {};
    gsr::PendingFrame pend;
    double host_ms[3] = {};  // host time in gsr_render: enqueue before the wait, the wait, enqueue after
    int64_t host_frames = 0;
    int64_t prof_frames = 0;
    // group profiling (gsr_context_set_profiling(ctx, 2) on a group's first
    // context): HIP events around each k_composite_views launch of the groups
    // this context leads, two launches in flight
    bool prof_group = false;
    hipEvent_t evg[2][2] = {};
    bool evg_pending[2] = {false, false};
    int evg_views[2] = {0, 0};
    int evg_slot = 0;
    double group_comp_ms = 0.0;
    int64_t group_launches = 0, group_views = 0;
    // ... and each launch's own span from in-kernel clock stamps (first block
    // start to last wave end): the kernel's execution, without the time its
    // dispatch waited on the stream behind other streams' work
    gsr::DevBuf<uint64_t> stamps;  // not in the workspace (profiling only): the launches' stamps, appended
    size_t stamp_used = 0;
    std::vector<std::pair<size_t, size_t>> spans;  // per recorded launch: (offset, blocks) in `stamps`
    bool failed = false;           // a wait timed out or the stream faulted: no further frames
    int64_t wait_timeout_ms = 2000;
    gsr::Arena arena;              // caller workspace (gsr_context_attach_workspace) or sizing pass
    bool has_arena = false;
};

namespace gsr {
namespace {
// Every device buffer of a context (workspace accounting and release).
template <typename F>
void each_buf(gsr_context* c, F&& f) {
    f(c->vis_mask); f(c->wave_counts); f(c->block_ranges); f(c->scan_tmp); f(c->recs);
    f(c->keys_a); f(c->keys_b); f(c->vals_a); f(c->vals_b); f(c->trect); f(c->trect_sorted);
    f(c->rect4_a); f(c->rect4_b); f(c->bin_tmp); f(c->tkeys_a); f(c->tkeys_b); f(c->tvals_a); f(c->tvals_b);
    f(c->tpay_a); f(c->tpay_b); f(c->long_runs);
    f(c->radix_tmp); f(c->zero); f(c->chunk_cnt); f(c->chunk_base); f(c->chunk_desc); f(c->chunk_order);
    f(c->partial); f(c->tmax); f(c->done_ctr);
}
}  // namespace
}  // namespace gsr

namespace gsr {
namespace {

int build_uniforms(const gsr_scene* sc, const gsr_camera* cam, const gsr_settings* st, FrameUniforms& u) {
    if (cam->width <= 0 || cam->height <= 0 || cam->width > 32768 || cam->height > 32768)
        return set_error(GSR_ERR_INVALID, "camera: width/height out of range");
    if (st->out_layout != 0 && st->out_layout != 1)
        return set_error(GSR_ERR_INVALID, "settings: out_layout must be 0 ([3,H,W]) or 1 ([H,W,3])");
    if (!(st->t_min >= 0.f && st->t_min < 1.f))
        return set_error(GSR_ERR_INVALID, "settings: t_min must be in [0, 1)");
    if (st->blend != GSR_BLEND_FLOAT && st->blend != GSR_BLEND_UNORM8)
        return set_error(GSR_ERR_INVALID, "settings: blend must be GSR_BLEND_FLOAT or GSR_BLEND_UNORM8");
    std::memcpy(u.V, cam->view, sizeof(u.V));
    std::memcpy(u.P, cam->proj, sizeof(u.P));
    std::memcpy(u.hfov, cam->hfovxy_focal, sizeof(u.hfov));
    std::memcpy(u.campos, cam->campos, sizeof(u.campos));
    u.gsf = st->scale_modifier;
    u.sdsf = st->screen_scale;
    u.dc_factor = st->dc_factor;
    u.extra_factor = st->extra_factor;
    std::memcpy(u.cscale, st->color_scale, sizeof(u.cscale));
    std::memcpy(u.rotmod, st->rot_modifier, sizeof(u.rotmod));
    for (int k = 0; k < 3; ++k) {
        // radians() in float32 (gau_vert.glsl:148), cos/sin once per frame
        const float rad = st->light_rotation[k] * (float)(M_PI / 180.0);
        u.lcos[k] = std::cos(rad);
        u.lsin[k] = std::sin(rad);
    }
    std::memcpy(u.pcenter, st->points_center, sizeof(u.pcenter));
    {
        // inverse(cube_rotation) (gau_vert.glsl:180) in double, once per frame
        const float* m = st->cube_rotation;
        double a[9];
        for (int k = 0; k < 9; ++k) a[k] = m[k];
        const double c00 = a[4] * a[8] - a[5] * a[7], c01 = a[5] * a[6] - a[3] * a[8], c02 = a[3] * a[7] - a[4] * a[6];
        const double det = a[0] * c00 + a[1] * c01 + a[2] * c02;
        if (st->enable_obb == 1 && !(std::fabs(det) > 0.0))
            return set_error(GSR_ERR_INVALID, "settings: cube_rotation is singular");
        const double id = det != 0.0 ? 1.0 / det : 0.0;
        const double inv[9] = {c00 * id, (a[2] * a[7] - a[1] * a[8]) * id, (a[1] * a[5] - a[2] * a[4]) * id,
                               c01 * id, (a[0] * a[8] - a[2] * a[6]) * id, (a[2] * a[3] - a[0] * a[5]) * id,
                               c02 * id, (a[1] * a[6] - a[0] * a[7]) * id, (a[0] * a[4] - a[1] * a[3]) * id};
        for (int k = 0; k < 9; ++k) u.obb_inv[k] = (float)inv[k];
    }
    std::memcpy(u.cmin, st->cube_min, sizeof(u.cmin));
    std::memcpy(u.cmax, st->cube_max, sizeof(u.cmax));
    u.enable_aabb = st->enable_aabb;
    u.enable_obb = st->enable_obb;
    u.render_mod = st->render_mod;
    u.sh_dim = sc->d.sh_dim;
    u.width = cam->width;
    u.height = cam->height;
    u.tiles_x = (cam->width + kTile - 1) / kTile;
    u.tiles_y = (cam->height + kTile - 1) / kTile;
    u.plain_rec = st->blend == GSR_BLEND_UNORM8;
    return GSR_OK;
}

// 32-bit depth keys: 4 passes of <= 8 bits (width chosen on the device: a
// camera's keys span ~24 bits, i.e. 6-bit digits).  3 passes of <= 11 bits
// are 4 us faster alone, but their kernels need LDS for 2048 digits; with
// views in flight the 8-bit kernels (28 KB per block, 5 blocks per CU beside
// the compositor) win: 0.194 -> 0.187 ms per frame (profiles/r2_s24).
#ifndef GSR_DEPTH_PASSES
#define GSR_DEPTH_PASSES 4
#endif
constexpr int kDepthPasses = GSR_DEPTH_PASSES;
// A frame rendered alone (gsr_render: begin + finish, nothing else in flight)
// sorts in 3 passes of <= 11 bits: its kernels' LDS competes with no other
// view's, and a pass costs more than the wider digits do (r2_s46: depth sort
// 83.6 -> 78 us, latency 0.383 -> 0.376 ms).

int bits_for(uint32_t v) {  // bits needed to represent values < v
    int b = 0;
    while (b < 32 && (1ull << b) < v) ++b;
    return b;
}

// Per-frame scratch block: [0,4) counters {V, D, extra chunks, -} are
// overwritten every frame; from `cleared` on, the depth-key range
// {~kmin, kmax}, the radix digit totals (depth sort, tile sort), the tile
// ranges (uint2, 16-B aligned), the saturation words (4 per tile), the chunk
// completion counters of the tail merge (1 per tile, right after the
// saturation words) and the count of the coarse order's long runs are
// zeroed by k_cull (or the fused preprocess, from `ranges` on).
struct ZeroLayout {
    size_t counters = 0, cleared = 4, key_range = 4, totals_depth = 8, totals_tile = 0, ranges = 0, sat = 0,
           long_runs = 0, total = 0;
    explicit ZeroLayout(int num_tiles) {
        const size_t tot = radix_totals_elems();
        totals_tile = totals_depth + tot;
        ranges = (totals_tile + tot + 3) & ~(size_t)3;
        sat = ranges + 2 * (size_t)num_tiles;
        long_runs = sat + 5 * (size_t)num_tiles;
        total = long_runs + 4;
    }
};

// Sizes the per-Gaussian buffers.  Enqueues nothing: the load-time callers
// (gsr_context_reserve, gsr_context_attach_workspace, the sort services) may
// pass any stream, so no device work may come from here (see arm_done_ctr).
int ensure_scene_buffers(gsr_context* c, size_t n) {
    const size_t nw = (n + 63) / 64 + 4;
    int rc;
    if (!c->fused_cull) {  // the separate cull's visibility masks and compaction scan
        if ((rc = c->vis_mask.ensure(nw, "vis_mask"))) return rc;
        if ((rc = c->wave_counts.ensure(nw, "wave_counts"))) return rc;
        if ((rc = c->block_ranges.ensure(n / kCullBlock + 1, "block_ranges"))) return rc;
        const size_t scan_need = std::max(scan_tmp_elems(nw), scan_tmp_elems(n));
        if ((rc = c->scan_tmp.ensure(scan_need, "scan_tmp"))) return rc;
    }
    if ((rc = c->recs.ensure(n, "recs"))) return rc;
    if ((rc = c->keys_a.ensure(n, "keys"))) return rc;
    if ((rc = c->keys_b.ensure(n, "keys"))) return rc;
    if ((rc = c->vals_a.ensure(n, "vals"))) return rc;
    if ((rc = c->vals_b.ensure(n, "vals"))) return rc;
    if ((rc = c->trect.ensure(n, "trect"))) return rc;
    if ((rc = c->trect_sorted.ensure(n, "trect_sorted"))) return rc;
    if ((rc = c->rect4_a.ensure(n, "rect4"))) return rc;
    if ((rc = c->rect4_b.ensure(n, "rect4"))) return rc;
    if ((rc = c->bin_tmp.ensure(bin_tmp_elems(n), "bin_tmp"))) return rc;
    if ((rc = c->radix_tmp.ensure(radix_tmp_elems(n), "radix_tmp"))) return rc;
    if ((rc = c->done_ctr.ensure(kDoneCtrWords, "done_ctr"))) return rc;
    if (c->has_arena && c->arena.measure) return GSR_OK;  // gsr_workspace_size: sizes only, no HIP call
    if (!c->host_counters) {
        if (hipHostMalloc(&c->host_counters, 4 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess) {
            c->host_counters = nullptr;
            return set_error(GSR_ERR_NOMEM, "context: hipHostMalloc failed");
        }
        std::memset(c->host_counters, 0, 4 * sizeof(uint32_t));
        GSR_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->host_counters_dev), c->host_counters, 0));
    }
    return GSR_OK;
}

// The completion counter is zeroed once, on the stream of the context's first
// frame, right before that frame's preprocess.  Zeroing it anywhere else (the
// caller's stream of a reservation, the null stream of a plain hipMemset)
// leaves the memset unordered against the non-blocking streams frames run on
// (torch's), and a preprocess counting on top of a memset still in flight
// never publishes its (V, D, seq).  Later frames need no zeroing: the last
// preprocess block re-arms the counter, and the host waits for it before the
// context's next frame begins.
int arm_done_ctr(gsr_context* c, hipStream_t s) {
    if (c->done_armed) return GSR_OK;
    GSR_HIP_CHECK(hipMemsetAsync(c->done_ctr.p, 0, kDoneCtrWords * sizeof(unsigned long long), s));
    c->done_armed = true;
    return GSR_OK;
}

// Event slots: 0 start | cull+scan | 1 | preprocess | 2 ~sync~ 3 | depth sort | 4 |
// counts+scan | 5 ~sync~ 6 | instance write | 7 | tile sort | 8 | ranges | 9 | composite | 10 | merge | 11
enum { EV_START = 0, EV_CULL, EV_PRE, EV_AFTER_SYNC1, EV_DSORT, EV_COUNTS, EV_AFTER_SYNC2, EV_DUPW, EV_TSORT,
       EV_RANGES_END_COMPOSITE_START, EV_COMPOSITE, EV_COUNT };

int prof_record(gsr_context* c, int slot, int ev, hipStream_t s) {
    if (!c->prof_on) return GSR_OK;
    GSR_HIP_CHECK(hipEventRecord(c->ev[slot][ev], s));
    return GSR_OK;
}

void prof_accumulate(gsr_context* c, int slot, bool wait) {
    if (!c->ev_pending[slot]) return;
    hipEvent_t* e = c->ev[slot];
    if (wait) (void)hipEventSynchronize(e[EV_COUNT]);
    else if (hipEventQuery(e[EV_COUNT]) != hipSuccess) return;
    auto el = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e[a], e[b]);
        return (double)ms;
    };
    c->acc_ms[GSR_STAGE_CULL] += el(EV_START, EV_CULL);
    c->acc_ms[GSR_STAGE_PREPROCESS] += el(EV_CULL, EV_PRE);
    c->acc_ms[GSR_STAGE_SYNC] += el(EV_PRE, EV_AFTER_SYNC1) + el(EV_COUNTS, EV_AFTER_SYNC2);
    c->acc_ms[GSR_STAGE_DEPTH_SORT] += el(EV_AFTER_SYNC1, EV_DSORT);
    c->acc_ms[GSR_STAGE_BINNING] += el(EV_DSORT, EV_COUNTS) + el(EV_AFTER_SYNC2, EV_DUPW);
    c->acc_ms[GSR_STAGE_TILE_SORT] += el(EV_DUPW, EV_TSORT);
    c->acc_ms[GSR_STAGE_RANGES] += el(EV_TSORT, EV_RANGES_END_COMPOSITE_START);
    c->acc_ms[GSR_STAGE_COMPOSITE] += el(EV_RANGES_END_COMPOSITE_START, EV_COMPOSITE);
    c->acc_ms[GSR_STAGE_MERGE] += el(EV_COMPOSITE, EV_COUNT);
    c->prof_frames += 1;
    c->ev_pending[slot] = false;
}

void prof_group_accumulate(gsr_context* c, int slot) {
    if (!c->evg_pending[slot]) return;
    (void)hipEventSynchronize(c->evg[slot][1]);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->evg[slot][0], c->evg[slot][1]);
    c->group_comp_ms += ms;
    c->group_launches += 1;
    c->group_views += c->evg_views[slot];
    c->evg_pending[slot] = false;
}

// Stable sort of (key, val) pairs; totals = digit-total scratch.
// The frame's depth sort (pairs (depth key, slot), over the upper bound n; the
// device count V bounds the work); carries the packed tile rects as payload
// when the frame's tiles fit 8 bits per coordinate.
// A frame alone's compositing chunk: `chunk`, or longer when the frame has
// more instances than chunk_target chunks of it would hold (fewer partials and
// merges, and chunks long enough to saturate slices themselves)
uint32_t frame_chunk(const gsr_context* c, uint32_t n_dup) {
    if (!c->chunk_target) return c->chunk;
    const uint64_t want = ((uint64_t)n_dup + c->chunk_target - 1) / c->chunk_target;
    const uint32_t r = (uint32_t)std::min<uint64_t>((want + 63u) & ~63ull, 1u << 20);
    return std::max(c->chunk, std::min(r, std::max(c->chunk, c->chunk_views)));
}

int depth_sort(gsr_context* c, PendingFrame& f, const uint32_t* counters, const uint32_t* key_range, uint32_t* totals,
               hipStream_t s);

int sort_pairs(gsr_context* c, uint32_t** ka, uint32_t** va, uint32_t** kb, uint32_t** vb, bool ident, size_t n,
               const uint32_t* n_dev, int bits, int passes, const uint32_t* key_range, uint32_t* totals,
               hipStream_t s, int first_pass = 0) {
    return radix_sort_pairs(ka, va, kb, vb, ident, n, n_dev, bits, passes, key_range, c->radix_tmp.p, totals, s,
                            nullptr, nullptr, nullptr, first_pass);
}

bool rects_packable(const gsr_context* c, const FrameUniforms& u) {
    return c->rect_payload && u.tiles_x <= kPackedRectTiles && u.tiles_y <= kPackedRectTiles;
}

int depth_sort(gsr_context* c, PendingFrame& f, const uint32_t* counters, const uint32_t* key_range, uint32_t* totals,
               hipStream_t s) {
    f.ka = c->keys_a.p, f.kb = c->keys_b.p, f.va = c->vals_a.p, f.vb = c->vals_b.p;
    f.pa = c->rect4_a.p, f.pb = c->rect4_b.p;
    f.packed = rects_packable(c, f.u);
    f.coarse = 0;
    if (f.n == 0) return GSR_OK;
    // (the payload only when the rects are packed: an unpacked frame gathers them)
    const uint2* rect_in = f.packed ? c->trect.p : nullptr;
    uint32_t** pay_io = f.packed ? &f.pa : nullptr;
    uint32_t** pay_alt = f.packed ? &f.pb : nullptr;
    // a frame alone with the fused binning (which carries the sorted keys to the repair): the coarse order,
    // for scenes of at most kCoarseMaxN Gaussians; larger ones sort exactly in 4 passes of <= 8 bits
    if (c->depth_passes_now && c->depth_coarse_alone && c->bin_fused && f.n <= kCoarseMaxN) {
        f.coarse = c->depth_coarse_alone;
        return radix_sort_pairs(&f.ka, &f.va, &f.kb, &f.vb, true, f.n, counters, (int)f.coarse, 2, key_range,
                                c->radix_tmp.p, totals, s, rect_in, pay_io, pay_alt, 0, c->fused_cull, f.coarse);
    }
    const int passes = !c->depth_passes_now                                     ? kDepthPasses
                       : (c->depth_coarse_alone && f.n > kCoarseMaxN)           ? kDepthPassesBigAlone
                                                                                : c->depth_passes_now;
    // (an exact order: nothing reads the sorted keys, so the last pass writes none)
    return radix_sort_pairs(&f.ka, &f.va, &f.kb, &f.vb, true, f.n, counters, 32, passes, key_range,
                            c->radix_tmp.p, totals, s, rect_in, pay_io, pay_alt, 0, c->fused_cull, 0u, false);
}

// Wait until the last preprocess block has stored this frame's (V, D, seq) to
// host-mapped memory.  Polling the sequence number needs no event record in
// the stream (each one stalls the GPU for several microseconds).  Only after
// a spin far longer than any frame is the stream queried (a query may itself
// enqueue a marker, i.e. a stall): a stream that stopped making progress (a
// fault) is then synchronised, which reports the error.
// The wait has a hard deadline (GSR_WAIT_TIMEOUT_MS, default 2000 ms): a
// stream that makes no progress for that long (a hung kernel, or work queued
// ahead of the frame that never finishes) fails the call with GSR_ERR_HIP and
// marks the context failed instead of spinning forever; a failed context
// refuses further frames (destroy it).
// The frame's tile instances must fit 32 bits (the last preprocess block
// publishes the count's high word beside it): a scene whose splats cover that
// many tiles fails the frame instead of overrunning the instance buffers.
int check_instances(gsr_context* c) {
    const uint32_t hi = __atomic_load_n(&c->host_counters[3], __ATOMIC_ACQUIRE);
    if (hi == 0) return GSR_OK;
    return set_error(GSR_ERR_OVERFLOW, "render: the frame has " +
                                           std::to_string(((uint64_t)hi << 32) | c->host_counters[1]) +
                                           " tile instances (at most 2^32 - 1)");
}

int wait_counts(gsr_context* c, hipStream_t s) {
    const uint32_t want = c->seq;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        if (__atomic_load_n(&c->host_counters[2], __ATOMIC_ACQUIRE) == want) return GSR_OK;
        if ((spin & 4095) == 4095 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {  // stream drained: the store must be visible now
                if (__atomic_load_n(&c->host_counters[2], __ATOMIC_ACQUIRE) == want) return GSR_OK;
                c->failed = true;
                return set_error(GSR_ERR_HIP, "render: frame counters were not published");
            }
            if (q != hipErrorNotReady) {
                c->failed = true;
                return set_error(GSR_ERR_HIP, std::string("render: stream error ") + hipGetErrorString(q));
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(c->wait_timeout_ms)) {
                c->failed = true;
                return set_error(GSR_ERR_HIP, "render: timed out waiting for the frame's counts (stream not "
                                              "progressing); the context is marked failed");
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

}  // namespace
}  // namespace gsr

using namespace gsr;

namespace {
// Test hook: one wave that keeps its stream busy for a bounded time (the
// deadline of the host wait for a frame's counts is tested against it).
__global__ void k_stall(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }

const char* gsr_last_error(void) { return last_error_ref().c_str(); }

void gsr_settings_default(gsr_settings* s) {
    if (!s) return;
    std::memset(s, 0, sizeof(*s));
    s->scale_modifier = 1.f;   // main.py:131
    s->screen_scale = 1.f;     // main.py:132
    s->render_mod = 6;         // main.py:134 (g_render_mode - 3 = 6: SH 0..3)
    s->dc_factor = 1.f;        // renderer_ogl.py:185
    s->extra_factor = 1.f;     // renderer_ogl.py:187
    s->color_scale[0] = s->color_scale[1] = s->color_scale[2] = 1.f;  // renderer_ogl.py:183
    s->rot_modifier[3] = 1.f;  // euler_to_quaternion(0,0,0) -> (x,y,z,w) = (0,0,0,1)
    s->cube_rotation[0] = s->cube_rotation[4] = s->cube_rotation[8] = 1.f;
    s->t_min = 1e-4f;
    s->out_layout = 0;
}

static int validate_sh_dim(int32_t sh_dim) {
    if (sh_dim < 3 || sh_dim > 48 || sh_dim % 3 != 0)
        return set_error(GSR_ERR_INVALID, "sh_dim must be a multiple of 3 in [3, 48]");
    return GSR_OK;
}

static int make_scene(int64_t n, int32_t sh_dim, gsr_scene** out, gsr_scene** sc) {
    if (!out) return set_error(GSR_ERR_INVALID, "out is null");
    *out = nullptr;
    if (n < 0 || n > (int64_t)0x7fffffff) return set_error(GSR_ERR_OVERFLOW, "n out of range [0, 2^31)");
    int rc = validate_sh_dim(sh_dim);
    if (rc) return rc;
    *sc = new gsr_scene();
    (*sc)->d.n = n;
    (*sc)->d.sh_dim = sh_dim;
    (*sc)->d.sh_planes = (sh_dim + 3) / 4;
    (void)hipGetDevice(&(*sc)->device);
    return GSR_OK;
}

int gsr_scene_create(const float* xyz, const float* rot, const float* scale, const float* opacity, const float* sh,
                     int64_t n, int32_t sh_dim, void* stream, gsr_scene** out) {
    gsr_scene* sc = nullptr;
    int rc = make_scene(n, sh_dim, out, &sc);
    if (rc) return rc;
    if (n > 0 && (!xyz || !rot || !scale || !opacity || !sh)) {
        delete sc;
        return set_error(GSR_ERR_INVALID, "null device pointer");
    }
    rc = scene_repack_from_fields(sc->d, xyz, rot, scale, opacity, sh, (hipStream_t)stream);
    if (rc) {
        if (sc->d.block) (void)hipFree(sc->d.block);
        delete sc;
        return rc;
    }
    *out = sc;
    return GSR_OK;
}

int gsr_scene_load_ply(const char* path, float scale_to_interval, int32_t n_threads, void* stream, gsr_scene** out,
                       gsr_ply_scene_info* info) {
    if (!path || !out) return set_error(GSR_ERR_INVALID, "scene_load_ply: null argument");
    *out = nullptr;
    hipStream_t s = (hipStream_t)stream;
    float* flat = nullptr;
    int64_t n = 0;
    int32_t sh_dim = 0;
    int rc = ply_stream_flat(path, n_threads, s, &flat, &n, &sh_dim);
    if (rc) return rc;
    // scratch: 6 min/max keys, (centre, factor), points_center, xyz [n,3]
    void* tmp = nullptr;
    const size_t tmp_bytes = 64 + (size_t)std::max<int64_t>(n, 1) * 3 * sizeof(float);
    if (hipMalloc(&tmp, tmp_bytes) != hipSuccess) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(flat);
        return set_error(GSR_ERR_NOMEM, "scene_load_ply: scratch allocation failed");
    }
    uint32_t* keys = static_cast<uint32_t*>(tmp);
    float* cf = reinterpret_cast<float*>(keys + 8);  // centre xyz, factor
    float* pc = cf + 4;                               // points_center
    float* xyz = pc + 4;
    float host[8] = {0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 0.f};
    gsr_scene* sc = nullptr;
    auto fail = [&](int code) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(flat);
        (void)hipFree(tmp);
        if (sc) {
            if (sc->d.block) (void)hipFree(sc->d.block);
            delete sc;
        }
        return code;
    };
    if ((rc = make_scene(n, sh_dim, out, &sc))) return fail(rc);
    if ((rc = ply_activate_flat(flat, n, sh_dim, scale_to_interval, keys, cf, xyz, s))) return fail(rc);
    if (n > 0 && (rc = launch_points_center(xyz, n, pc, s))) return fail(rc);
    if ((rc = scene_repack_from_flat(sc->d, flat, s))) return fail(rc);
    if (scale_to_interval > 0.f && n > 0 &&
        hipMemcpyAsync(host, cf, 4 * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail(set_error(GSR_ERR_HIP, "scene_load_ply: copy back failed"));
    if (n > 0 && hipMemcpyAsync(host + 4, pc, 3 * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail(set_error(GSR_ERR_HIP, "scene_load_ply: copy back failed"));
    if (hipStreamSynchronize(s) != hipSuccess) return fail(set_error(GSR_ERR_HIP, "scene_load_ply: stream failed"));
    (void)hipFree(flat);
    (void)hipFree(tmp);
    if (info) {
        info->n = n;
        info->sh_dim = sh_dim;
        info->pad = 0;
        for (int k = 0; k < 3; ++k) {
            info->bbox_center[k] = host[k];
            info->points_center[k] = host[4 + k];
        }
        info->scale_factor = host[3];
    }
    *out = sc;
    return GSR_OK;
}

int gsr_scene_read_flat(const gsr_scene* sc, float* flat_dev, void* stream) {
    if (!sc || (!flat_dev && sc->d.n > 0)) return set_error(GSR_ERR_INVALID, "scene_read_flat: null argument");
    return scene_unpack_flat(sc->d, flat_dev, (hipStream_t)stream);
}

int gsr_scene_create_flat(const float* flat, int64_t n, int32_t sh_dim, void* stream, gsr_scene** out) {
    gsr_scene* sc = nullptr;
    int rc = make_scene(n, sh_dim, out, &sc);
    if (rc) return rc;
    if (n > 0 && !flat) {
        delete sc;
        return set_error(GSR_ERR_INVALID, "null device pointer");
    }
    rc = scene_repack_from_flat(sc->d, flat, (hipStream_t)stream);
    if (rc) {
        if (sc->d.block) (void)hipFree(sc->d.block);
        delete sc;
        return rc;
    }
    *out = sc;
    return GSR_OK;
}

int gsr_scene_destroy(gsr_scene* scene) {
    if (!scene) return GSR_OK;
    if (scene->d.block) {
        (void)hipDeviceSynchronize();
        (void)hipFree(scene->d.block);
    }
    delete scene;
    return GSR_OK;
}

int64_t gsr_scene_count(const gsr_scene* scene) { return scene ? scene->d.n : -1; }
int32_t gsr_scene_sh_dim(const gsr_scene* scene) { return scene ? scene->d.sh_dim : -1; }

int gsr_context_create(gsr_context** out) {
    if (!out) return set_error(GSR_ERR_INVALID, "out is null");
    *out = new gsr_context();
    if (const char* e = std::getenv("GSR_CHUNK")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 16 && v <= (1 << 20)) (*out)->chunk = (uint32_t)v;
    }
    if (const char* e = std::getenv("GSR_CHUNK_TARGET")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 0 && v <= (1 << 24)) (*out)->chunk_target = (uint32_t)v;
    }
    if (const char* e = std::getenv("GSR_CHUNK_VIEWS")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 16 && v <= (1 << 20)) (*out)->chunk_views = (uint32_t)v;
    }
    if (const char* e = std::getenv("GSR_LEN_CLASSES")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 2 && v <= gsr::kMaxLenClasses) (*out)->len_classes = (uint32_t)v;
    }
    if (const char* e = std::getenv("GSR_DEPTH_PASSES_ALONE")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 3 && v <= 4) (*out)->depth_passes_alone = (int)v;
    }
    if (const char* e = std::getenv("GSR_FIRST_MAJOR")) (*out)->first_major = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_BIN_FUSED")) (*out)->bin_fused = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_DEPTH_COARSE")) {
        // 0: exact depth sort; 8..16: coarse bits of a frame alone (2 passes of <= 8; wider needs a third pass,
        // whose keys the fused binning would not carry)
        const long v = std::strtol(e, nullptr, 10);
        if (v == 0 || (v >= 8 && v <= (long)kDepthCoarseMax)) (*out)->depth_coarse_alone = (uint32_t)v;
    }
    if (std::getenv("GSR_NO_RECT_PAYLOAD")) (*out)->rect_payload = false;
    if (const char* e = std::getenv("GSR_FUSED_CULL")) (*out)->fused_cull = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_BOUND_ALONE")) (*out)->bound_alone = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_CHUNK_SINGLE")) (*out)->chunk_single = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_FIRST_MAJOR_ALONE"))
        (*out)->first_major_alone = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_VIEWS_INTERLEAVE")) (*out)->views_interleave = std::strtol(e, nullptr, 10) != 0;
    // stage forms and test knobs, read once here so that every launch of a frame sees the same value
    if (const char* e = std::getenv("GSR_TAIL_MERGE")) (*out)->tail_merge_group = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_TAIL_MERGE_ALONE"))
        (*out)->tail_merge_alone = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("GSR_BIN_STAGE_LIMIT"))
        (*out)->bin_stage_limit = gsr::clamp_stage_limit(std::strtol(e, nullptr, 10));
    if (const char* e = std::getenv("GSR_DEBUG_HANDOFF")) (*out)->debug_handoff = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("GSR_WAIT_TIMEOUT_MS")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1) (*out)->wait_timeout_ms = v;
    }
    return GSR_OK;
}

int gsr_context_destroy(gsr_context* c) {
    if (!c) return GSR_OK;
    (void)hipDeviceSynchronize();
    each_buf(c, [](auto& b) { b.release(); });
    if (c->host_counters) (void)hipHostFree(c->host_counters);
    for (auto& row : c->ev)
        for (auto& e : row)
            if (e) (void)hipEventDestroy(e);
    for (auto& row : c->evg)
        for (auto& e : row)
            if (e) (void)hipEventDestroy(e);
    c->stamps.release();
    delete c;
    return GSR_OK;
}

int gsr_context_knob(const gsr_context* c, const char* name, int64_t* value) {
    if (!c || !name || !value) return set_error(GSR_ERR_INVALID, "null argument");
    const std::pair<const char*, int64_t> knobs[] = {
        {"rect_payload", c->rect_payload}, {"fused_cull", c->fused_cull}, {"bin_fused", c->bin_fused},
        {"depth_coarse_alone", c->depth_coarse_alone}, {"chunk", c->chunk}, {"chunk_target", c->chunk_target},
        {"chunk_views", c->chunk_views}, {"tail_merge_alone", c->tail_merge_alone},
        {"tail_merge_group", c->tail_merge_group}, {"first_major", c->first_major},
        {"first_major_alone", c->first_major_alone}, {"bound_alone", c->bound_alone},
        {"chunk_single", c->chunk_single},
        {"frame_packed", c->last_packed},
        {"frame_coarse", c->last_coarse}, {"frame_chunk", c->last_chunk}, {"frame_deep", c->last_deep}};
    for (const auto& k : knobs)
        if (std::strcmp(k.first, name) == 0) {
            *value = k.second;
            return GSR_OK;
        }
    return set_error(GSR_ERR_INVALID, std::string("context_knob: unknown knob ") + name);
}

int gsr_context_stats(const gsr_context* c, gsr_frame_stats* out) {
    if (!c || !out) return set_error(GSR_ERR_INVALID, "null argument");
    *out = c->stats;
    return GSR_OK;
}

int gsr_context_reserve(gsr_context* c, int64_t n, int32_t width, int32_t height, int64_t max_instances,
                        void* stream) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    if (n < 0 || width <= 0 || height <= 0 || width > 32768 || height > 32768)
        return set_error(GSR_ERR_INVALID, "context_reserve: n >= 0 and 1..32768 pixels per side");
    if (c->pend.active || c->pend.sort_ready)
        return set_error(GSR_ERR_INVALID, "context_reserve: a frame is in flight on this context");
    (void)stream;  // sizing only: nothing is enqueued (the first frame zeroes its counter, arm_done_ctr)
    const size_t un = (size_t)n;
    const size_t d = max_instances > 0 ? (size_t)max_instances : 4 * un;
    const int num_tiles = ((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile);
    int rc;
    // the shared radix scratch at its final size first: a smaller block sized by
    // ensure_scene_buffers would be retired (and, in a caller's workspace, wasted)
    const int rtbits = bits_for((uint32_t)num_tiles);
    const size_t rhist = bin_hist_elems(un, rtbits > 0 ? rtbits : 1, std::max(1, radix_passes_for(rtbits)));
    if ((rc = c->radix_tmp.ensure(std::max({radix_tmp_elems(d), radix_tmp_elems(un), rhist}), "radix_tmp"))) return rc;
    if ((rc = ensure_scene_buffers(c, un))) return rc;
    if ((rc = c->zero.ensure(ZeroLayout(num_tiles).total, "zero block"))) return rc;
    if ((rc = c->tkeys_a.ensure(d, "tile_keys"))) return rc;
    if ((rc = c->tkeys_b.ensure(d, "tile_keys"))) return rc;
    if ((rc = c->tvals_a.ensure(d, "tile_vals"))) return rc;
    if ((rc = c->tvals_b.ensure(d, "tile_vals"))) return rc;
    if (c->depth_coarse_alone && c->bin_fused) {  // a frame alone's depth keys through the tile sort
        if ((rc = c->tpay_a.ensure(d, "tile_pay"))) return rc;
        if ((rc = c->tpay_b.ensure(d, "tile_pay"))) return rc;
        if ((rc = c->long_runs.ensure(long_runs_elems(d), "long_runs"))) return rc;
    }
    if ((rc = c->radix_tmp.ensure(std::max({radix_tmp_elems(d), radix_tmp_elems(un), rhist}), "radix_tmp"))) return rc;
    const size_t mc = (size_t)num_tiles + d / std::min(c->chunk, c->chunk_views) + 1;
    if ((rc = c->chunk_cnt.ensure(chunk_cnt_elems(num_tiles), "chunk_cnt"))) return rc;
    if ((rc = c->chunk_base.ensure((size_t)num_tiles, "chunk_base"))) return rc;
    if ((rc = c->chunk_desc.ensure(mc, "chunk_desc"))) return rc;
    if ((rc = c->chunk_order.ensure(mc, "chunk_order"))) return rc;
    if ((rc = c->partial.ensure(mc * 256, "partial"))) return rc;
    if ((rc = c->tmax.ensure(mc, "tmax"))) return rc;
    return GSR_OK;
}

int64_t gsr_context_workspace(gsr_context* c, int64_t* n_allocations) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    int64_t bytes = 0, allocs = 0;
    each_buf(c, [&](auto& b) {
        bytes += (int64_t)b.bytes();
        allocs += b.allocs;
    });
    if (n_allocations) *n_allocations = allocs;
    return bytes;
}

int64_t gsr_workspace_size(int64_t n, int32_t width, int32_t height, int64_t max_instances) {
    gsr_context* c = nullptr;
    int rc = gsr_context_create(&c);
    if (rc) return rc;
    c->has_arena = true;
    c->arena.measure = true;
    gsr::each_buf(c, [&](auto& b) { b.arena = &c->arena; });
    rc = gsr_context_reserve(c, n, width, height, max_instances, nullptr);
    const int64_t bytes = (int64_t)(c->arena.used + gsr::kArenaAlign);  // + slack for an unaligned base
    delete c;  // nothing was allocated
    return rc ? (int64_t)rc : bytes;
}

int gsr_context_attach_workspace(gsr_context* c, void* ws_dev, size_t ws_bytes, int64_t n, int32_t width,
                                 int32_t height, int64_t max_instances, void* stream) {
    if (!c || !ws_dev) return gsr::set_error(GSR_ERR_INVALID, "null argument");
    bool fresh = !c->has_arena;
    gsr::each_buf(c, [&](auto& b) { fresh = fresh && b.p == nullptr; });
    if (!fresh)
        return gsr::set_error(GSR_ERR_INVALID,
                              "context_attach_workspace: the context already holds a workspace (use a new context)");
    // carve from the first 256-B boundary of the caller's block
    const uintptr_t a = ((uintptr_t)ws_dev + gsr::kArenaAlign - 1) & ~(uintptr_t)(gsr::kArenaAlign - 1);
    const size_t skip = (size_t)(a - (uintptr_t)ws_dev);
    c->has_arena = true;
    c->arena = gsr::Arena{};
    c->arena.base = reinterpret_cast<char*>(a);
    c->arena.bytes = ws_bytes > skip ? ws_bytes - skip : 0;
    gsr::each_buf(c, [&](auto& b) { b.arena = &c->arena; });
    const int rc = gsr_context_reserve(c, n, width, height, max_instances, stream);
    if (rc == GSR_OK) c->arena.sealed = true;  // frames within the bounds reuse; beyond them: GSR_ERR_NOMEM
    return rc;
}

int gsr_render_begin(gsr_context* c, const gsr_scene* sc, const gsr_camera* cam, const gsr_settings* st, float* out,
                     int32_t* radii, void* stream) {
    if (!c || !sc || !cam || !st || !out) return set_error(GSR_ERR_INVALID, "null argument");
    if (c->failed) return set_error(GSR_ERR_HIP, "render: the context failed earlier (destroy it)");
    if (c->pend.active || c->pend.sort_ready)
        return set_error(GSR_ERR_INVALID, "render_begin: the previous frame was not finished");
    hipStream_t s = (hipStream_t)stream;
    const auto h0 = std::chrono::steady_clock::now();
    FrameUniforms u;
    int rc = build_uniforms(sc, cam, st, u);
    if (rc) return rc;
    const size_t n = (size_t)sc->d.n;
    const int num_tiles = u.tiles_x * u.tiles_y;
    if ((rc = ensure_scene_buffers(c, n))) return rc;
    if ((rc = arm_done_ctr(c, s))) return rc;
    const ZeroLayout zl(num_tiles);
    if ((rc = c->zero.ensure(zl.total, "zero block"))) return rc;
    uint32_t* counters = c->zero.p + zl.counters;
    const int slot = (int)(c->frame_idx & 1);
    if (c->prof_on) prof_accumulate(c, slot, true);  // slot reuse: frame k-2 is long done

    c->stats = gsr_frame_stats{};
    c->stats.n_gaussians = (int64_t)n;
    c->stats.tiles_x = u.tiles_x;
    c->stats.tiles_y = u.tiles_y;
    c->last_depth_order = c->last_tile_list = nullptr;
    c->last_tiles = num_tiles;
    c->last_ranges = reinterpret_cast<uint2*>(c->zero.p + zl.ranges);

    if ((rc = prof_record(c, slot, EV_START, s))) return rc;
    if (n == 0) GSR_HIP_CHECK(hipMemsetAsync(c->zero.p, 0, sizeof(uint32_t) * zl.total, s));
    if (n > 0 && c->fused_cull) {
        // one launch: cull, preprocess, V / D / key range, and the zero block's clearing
        if ((rc = prof_record(c, slot, EV_CULL, s))) return rc;
        if ((rc = launch_preprocess_fc(sc->d, u, c->recs.p, c->keys_a.p, c->trect.p, counters, c->zero.p + zl.key_range,
                                       c->zero.p + zl.ranges, (uint32_t)(zl.total - zl.ranges), c->done_ctr.p,
                                       c->host_counters_dev, ++c->seq, radii, s)))
            return rc;
    } else if (n > 0) {
        const size_t nw = (n + 63) / 64;
        // k_cull clears the tile ranges and saturation words; every other word
        // of the zero block is overwritten (not accumulated) before it is read
        if ((rc = launch_cull(sc->d, u, c->vis_mask.p, c->wave_counts.p, c->block_ranges.p, c->zero.p + zl.cleared,
                              (uint32_t)(zl.total - zl.cleared), s)))
            return rc;
        // visible-compaction offsets + V, and the frame's depth-key range
        if ((rc = scan_exclusive(c->wave_counts.p, c->wave_counts.p, nw, c->scan_tmp.p, counters + 0, s,
                                 c->block_ranges.p, (n + kCullBlock - 1) / kCullBlock, c->zero.p + zl.key_range)))
            return rc;
    }
    if (!(n > 0 && c->fused_cull) && (rc = prof_record(c, slot, EV_CULL, s))) return rc;
    if (n > 0 && !c->fused_cull && (rc = launch_preprocess(sc->d, u, c->vis_mask.p, c->wave_counts.p, counters + 0, c->recs.p,
                                         c->keys_a.p, c->trect.p, counters, c->done_ctr.p, c->host_counters_dev,
                                         ++c->seq, radii, s)))
        return rc;
    if ((rc = prof_record(c, slot, EV_PRE, s))) return rc;
    if ((rc = prof_record(c, slot, EV_AFTER_SYNC1, s))) return rc;

    // depth sort over the upper bound N; the device count V bounds the work
    PendingFrame& f = c->pend;
    f.n = n;
    f.u = u;
    if ((rc = depth_sort(c, f, counters + 0, c->zero.p + zl.key_range, c->zero.p + zl.totals_depth, s))) return rc;
    if ((rc = prof_record(c, slot, EV_DSORT, s))) return rc;
    f.active = true;
    f.u = u;
    f.t_min = st->t_min;
    std::memcpy(f.bg, st->bg, sizeof(f.bg));
    f.out_layout = st->out_layout;
    f.blend = st->blend;
    f.out = out;
    f.stream = s;
    f.n = n;
    f.slot = slot;
    c->host_ms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
    return GSR_OK;
}

int gsr_render_begin_views(gsr_context* const* ctxs, int32_t k, const gsr_scene* sc, const gsr_camera* cams,
                           const gsr_settings* st, float* const* outs, int32_t* const* radii, void* stream) {
    if (!ctxs || !sc || !cams || !st || !outs) return set_error(GSR_ERR_INVALID, "null argument");
    if (k < 1 || k > GSR_MAX_VIEWS) return set_error(GSR_ERR_INVALID, "render_begin_views: k out of range");
    for (int v = 0; v < k; ++v) {
        if (!ctxs[v] || !outs[v]) return set_error(GSR_ERR_INVALID, "null argument");
        if (ctxs[v]->failed) return set_error(GSR_ERR_HIP, "render: a context failed earlier (destroy it)");
        if (ctxs[v]->pend.active || ctxs[v]->pend.sort_ready)
            return set_error(GSR_ERR_INVALID, "render_begin_views: a view's previous frame was not finished");
        if (ctxs[v]->prof_on) return set_error(GSR_ERR_INVALID, "render_begin_views: stage profiling is per view only");
        for (int w = 0; w < v; ++w)
            if (ctxs[w] == ctxs[v]) return set_error(GSR_ERR_INVALID, "render_begin_views: contexts must differ");
    }
    hipStream_t s = (hipStream_t)stream;
    const size_t n = (size_t)sc->d.n;
    FrameUniforms u[GSR_MAX_VIEWS];
    ViewCullArgs cull[GSR_MAX_VIEWS];
    ViewPreArgs pre[GSR_MAX_VIEWS];
    ViewPreFcArgs pfc[GSR_MAX_VIEWS];
    const bool fc = ctxs[0]->fused_cull;
    for (int v = 1; v < k; ++v)
        if (ctxs[v]->fused_cull != fc)
            return set_error(GSR_ERR_INVALID, "render_begin_views: contexts differ in the cull mode (GSR_FUSED_CULL)");
    int rc;
    for (int v = 0; v < k; ++v) {
        gsr_context* c = ctxs[v];
        const auto h0 = std::chrono::steady_clock::now();
        if ((rc = build_uniforms(sc, &cams[v], st, u[v]))) return rc;
        const int num_tiles = u[v].tiles_x * u[v].tiles_y;
        if ((rc = ensure_scene_buffers(c, n))) return rc;
        if ((rc = arm_done_ctr(c, s))) return rc;
        const ZeroLayout zl(num_tiles);
        if ((rc = c->zero.ensure(zl.total, "zero block"))) return rc;
        uint32_t* counters = c->zero.p + zl.counters;
        c->stats = gsr_frame_stats{};
        c->stats.n_gaussians = (int64_t)n;
        c->stats.tiles_x = u[v].tiles_x;
        c->stats.tiles_y = u[v].tiles_y;
        c->last_depth_order = c->last_tile_list = nullptr;
        c->last_tiles = num_tiles;
        c->last_ranges = reinterpret_cast<uint2*>(c->zero.p + zl.ranges);
        if (n == 0) GSR_HIP_CHECK(hipMemsetAsync(c->zero.p, 0, sizeof(uint32_t) * zl.total, s));
        cull[v] = ViewCullArgs{&u[v], c->vis_mask.p, c->wave_counts.p, c->block_ranges.p, c->zero.p + zl.cleared,
                               (uint32_t)(zl.total - zl.cleared)};
        pre[v] = ViewPreArgs{&u[v], c->vis_mask.p, c->wave_counts.p, counters + 0, c->recs.p, c->keys_a.p,
                             c->trect.p, counters, c->done_ctr.p, c->host_counters_dev, radii ? radii[v] : nullptr,
                             ++c->seq};
        pfc[v] = ViewPreFcArgs{&u[v], c->recs.p, c->keys_a.p, c->trect.p, counters, c->zero.p + zl.key_range,
                               c->zero.p + zl.ranges, c->done_ctr.p, c->host_counters_dev,
                               radii ? radii[v] : nullptr, (uint32_t)(zl.total - zl.ranges), c->seq};
        PendingFrame& f = c->pend;
        f.u = u[v];
        f.t_min = st->t_min;
        std::memcpy(f.bg, st->bg, sizeof(f.bg));
        f.out_layout = st->out_layout;
        f.blend = st->blend;
        f.out = outs[v];
        f.n = n;
        f.slot = (int)(c->frame_idx & 1);
        c->host_ms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
    }
    if (n > 0 && fc) {
        if ((rc = launch_preprocess_fc_views(sc->d, pfc, k, s))) return rc;
    } else if (n > 0) {
        if ((rc = launch_cull_views(sc->d, cull, k, s))) return rc;
        const size_t nw = (n + 63) / 64;
        const size_t n_kr = (n + kCullBlock - 1) / kCullBlock;
        // visible-compaction offsets + V, and the frame's depth-key range:
        // one launch for the group when the arrays fit the one-pass scan
        if (scan_views_fits(nw)) {
            const uint32_t* in[GSR_MAX_VIEWS];
            uint32_t *out[GSR_MAX_VIEWS], *tot[GSR_MAX_VIEWS], *kro[GSR_MAX_VIEWS];
            const uint2* kri[GSR_MAX_VIEWS];
            for (int v = 0; v < k; ++v) {
                gsr_context* c = ctxs[v];
                const ZeroLayout zl(u[v].tiles_x * u[v].tiles_y);
                in[v] = out[v] = c->wave_counts.p;
                tot[v] = c->zero.p + zl.counters;
                kri[v] = c->block_ranges.p;
                kro[v] = c->zero.p + zl.key_range;
            }
            if ((rc = scan_exclusive_views(in, out, nw, tot, kri, n_kr, kro, k, s))) return rc;
        } else {
            for (int v = 0; v < k; ++v) {
                gsr_context* c = ctxs[v];
                const ZeroLayout zl(u[v].tiles_x * u[v].tiles_y);
                if ((rc = scan_exclusive(c->wave_counts.p, c->wave_counts.p, nw, c->scan_tmp.p, c->zero.p + zl.counters,
                                         s, c->block_ranges.p, n_kr, c->zero.p + zl.key_range)))
                    return rc;
            }
        }
        if ((rc = launch_preprocess_views(sc->d, pre, k, s))) return rc;
    }
    for (int v = 0; v < k; ++v) ctxs[v]->pend.sort_ready = true;
    return GSR_OK;
}

int gsr_render_begin_sort(gsr_context* c, void* stream) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    PendingFrame& f = c->pend;
    if (!f.sort_ready) return set_error(GSR_ERR_INVALID, "render_begin_sort: no gsr_render_begin_views frame");
    hipStream_t s = (hipStream_t)stream;
    const ZeroLayout zl(f.u.tiles_x * f.u.tiles_y);
    uint32_t* counters = c->zero.p + zl.counters;
    // depth sort over the upper bound N; the device count V bounds the work
    int rc;
    if ((rc = depth_sort(c, f, counters + 0, c->zero.p + zl.key_range, c->zero.p + zl.totals_depth, s))) return rc;
    f.sort_ready = false;
    f.active = true;
    f.stream = s;
    return GSR_OK;
}

int gsr_render_begin_sorts(gsr_context* const* ctxs, int32_t k, void* stream) {
    if (!ctxs) return set_error(GSR_ERR_INVALID, "null argument");
    if (k < 1 || k > GSR_MAX_VIEWS) return set_error(GSR_ERR_INVALID, "render_begin_sorts: k out of range");
    hipStream_t s = (hipStream_t)stream;
    RadixViewArgs views[GSR_MAX_VIEWS];
    size_t n = 0;
    for (int v = 0; v < k; ++v) {
        gsr_context* c = ctxs[v];
        if (!c) return set_error(GSR_ERR_INVALID, "null argument");
        PendingFrame& f = c->pend;
        if (!f.sort_ready) return set_error(GSR_ERR_INVALID, "render_begin_sorts: no gsr_render_begin_views frame");
        if (v == 0) n = f.n;
        if (f.n != n) return set_error(GSR_ERR_INVALID, "render_begin_sorts: views of different scenes");
        for (int w = 0; w < v; ++w)
            if (ctxs[w] == c) return set_error(GSR_ERR_INVALID, "render_begin_sorts: contexts must differ");
        const ZeroLayout zl(f.u.tiles_x * f.u.tiles_y);
        f.ka = c->keys_a.p, f.kb = c->keys_b.p, f.va = c->vals_a.p, f.vb = c->vals_b.p;
        f.pa = c->rect4_a.p, f.pb = c->rect4_b.p;
        f.packed = rects_packable(c, f.u);
        if (f.packed != rects_packable(ctxs[0], ctxs[0]->pend.u))
            return set_error(GSR_ERR_INVALID, "render_begin_sorts: views differ in frame size or rect payload");
        // a group's frames: the exact sort (kDepthCoarseAlone); its last pass writes no keys (none are read)
        views[v] = RadixViewArgs{&f.ka, &f.va, &f.kb, &f.vb, c->zero.p + zl.counters, c->zero.p + zl.key_range,
                                 c->radix_tmp.p, c->zero.p + zl.totals_depth, f.packed ? c->trect.p : nullptr,
                                 f.packed ? &f.pa : nullptr, f.packed ? &f.pb : nullptr, c->fused_cull, 0u, false};
        f.coarse = 0;
    }
    int rc;
    if (n > 0 && (rc = radix_sort_pairs_views(views, k, true, n, 32, kDepthPasses, s))) return rc;
    for (int v = 0; v < k; ++v) {
        PendingFrame& f = ctxs[v]->pend;
        f.sort_ready = false;
        f.active = true;
        f.stream = s;
    }
    return GSR_OK;
}

int gsr_render_finish(gsr_context* c, void* stream) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    PendingFrame& f = c->pend;
    if (!f.active) return set_error(GSR_ERR_INVALID, "render_finish: no frame was begun");
    if ((hipStream_t)stream != f.stream) return set_error(GSR_ERR_INVALID, "render_finish: not the frame's stream");
    f.active = false;
    hipStream_t s = f.stream;
    const FrameUniforms& u = f.u;
    const size_t n = f.n;
    const int slot = f.slot;
    const int num_tiles = u.tiles_x * u.tiles_y;
    const ZeroLayout zl(num_tiles);
    uint32_t* counters = c->zero.p + zl.counters;
    uint2* ranges = reinterpret_cast<uint2*>(c->zero.p + zl.ranges);
    uint32_t* sat = c->zero.p + zl.sat;
    int rc;

    // host: V and D (the GPU is busy with the depth sort meanwhile)
    const auto h1 = std::chrono::steady_clock::now();
    if (n > 0 && (rc = wait_counts(c, s))) return rc;
    const auto h2 = std::chrono::steady_clock::now();
    const uint32_t n_vis = n > 0 ? __atomic_load_n(&c->host_counters[0], __ATOMIC_ACQUIRE) : 0u;
    const uint32_t n_dup = n > 0 ? __atomic_load_n(&c->host_counters[1], __ATOMIC_ACQUIRE) : 0u;
    if (n > 0 && (rc = check_instances(c))) return rc;
    if (c->prof_on) prof_accumulate(c, slot ^ 1, false);
    if (n_vis > 0) c->last_depth_order = f.va;

    uint32_t* tile_list = c->tvals_a.p;
    const int tbits = bits_for((uint32_t)num_tiles);
    const int tpasses = radix_passes_for(tbits);
    const bool fused = c->bin_fused;
    const bool carry = f.coarse && fused;  // the instances' depth keys ride along (coarse order repair)
    uint32_t *tpa = c->tpay_a.p, *tpb = c->tpay_b.p;
    if (n_dup > 0) {
        if ((rc = c->tkeys_a.ensure(n_dup, "tile_keys"))) return rc;
        if ((rc = c->tkeys_b.ensure(n_dup, "tile_keys"))) return rc;
        if ((rc = c->tvals_a.ensure(n_dup, "tile_vals"))) return rc;
        if ((rc = c->tvals_b.ensure(n_dup, "tile_vals"))) return rc;
        if ((rc = c->radix_tmp.ensure(std::max({radix_tmp_elems(n_dup), radix_tmp_elems(n),
                                                bin_hist_elems(n_vis, tbits > 0 ? tbits : 1, tpasses > 0 ? tpasses : 1)}),
                                      "radix_tmp")))
            return rc;
        if (carry && ((rc = c->tpay_a.ensure(n_dup, "tile_pay"))) == 0) rc = c->tpay_b.ensure(n_dup, "tile_pay");
        if (carry && rc == 0) rc = c->long_runs.ensure(long_runs_elems(n_dup), "long_runs");
        if (rc) return rc;
        tpa = c->tpay_a.p, tpb = c->tpay_b.p;
        if (fused)  // the tile sort's pass 0 in the binning: instances leave it ordered by digit 0
            rc = launch_binning_sorted(f.va, c->trect.p, f.packed ? f.pa : nullptr, n_vis, u.tiles_x, tbits, tpasses,
                                       c->radix_tmp.p, c->zero.p + zl.totals_tile, c->trect_sorted.p, c->tkeys_a.p,
                                       c->tvals_a.p, s, carry ? f.ka : nullptr, carry ? c->tpay_a.p : nullptr);
        else
            rc = launch_binning(f.va, c->trect.p, f.packed ? f.pa : nullptr, n_vis, u.tiles_x, c->bin_tmp.p,
                                c->trect_sorted.p, c->tkeys_a.p, c->tvals_a.p, c->bin_stage_limit, s);
        if (rc) return rc;
    }
    if ((rc = prof_record(c, slot, EV_COUNTS, s))) return rc;
    if ((rc = prof_record(c, slot, EV_AFTER_SYNC2, s))) return rc;
    if ((rc = prof_record(c, slot, EV_DUPW, s))) return rc;
    uint32_t *tka = c->tkeys_a.p, *tkb = c->tkeys_b.p, *tva = c->tvals_a.p, *tvb = c->tvals_b.p;
    if (n_dup > 0) {
        if (tbits > 0 && (rc = radix_sort_pairs(&tka, &tva, &tkb, &tvb, false, n_dup, nullptr, tbits, tpasses, nullptr,
                                                c->radix_tmp.p, c->zero.p + zl.totals_tile, s, nullptr,
                                                carry ? &tpa : nullptr, carry ? &tpb : nullptr, fused ? 1 : 0)))
            return rc;
        tile_list = tva;
        c->last_tile_list = tva;
    }
    if ((rc = prof_record(c, slot, EV_TSORT, s))) return rc;
    // tile ranges, and (coarse order) the repair of each tile list's runs of equal coarse keys: in registers,
    // or, for the runs that outgrow the window, k_long_runs
    const RunFix fix{tva, c->zero.p + zl.key_range, f.coarse, tkb, tvb, carry ? tpa : nullptr,
                     carry ? c->long_runs.p : nullptr, c->zero.p + zl.long_runs};
    if (n_dup > 0 && (rc = launch_tile_ranges(tka, n_dup, ranges, fix, s))) return rc;
    // the runs longer than the repair's: by the chunk-count launch, or alone (no chunks: RGBA8)
    const LongRuns long_runs{tka, n_dup, fix};
    const bool runs_apart = n_dup > 0 && f.coarse && f.blend == GSR_BLEND_UNORM8;
    if (runs_apart && (rc = launch_long_runs(tka, n_dup, ranges, fix, s))) return rc;

    if (f.blend == GSR_BLEND_UNORM8) {  // the RGBA8 framebuffer: whole lists, back to front, no chunks
        if ((rc = prof_record(c, slot, EV_RANGES_END_COMPOSITE_START, s))) return rc;
        if ((rc = launch_composite_unorm8(ranges, tile_list, c->recs.p, u, frag_class_of(u.render_mod), f.bg,
                                          f.out_layout, f.out, s)))
            return rc;
        if ((rc = prof_record(c, slot, EV_COMPOSITE, s))) return rc;
    } else {
        // compositing chunks: at most one per tile plus one per `chunk` instances
        // a frame of many instances (frame_chunk longer than `chunk`): longer chunks, first chunks
        // dispatched first, and later chunks stopped by the earlier ones' transmittance bound
        const uint32_t chunk = frame_chunk(c, n_dup);
        const bool deep = chunk > c->chunk || (c->bound_alone && f.t_min > 0.f);
        const size_t max_chunks = (size_t)num_tiles + n_dup / chunk + 1;
        if ((rc = c->chunk_cnt.ensure(chunk_cnt_elems(num_tiles), "chunk_cnt"))) return rc;
        if ((rc = c->chunk_base.ensure((size_t)num_tiles, "chunk_base"))) return rc;
        if ((rc = c->chunk_desc.ensure(max_chunks, "chunk_desc"))) return rc;
        if ((rc = c->chunk_order.ensure(max_chunks, "chunk_order"))) return rc;
        if ((rc = c->partial.ensure(max_chunks * 256, "partial"))) return rc;
        if ((rc = c->tmax.ensure(max_chunks, "tmax"))) return rc;
        float4* const tmax = deep ? c->tmax.p : nullptr;  // (after its ensure: it may have moved)
        if ((rc = launch_chunks(ranges, num_tiles, chunk, c->len_classes, c->chunk_cnt.p, c->chunk_base.p, counters + 2,
                                c->chunk_desc.p, c->chunk_order.p, tmax, s, c->first_major_alone || deep,
                                f.coarse ? &long_runs : nullptr, c->chunk_single ? n_dup / chunk : 0xffffffffu)))
            return rc;
        if ((rc = prof_record(c, slot, EV_RANGES_END_COMPOSITE_START, s))) return rc;
        if ((rc = launch_composite(c->chunk_desc.p, c->chunk_order.p, counters + 2, (uint32_t)max_chunks, c->chunk_cnt.p, c->chunk_base.p,
                                   sat, tile_list, c->recs.p, u, frag_class_of(u.render_mod), f.t_min, f.bg,
                                   f.out_layout, f.out, c->partial.p, tmax, c->tail_merge_alone, s)))
            return rc;
        if ((rc = prof_record(c, slot, EV_COMPOSITE, s))) return rc;
        if ((rc = launch_merge(c->chunk_cnt.p, c->chunk_base.p, c->partial.p, sat, u, f.t_min, f.bg, f.out_layout,
                               f.out, c->tail_merge_alone, s)))
            return rc;
    }
    if ((rc = prof_record(c, slot, EV_COUNT, s))) return rc;
    if (c->prof_on) c->ev_pending[slot] = true;
    {
        const auto h3 = std::chrono::steady_clock::now();
        using ms = std::chrono::duration<double, std::milli>;
        c->host_ms[1] += ms(h2 - h1).count();
        c->host_ms[2] += ms(h3 - h2).count();
        c->host_frames += 1;
    }
    c->frame_idx += 1;
    c->stats.n_visible = n_vis;
    c->stats.n_instances = n_dup;
    c->last_packed = f.packed;
    c->last_coarse = f.coarse;
    c->last_chunk = f.blend == GSR_BLEND_UNORM8 ? 0u : frame_chunk(c, n_dup);
    c->last_deep = f.blend != GSR_BLEND_UNORM8 && (c->last_chunk > c->chunk || (c->bound_alone && f.t_min > 0.f));
    return GSR_OK;
}

// The second halves of a group of frames in one set of launches (view =
// blockIdx.y in every kernel): binning, tile sort, ranges, chunks, composite
// and merge are each one launch for the group instead of one per view.
int gsr_render_wait_counts(gsr_context* ctx) {
    if (!ctx) return set_error(GSR_ERR_INVALID, "null argument");
    if (!ctx->pend.active) return set_error(GSR_ERR_INVALID, "render_wait_counts: no frame was begun");
    if (ctx->failed) return set_error(GSR_ERR_HIP, "render: the context failed earlier (destroy it)");
    return ctx->pend.n > 0 ? wait_counts(ctx, ctx->pend.stream) : GSR_OK;
}

int gsr_render_finish_views(gsr_context* const* ctxs, int32_t k, void* stream) {
    if (!ctxs) return set_error(GSR_ERR_INVALID, "null argument");
    if (k < 1 || k > GSR_MAX_VIEWS) return set_error(GSR_ERR_INVALID, "render_finish_views: k out of range");
    hipStream_t s = (hipStream_t)stream;
    gsr_context* c0 = ctxs[0];
    if (!c0) return set_error(GSR_ERR_INVALID, "null argument");
    for (int v = 0; v < k; ++v) {
        gsr_context* c = ctxs[v];
        if (!c) return set_error(GSR_ERR_INVALID, "null argument");
        const PendingFrame& f = c->pend;
        const PendingFrame& f0 = c0->pend;
        if (!f.active) return set_error(GSR_ERR_INVALID, "render_finish_views: no frame was begun");
        if (f.stream != s) return set_error(GSR_ERR_INVALID, "render_finish_views: not the frames' stream");
        if (c->prof_on) return set_error(GSR_ERR_INVALID, "render_finish_views: profiling is per view");
        for (int w = 0; w < v; ++w)
            if (ctxs[w] == c) return set_error(GSR_ERR_INVALID, "render_finish_views: contexts must differ");
        // (only gsr_render sorts coarsely, and it finishes its own frame: an internal invariant)
        if (f.coarse)
            return set_error(GSR_ERR_INVALID, "render_finish_views: internal error: a coarse depth order (gsr_render's "
                                              "own) reached a group finish");
        if (f.u.width != f0.u.width || f.u.height != f0.u.height || f.t_min != f0.t_min || f.bg[0] != f0.bg[0] ||
            f.bg[1] != f0.bg[1] || f.bg[2] != f0.bg[2] || f.out_layout != f0.out_layout || f.blend != f0.blend ||
            frag_class_of(f.u.render_mod) != frag_class_of(f0.u.render_mod) || c->chunk_views != c0->chunk_views ||
            c->len_classes != c0->len_classes || c->first_major != c0->first_major)
            return set_error(GSR_ERR_INVALID, "render_finish_views: views differ in frame size or settings");
    }
    const FrameUniforms& u0 = c0->pend.u;
    const int num_tiles = u0.tiles_x * u0.tiles_y;
    const ZeroLayout zl(num_tiles);
    FinishView fv[GSR_MAX_VIEWS];
    RadixViewArgs rv[GSR_MAX_VIEWS];
    uint32_t *tka[GSR_MAX_VIEWS], *tkb[GSR_MAX_VIEWS], *tva[GSR_MAX_VIEWS], *tvb[GSR_MAX_VIEWS];
    uint32_t n_vis_max = 0, n_dup_max = 0;
    size_t max_chunks = 0;
    int rc;
    const auto h1 = std::chrono::steady_clock::now();
    // From here on the group's frames are consumed whatever happens: a failure
    // (a wait that timed out, a bound of a caller's workspace exceeded) ends
    // every view's frame, so each context can begin a new one.
    for (int v = 0; v < k; ++v) ctxs[v]->pend.active = false;
    // the frames' counts (published together by the shared preprocess, or one by one)
    for (int v = 0; v < k; ++v)
        if (ctxs[v]->pend.n > 0 && (rc = wait_counts(ctxs[v], s))) return rc;
    const auto h2 = std::chrono::steady_clock::now();
    for (int v = 0; v < k; ++v) {
        gsr_context* c = ctxs[v];
        PendingFrame& f = c->pend;
        const uint32_t n_vis = f.n > 0 ? __atomic_load_n(&c->host_counters[0], __ATOMIC_ACQUIRE) : 0u;
        const uint32_t n_dup = f.n > 0 ? __atomic_load_n(&c->host_counters[1], __ATOMIC_ACQUIRE) : 0u;
        if (f.n > 0 && (rc = check_instances(c))) return rc;
        n_vis_max = std::max(n_vis_max, n_vis);
        n_dup_max = std::max(n_dup_max, n_dup);
        if (n_vis > 0) c->last_depth_order = f.va;
        if (n_dup > 0) {
            if ((rc = c->tkeys_a.ensure(n_dup, "tile_keys"))) return rc;
            if ((rc = c->tkeys_b.ensure(n_dup, "tile_keys"))) return rc;
            if ((rc = c->tvals_a.ensure(n_dup, "tile_vals"))) return rc;
            if ((rc = c->tvals_b.ensure(n_dup, "tile_vals"))) return rc;
        }
        const size_t mc = (size_t)num_tiles + n_dup / c->chunk_views + 1;
        max_chunks = std::max(max_chunks, mc);
        if ((rc = c->chunk_cnt.ensure(chunk_cnt_elems(num_tiles), "chunk_cnt"))) return rc;
        if ((rc = c->chunk_base.ensure((size_t)num_tiles, "chunk_base"))) return rc;
        if ((rc = c->chunk_desc.ensure(mc, "chunk_desc"))) return rc;
        if ((rc = c->chunk_order.ensure(mc, "chunk_order"))) return rc;
        if ((rc = c->partial.ensure(mc * 256, "partial"))) return rc;
        if ((rc = c->tmax.ensure(mc, "tmax"))) return rc;
        uint32_t* counters = c->zero.p + zl.counters;
        tka[v] = c->tkeys_a.p, tkb[v] = c->tkeys_b.p, tva[v] = c->tvals_a.p, tvb[v] = c->tvals_b.p;
        if (f.packed != c0->pend.packed)
            return set_error(GSR_ERR_INVALID, "render_finish_views: views differ in frame size or settings");
        fv[v] = FinishView{f.va, c->trect.p, f.packed ? f.pa : nullptr, n_vis, n_dup, c->bin_tmp.p, c->trect_sorted.p, tka[v], tva[v], RunFix{},
                           reinterpret_cast<uint2*>(c->zero.p + zl.ranges), c->chunk_cnt.p, c->chunk_base.p,
                           counters + 2, c->chunk_desc.p, c->chunk_order.p, c->tmax.p, c->zero.p + zl.sat,
                           c->recs.p, f.out, c->partial.p};
        rv[v] = RadixViewArgs{&tka[v], &tva[v], &tkb[v], &tvb[v], counters + 1, nullptr, c->radix_tmp.p,
                              c->zero.p + zl.totals_tile};
    }
    // every view's sort temporaries cover the largest view (the grids do)
    const int tbits = bits_for((uint32_t)num_tiles);
    const int tpasses = radix_passes_for(tbits);
    const bool fused = c0->bin_fused;
    uint32_t* hist[GSR_MAX_VIEWS];
    uint32_t* ttot[GSR_MAX_VIEWS];
    for (int v = 0; v < k && n_dup_max > 0; ++v) {
        gsr_context* c = ctxs[v];
        if ((rc = c->radix_tmp.ensure(std::max({radix_tmp_elems(n_dup_max), radix_tmp_elems(c->pend.n),
                                                bin_hist_elems(n_vis_max, tbits > 0 ? tbits : 1,
                                                               tpasses > 0 ? tpasses : 1)}),
                                      "radix_tmp")))
            return rc;
        rv[v].tmp = c->radix_tmp.p;
        hist[v] = c->radix_tmp.p;
        ttot[v] = c->zero.p + zl.totals_tile;
    }
    if (n_vis_max > 0 && n_dup_max > 0) {
        rc = fused ? launch_binning_sorted_views(fv, hist, ttot, k, u0.tiles_x, tbits, tpasses, s)
                   : launch_binning_views(fv, k, u0.tiles_x, c0->bin_stage_limit, s);
        if (rc) return rc;
    }
    if (n_dup_max > 0 && tbits > 0 &&
        (rc = radix_sort_pairs_views(rv, k, false, n_dup_max, tbits, tpasses, s, fused ? 1 : 0)))
        return rc;
    for (int v = 0; v < k; ++v) {
        fv[v].tile_keys = tka[v];
        fv[v].tile_vals = tva[v];
        fv[v].fix = RunFix{};  // (a group's frames are sorted exactly: nothing to repair)
        if (fv[v].n_dup > 0) ctxs[v]->last_tile_list = tva[v];
    }
    if ((rc = launch_tile_ranges_views(fv, k, s))) return rc;
    const PendingFrame& f0 = c0->pend;
    if (f0.blend == GSR_BLEND_UNORM8) {  // the RGBA8 framebuffer: one launch per view, no chunks
        for (int v = 0; v < k; ++v)
            if ((rc = launch_composite_unorm8(fv[v].ranges, fv[v].tile_vals, fv[v].recs, u0,
                                              frag_class_of(u0.render_mod), f0.bg, f0.out_layout, fv[v].out, s)))
                return rc;
    } else {
        if ((rc = launch_chunks_views(fv, k, num_tiles, c0->chunk_views, c0->len_classes, c0->first_major, s))) return rc;
        const int gslot = c0->evg_slot;
        if (c0->prof_group) {
            prof_group_accumulate(c0, gslot);  // slot reuse: that launch is two groups back
            GSR_HIP_CHECK(hipEventRecord(c0->evg[gslot][0], s));
        }
        // in-kernel clock stamps of the launch (profiling): room for kSpanLaunches
        // launches of this size is reserved at the first one, so recording
        // never reallocates inside a profiled region
        uint64_t* stamps = nullptr;
        const size_t blocks = composite_views_blocks((uint32_t)max_chunks, k);
        const size_t words = blocks * (1 + (size_t)composite_views_waves_per_block());  // block starts + wave ends
        if (c0->prof_group) {
            if (!c0->stamps.p && (rc = c0->stamps.ensure(kSpanLaunches * words, "stamps"))) return rc;
            if (c0->stamp_used + words <= c0->stamps.cap) {
                stamps = c0->stamps.p + c0->stamp_used;
                c0->spans.emplace_back(c0->stamp_used, blocks);
                c0->stamp_used += words;
            }
        }
        if ((rc = launch_composite_views(fv, k, (uint32_t)max_chunks, c0->len_classes, c0->first_major, c0->views_interleave, u0,
                                         frag_class_of(u0.render_mod), f0.t_min, f0.bg, f0.out_layout,
                                         c0->tail_merge_group, c0->debug_handoff, s, stamps)))
            return rc;
        if (c0->prof_group) {
            GSR_HIP_CHECK(hipEventRecord(c0->evg[gslot][1], s));
            c0->evg_pending[gslot] = true;
            c0->evg_views[gslot] = k;
            c0->evg_slot = gslot ^ 1;
        }
        if ((rc = launch_merge_views(fv, k, u0, f0.t_min, f0.bg, f0.out_layout, c0->tail_merge_group, s)))
            return rc;
    }
    const auto h3 = std::chrono::steady_clock::now();
    using ms = std::chrono::duration<double, std::milli>;
    for (int v = 0; v < k; ++v) {
        gsr_context* c = ctxs[v];
        c->host_ms[1] += ms(h2 - h1).count() / k;
        c->host_ms[2] += ms(h3 - h2).count() / k;
        c->host_frames += 1;
        c->frame_idx += 1;
        c->stats.n_visible = fv[v].n_vis;
        c->stats.n_instances = fv[v].n_dup;
        c->last_packed = c->pend.packed;
        c->last_coarse = 0;
        c->last_chunk = f0.blend == GSR_BLEND_UNORM8 ? 0u : c0->chunk_views;
        c->last_deep = false;
    }
    return GSR_OK;
}

int gsr_render(gsr_context* c, const gsr_scene* sc, const gsr_camera* cam, const gsr_settings* st, float* out,
               int32_t* radii, void* stream) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    c->depth_passes_now = c->depth_passes_alone;  // nothing else in flight: the widest digits
    int rc = gsr_render_begin(c, sc, cam, st, out, radii, stream);
    c->depth_passes_now = 0;
    if (rc) return rc;
    return gsr_render_finish(c, stream);
}

int gsr_context_set_profiling(gsr_context* c, int32_t enable) {
    if (!c) return set_error(GSR_ERR_INVALID, "null argument");
    if (enable < 0 || enable > 2) return set_error(GSR_ERR_INVALID, "set_profiling: enable must be 0, 1 or 2");
    if (enable == 2) {  // group compositing launches (gsr_render_finish_views led by this context)
        if (!c->evg[0][0])
            for (auto& row : c->evg)
                for (auto& e : row) GSR_HIP_CHECK(hipEventCreate(&e));
        for (int k = 0; k < 2; ++k) prof_group_accumulate(c, k);
        c->prof_group = true;
        c->prof_on = false;
        c->group_comp_ms = 0.0;
        c->group_launches = c->group_views = 0;
        c->stamp_used = 0;
        c->spans.clear();
        return GSR_OK;
    }
    c->prof_group = false;
    if (enable && !c->ev[0][0]) {
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b <= EV_COUNT; ++b) GSR_HIP_CHECK(hipEventCreate(&c->ev[a][b]));
    }
    c->prof_on = enable != 0;
    c->ev_pending[0] = c->ev_pending[1] = false;
    for (double& v : c->acc_ms) v = 0.0;
    c->prof_frames = 0;
    return GSR_OK;
}

int gsr_context_stage_times(gsr_context* c, double* ms_out, int64_t* frames_out) {
    if (!c || !ms_out) return set_error(GSR_ERR_INVALID, "null argument");
    for (int k = 0; k < 2; ++k) prof_accumulate(c, (int)((c->frame_idx + k) & 1), true);
    for (int k = 0; k < GSR_NUM_STAGES; ++k) ms_out[k] = c->acc_ms[k];
    if (frames_out) *frames_out = c->prof_frames;
    return GSR_OK;
}

int gsr_context_group_times(gsr_context* c, double* composite_ms, int64_t* launches, int64_t* views,
                            double* span_ms) {
    if (!c || !composite_ms || !launches || !views) return set_error(GSR_ERR_INVALID, "null argument");
    for (int k = 0; k < 2; ++k) prof_group_accumulate(c, (c->evg_slot + k) & 1);
    *composite_ms = c->group_comp_ms;
    *launches = c->group_launches;
    *views = c->group_views;
    if (span_ms) {
        *span_ms = 0.0;
        if (!c->spans.empty()) {
            std::vector<uint64_t> st(c->stamp_used);
            GSR_HIP_CHECK(hipDeviceSynchronize());
            GSR_HIP_CHECK(hipMemcpy(st.data(), c->stamps.p, c->stamp_used * sizeof(uint64_t), hipMemcpyDeviceToHost));
            uint64_t sum = 0;
            for (const auto& sp : c->spans) {
                const uint64_t* b = st.data() + sp.first;
                uint64_t lo = ~0ull, hi = 0;
                for (size_t i = 0; i < sp.second; ++i) lo = std::min(lo, b[i]);
                const size_t waves = (size_t)composite_views_waves_per_block() * sp.second;
                for (size_t i = 0; i < waves; ++i) hi = std::max(hi, b[sp.second + i]);
                sum += hi > lo ? hi - lo : 0;
            }
            *span_ms = (double)sum * 1e-5;  // 100 MHz constant clock
        }
    }
    return GSR_OK;
}

int64_t gsr_context_group_spans(gsr_context* c, uint64_t* spans_out, int64_t max_spans) {
    if (!c || (max_spans > 0 && !spans_out) || max_spans < 0) return set_error(GSR_ERR_INVALID, "null argument");
    if (c->spans.empty()) return 0;
    std::vector<uint64_t> st(c->stamp_used);
    GSR_HIP_CHECK(hipDeviceSynchronize());
    GSR_HIP_CHECK(hipMemcpy(st.data(), c->stamps.p, c->stamp_used * sizeof(uint64_t), hipMemcpyDeviceToHost));
    int64_t i = 0;
    for (const auto& sp : c->spans) {
        const uint64_t* b = st.data() + sp.first;
        uint64_t lo = ~0ull, hi = 0;
        for (size_t q = 0; q < sp.second; ++q) lo = std::min(lo, b[q]);
        const size_t waves = (size_t)composite_views_waves_per_block() * sp.second;
        for (size_t q = 0; q < waves; ++q) hi = std::max(hi, b[sp.second + q]);
        if (i < max_spans) {
            spans_out[2 * i] = lo;
            spans_out[2 * i + 1] = std::max(lo, hi);
        }
        ++i;
    }
    return i;
}

int gsr_debug_host_times(const gsr_context* c, double ms_out[3], int64_t* frames_out) {
    if (!c || !ms_out) return set_error(GSR_ERR_INVALID, "null argument");
    for (int k = 0; k < 3; ++k) ms_out[k] = c->host_ms[k];
    if (frames_out) *frames_out = c->host_frames;
    return GSR_OK;
}

int gsr_debug_stall(void* stream, uint32_t microseconds) {
    if (microseconds > 5000000u) return set_error(GSR_ERR_INVALID, "debug_stall: at most 5 s");
    const uint64_t ticks = (uint64_t)microseconds * 100u;  // s_memrealtime runs at 100 MHz
    k_stall<<<1, 64, 0, (hipStream_t)stream>>>(ticks);
    GSR_LAUNCH_CHECK("debug_stall");
    return GSR_OK;
}

int64_t gsr_debug_copy(const gsr_context* c, int32_t what, void* dst, int64_t max_bytes, void* stream) {
    if (!c || !dst || max_bytes < 0) return set_error(GSR_ERR_INVALID, "null argument");
    const void* src = nullptr;
    int64_t bytes = 0;
    switch (what) {
        case GSR_DEBUG_RECORDS:  // the fused cull's slots are not compacted: all n (slot n-1-i)
            src = c->recs.p;
            bytes = (c->fused_cull && c->stats.n_visible > 0 ? c->stats.n_gaussians : c->stats.n_visible) *
                    (int64_t)sizeof(SplatRec);
            break;
        case GSR_DEBUG_DEPTH_ORDER: src = c->last_depth_order; bytes = c->stats.n_visible * 4; break;
        case GSR_DEBUG_TILE_RANGES: src = c->last_ranges; bytes = c->last_tiles * 8; break;
        case GSR_DEBUG_TILE_LIST: src = c->last_tile_list; bytes = c->stats.n_instances * 4; break;
        default: return set_error(GSR_ERR_INVALID, "unknown debug array");
    }
    if (!src || bytes == 0) return 0;
    if (bytes > max_bytes) bytes = max_bytes;
    GSR_HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return bytes;
}

int gsr_debug_sort_pairs(gsr_context* c, const uint32_t* keys_dev, int64_t n, int32_t bits, int32_t passes,
                         uint32_t* keys_out_dev, uint32_t* vals_out_dev, void* stream) {
    if (!c || !keys_dev || !keys_out_dev || !vals_out_dev || n < 0) return set_error(GSR_ERR_INVALID, "null argument");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) return GSR_OK;
    const size_t un = (size_t)n;
    int rc = ensure_scene_buffers(c, un);
    if (rc) return rc;
    if ((rc = c->zero.ensure(ZeroLayout(0).total, "zero block"))) return rc;
    GSR_HIP_CHECK(hipMemcpyAsync(c->keys_a.p, keys_dev, un * 4, hipMemcpyDeviceToDevice, s));
    uint32_t *ka = c->keys_a.p, *kb = c->keys_b.p, *va = c->vals_a.p, *vb = c->vals_b.p;
    if ((rc = sort_pairs(c, &ka, &va, &kb, &vb, true, un, nullptr, bits, passes, nullptr,
                         c->zero.p + ZeroLayout(0).totals_depth, s)))
        return rc;
    GSR_HIP_CHECK(hipMemcpyAsync(keys_out_dev, ka, un * 4, hipMemcpyDeviceToDevice, s));
    GSR_HIP_CHECK(hipMemcpyAsync(vals_out_dev, va, un * 4, hipMemcpyDeviceToDevice, s));
    return GSR_OK;
}

int gsr_sort_depth(gsr_context* c, const gsr_scene* sc, const float view[16], int32_t* index_dev, void* stream) {
    if (!c || !sc || !view || !index_dev) return set_error(GSR_ERR_INVALID, "null argument");
    hipStream_t s = (hipStream_t)stream;
    const size_t n = (size_t)sc->d.n;
    if (n == 0) return GSR_OK;
    int rc = ensure_scene_buffers(c, n);
    if (rc) return rc;
    if ((rc = c->zero.ensure(ZeroLayout(0).total, "zero block"))) return rc;
    GSR_HIP_CHECK(hipMemsetAsync(c->zero.p, 0, sizeof(uint32_t) * ZeroLayout(0).total, s));
    if ((rc = launch_depth_keys_all(sc->d, view, c->keys_a.p, s))) return rc;
    uint32_t *ka = c->keys_a.p, *kb = c->keys_b.p, *va = c->vals_a.p, *vb = c->vals_b.p;
    if ((rc = sort_pairs(c, &ka, &va, &kb, &vb, true, n, nullptr, 32, kDepthPasses, nullptr,
                         c->zero.p + ZeroLayout(0).totals_depth, s)))
        return rc;
    GSR_HIP_CHECK(hipMemcpyAsync(index_dev, va, n * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    return GSR_OK;
}

}  // extern "C"

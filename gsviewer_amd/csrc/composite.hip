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
// one wave64 per tile, 4 pixels per lane (4 horizontal 16x4 slices).  The
// tile's instance list and the 64-B splat records are wave-uniform, so they
// are read with scalar loads (SMEM) straight into SGPRs: no LDS staging, no
// workgroup barriers, and every wave retires independently as soon as all its
// 256 pixels are saturated (transmittance < t_min).  Slices a splat's row span
// misses are skipped with a scalar branch.
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_dup_count(const uint32_t* __restrict__ sorted_ids,
                                                        const SplatRec* __restrict__ recs, uint32_t n_vis,
                                                        uint32_t* __restrict__ counts) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= n_vis) return;
    const int4 q = reinterpret_cast<const int4*>(recs + sorted_ids[r])[2];
    const int4 t = reinterpret_cast<const int4*>(recs + sorted_ids[r])[3];
    const int x0 = q.w, x1 = t.x, r0 = t.y, r1 = t.z;
    uint32_t c = 0;
    if (x0 <= x1 && r0 <= r1) c = (uint32_t)(((x1 >> 4) - (x0 >> 4) + 1) * ((r1 >> 4) - (r0 >> 4) + 1));
    counts[r] = c;
}

__global__ __launch_bounds__(kThreads) void k_dup_write(const uint32_t* __restrict__ sorted_ids,
                                                        const SplatRec* __restrict__ recs, uint32_t n_vis,
                                                        const uint32_t* __restrict__ offsets, int tiles_x,
                                                        uint32_t* __restrict__ tile_keys,
                                                        uint32_t* __restrict__ tile_vals) {
    const uint32_t r = blockIdx.x * kThreads + threadIdx.x;
    if (r >= n_vis) return;
    const uint32_t id = sorted_ids[r];
    const int4 q = reinterpret_cast<const int4*>(recs + id)[2];
    const int4 t = reinterpret_cast<const int4*>(recs + id)[3];
    const int x0 = q.w, x1 = t.x, r0 = t.y, r1 = t.z;
    if (x0 > x1 || r0 > r1) return;
    uint32_t o = offsets[r];
    for (int ty = r0 >> 4; ty <= (r1 >> 4); ++ty)
        for (int tx = x0 >> 4; tx <= (x1 >> 4); ++tx) {
            tile_keys[o] = (uint32_t)(ty * tiles_x + tx);
            tile_vals[o] = id;
            ++o;
        }
}

__global__ __launch_bounds__(kThreads) void k_tile_ranges(const uint32_t* __restrict__ keys, uint32_t n,
                                                          uint2* __restrict__ ranges) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = keys[i];
    if (i == 0 || keys[i - 1] != k) ranges[k].x = i;
    if (i == n - 1 || keys[i + 1] != k) ranges[k].y = i + 1;
}

struct CompositeArgs {
    int width, height, tiles_x, num_tiles;
    float t_min;
    float bg[3];
    int out_layout;
};

template <int FRAG>
__global__ __launch_bounds__(kThreads) void k_composite(const uint2* __restrict__ ranges,
                                                        const uint32_t* __restrict__ list,
                                                        const SplatRec* __restrict__ recs, CompositeArgs a,
                                                        float* __restrict__ out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.x * (kThreads / 64) + wave;
    if (tile >= a.num_tiles) return;
    const int lane = __lane_id();
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int x = tx * kTile + (lane & 15);
    const int row_base = ty * kTile;           // first image row of the tile (uniform)
    const int lrow = lane >> 4;                // row within a 16x4 slice
    const float px = (float)x + 0.5f;
    float pyw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) pyw[k] = (float)(a.height - 1 - (row_base + 4 * k + lrow)) + 0.5f;

    float T[4], cr[4], cg[4], cb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        T[k] = 1.f;
        cr[k] = cg[k] = cb[k] = 0.f;
    }
    const float t_min = a.t_min;
    const uint2 rg = ranges[tile];
    for (uint32_t i = rg.x; i < rg.y; ++i) {
        const SplatRec s = recs[list[i]];
        const bool inx = (x >= s.x0) & (x <= s.x1);
        const float dx = (px - s.cx) * s.sx;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int srow0 = row_base + 4 * k;
            if (srow0 > s.r1 || srow0 + 3 < s.r0) continue;  // scalar: slice misses the splat
            const int row = srow0 + lrow;
            const bool in = inx & (row >= s.r0) & (row <= s.r1) & (T[k] >= t_min);
            float alpha, fr = s.r, fg = s.g, fb = s.b;
            bool keep;
            if (FRAG == kFragBillboard) {
                alpha = 1.0f;
                keep = in;
            } else {
                const float dy = (pyw[k] - s.cy) * s.sy;
                const float power = -0.5f * (s.A * dx * dx + s.C * dy * dy) - s.B * dx * dy;
                const float e = __expf(power);
                alpha = fminf(0.99f, s.opacity * e);
                keep = in & !(power > 0.0f) & !(alpha < (1.0f / 255.0f));
                if (FRAG == kFragFlatBall || FRAG == kFragGaussBall) alpha = (alpha > 0.22f) ? 1.0f : 0.0f;
                if (FRAG == kFragGaussBall) {
                    fr = fminf(fmaxf(fr * e, 0.f), 1.f);
                    fg = fminf(fmaxf(fg * e, 0.f), 1.f);
                    fb = fminf(fmaxf(fb * e, 0.f), 1.f);
                }
            }
            if (keep) {
                const float w = alpha * T[k];
                cr[k] += fr * w;
                cg[k] += fg * w;
                cb[k] += fb * w;
                T[k] = T[k] * (1.0f - alpha);
            }
        }
        if (t_min > 0.f) {
            const bool live = (T[0] >= t_min) | (T[1] >= t_min) | (T[2] >= t_min) | (T[3] >= t_min);
            if (!__any(live)) break;
        }
    }

    if (x >= a.width) return;
    const size_t plane = (size_t)a.width * a.height;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = row_base + 4 * k + lrow;
        if (row >= a.height) continue;
        const float r = cr[k] + T[k] * a.bg[0];
        const float g = cg[k] + T[k] * a.bg[1];
        const float b = cb[k] + T[k] * a.bg[2];
        const size_t p = (size_t)row * a.width + x;
        if (a.out_layout == 0) {
            out[p] = r;
            out[plane + p] = g;
            out[2 * plane + p] = b;
        } else {
            out[3 * p] = r;
            out[3 * p + 1] = g;
            out[3 * p + 2] = b;
        }
    }
}

}  // namespace

int launch_dup_count(const uint32_t* sorted_ids, const SplatRec* recs, uint32_t n_vis, uint32_t* counts,
                     hipStream_t s) {
    if (n_vis == 0) return GSR_OK;
    k_dup_count<<<(n_vis + kThreads - 1) / kThreads, kThreads, 0, s>>>(sorted_ids, recs, n_vis, counts);
    GSR_LAUNCH_CHECK("dup_count");
    return GSR_OK;
}

int launch_dup_write(const uint32_t* sorted_ids, const SplatRec* recs, uint32_t n_vis, const uint32_t* offsets,
                     int tiles_x, uint32_t* tile_keys, uint32_t* tile_vals, hipStream_t s) {
    if (n_vis == 0) return GSR_OK;
    k_dup_write<<<(n_vis + kThreads - 1) / kThreads, kThreads, 0, s>>>(sorted_ids, recs, n_vis, offsets, tiles_x,
                                                                       tile_keys, tile_vals);
    GSR_LAUNCH_CHECK("dup_write");
    return GSR_OK;
}

int launch_tile_ranges(const uint32_t* tile_keys, uint32_t n_dup, uint2* ranges, hipStream_t s) {
    if (n_dup == 0) return GSR_OK;
    k_tile_ranges<<<(n_dup + kThreads - 1) / kThreads, kThreads, 0, s>>>(tile_keys, n_dup, ranges);
    GSR_LAUNCH_CHECK("tile_ranges");
    return GSR_OK;
}

int launch_composite(const uint2* ranges, const uint32_t* tile_vals, const SplatRec* recs, const FrameUniforms& u,
                     int frag_class, float t_min, const float* bg, int out_layout, float* out, hipStream_t s) {
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
    const unsigned grid = (unsigned)((a.num_tiles + 3) / 4);
    switch (frag_class) {
        case kFragGauss: k_composite<kFragGauss><<<grid, kThreads, 0, s>>>(ranges, tile_vals, recs, a, out); break;
        case kFragBillboard: k_composite<kFragBillboard><<<grid, kThreads, 0, s>>>(ranges, tile_vals, recs, a, out); break;
        case kFragFlatBall: k_composite<kFragFlatBall><<<grid, kThreads, 0, s>>>(ranges, tile_vals, recs, a, out); break;
        default: k_composite<kFragGaussBall><<<grid, kThreads, 0, s>>>(ranges, tile_vals, recs, a, out); break;
    }
    GSR_LAUNCH_CHECK("composite");
    return GSR_OK;
}

}  // namespace gsr

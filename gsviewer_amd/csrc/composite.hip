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
// one wave64 per chunk of a tile's list (see k_chunk_count), 4 pixels per lane
// (four horizontal 16x4 slices), records staged per wave through LDS, no
// workgroup barriers; a wave retires as soon as all its 256 pixels are
// saturated (transmittance < t_min).  Slices a splat's row span misses are
// skipped with a scalar branch.
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

constexpr int kBatch = 64;  // records staged per wave per LDS batch

// Chunks: every tile's instance list is cut into pieces of at most `chunk`
// instances (an empty tile gets one empty chunk so it still writes the
// background).  Front-to-back "over" is associative:
//   (C1, T1) then (C2, T2)  ==  (C1 + T1*C2, T1*T2)
// so chunks of one tile are composited by different waves in parallel and
// folded in depth order afterwards (k_merge).  This bounds the work of one
// wave, which is what the heavy tiles of a real scene (horizon lines,
// dense cores) need.
__global__ __launch_bounds__(kThreads) void k_chunk_count(const uint2* __restrict__ ranges, int num_tiles,
                                                          uint32_t chunk, uint32_t* __restrict__ counts) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= num_tiles) return;
    const uint2 r = ranges[t];
    const uint32_t len = r.y - r.x;
    counts[t] = len == 0 ? 1u : (len + chunk - 1) / chunk;
}

__global__ __launch_bounds__(kThreads) void k_chunk_write(const uint2* __restrict__ ranges, int num_tiles,
                                                          uint32_t chunk, const uint32_t* __restrict__ offsets,
                                                          uint4* __restrict__ desc) {
    const int t = blockIdx.x * kThreads + threadIdx.x;
    if (t >= num_tiles) return;
    const uint2 r = ranges[t];
    const uint32_t len = r.y - r.x;
    const uint32_t cnt = len == 0 ? 1u : (len + chunk - 1) / chunk;
    const uint32_t o = offsets[t];
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t b = r.x + k * chunk;
        const uint32_t e = min(r.y, b + chunk);
        desc[o + k] = make_uint4((uint32_t)t, b, e, (cnt << 16) | k);
    }
}

// One wave per chunk, 4 pixels per lane (four 16x4 slices of the 16x16 tile).
// Records of the chunk are gathered 64 at a time (one 64-B record per lane,
// prefetched one batch ahead in registers) into a wave-private LDS buffer and
// then read back with wave-uniform (broadcast) ds_read_b128.  No workgroup
// barriers: the four waves of a block are independent chunks.
template <int FRAG>
__global__ __launch_bounds__(kThreads) void k_composite(const uint4* __restrict__ desc,
                                                        const uint32_t* __restrict__ n_chunks_dev,
                                                        const uint32_t* __restrict__ list,
                                                        const SplatRec* __restrict__ recs, CompositeArgs a,
                                                        float* __restrict__ out, float4* __restrict__ partial) {
    __shared__ float4 lds[kThreads / 64][kBatch * 4];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t chunk_id = blockIdx.x * (kThreads / 64) + wave;
    if (chunk_id >= n_chunks_dev[0]) return;
    const uint4 d = desc[chunk_id];
    const int tile = (int)d.x;
    const uint32_t begin = d.y, end = d.z;
    const uint32_t nchunks = d.w >> 16;
    const int lane = __lane_id();
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int x = tx * kTile + (lane & 15);
    const int row_base = ty * kTile;
    const int lrow = lane >> 4;
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
    float4* my = lds[wave];

    // prefetch first batch
    float4 f0, f1, f2, f3;
    {
        const uint32_t i = begin + lane;
        if (i < end) {
            const float4* r = reinterpret_cast<const float4*>(recs + list[i]);
            f0 = r[0]; f1 = r[1]; f2 = r[2]; f3 = r[3];
        }
    }
    for (uint32_t b = begin; b < end; b += kBatch) {
        __builtin_amdgcn_wave_barrier();
        my[lane * 4 + 0] = f0;
        my[lane * 4 + 1] = f1;
        my[lane * 4 + 2] = f2;
        my[lane * 4 + 3] = f3;
        __builtin_amdgcn_wave_barrier();
        {  // prefetch next batch while this one is composited
            const uint32_t i = b + kBatch + lane;
            if (i < end) {
                const float4* r = reinterpret_cast<const float4*>(recs + list[i]);
                f0 = r[0]; f1 = r[1]; f2 = r[2]; f3 = r[3];
            }
        }
        const int nb = (int)min((uint32_t)kBatch, end - b);
        for (int j = 0; j < nb; ++j) {
            const float4 q0 = my[j * 4 + 0];  // cx cy sx sy
            const float4 q1 = my[j * 4 + 1];  // A B C opacity
            const float4 q2 = my[j * 4 + 2];  // r g b x0
            const float4 q3 = my[j * 4 + 3];  // x1 r0 r1 -
            const int sx0 = __float_as_int(q2.w), sx1 = __float_as_int(q3.x);
            const int sr0 = __builtin_amdgcn_readfirstlane(__float_as_int(q3.y));
            const int sr1 = __builtin_amdgcn_readfirstlane(__float_as_int(q3.z));
            const bool inx = (x >= sx0) & (x <= sx1);
            const float dx = (px - q0.x) * q0.z;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int srow0 = row_base + 4 * k;
                if (srow0 > sr1 || srow0 + 3 < sr0) continue;  // scalar: slice misses the splat
                const int row = srow0 + lrow;
                const bool in = inx & (row >= sr0) & (row <= sr1) & (T[k] >= t_min);
                float alpha, fr = q2.x, fg = q2.y, fb = q2.z;
                bool keep;
                if (FRAG == kFragBillboard) {
                    alpha = 1.0f;
                    keep = in;
                } else {
                    const float dy = (pyw[k] - q0.y) * q0.w;
                    const float power = -0.5f * (q1.x * dx * dx + q1.z * dy * dy) - q1.y * dx * dy;
                    const float e = __expf(power);
                    alpha = fminf(0.99f, q1.w * e);
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
        }
        if (t_min > 0.f) {
            // a pixel whose chunk-local T is below t_min has absolute T below it too
            const bool live = (T[0] >= t_min) | (T[1] >= t_min) | (T[2] >= t_min) | (T[3] >= t_min);
            if (!__any(live)) break;
        }
    }

    if (nchunks > 1) {
        // partial (C, T) per pixel, folded by k_merge; layout [chunk][k][lane]
        float4* p = partial + (size_t)chunk_id * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k) p[k * 64 + lane] = make_float4(cr[k], cg[k], cb[k], T[k]);
        return;
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
        const size_t pidx = (size_t)row * a.width + x;
        if (a.out_layout == 0) {
            out[pidx] = r;
            out[plane + pidx] = g;
            out[2 * plane + pidx] = b;
        } else {
            out[3 * pidx] = r;
            out[3 * pidx + 1] = g;
            out[3 * pidx + 2] = b;
        }
    }
}

// Fold the partial results of multi-chunk tiles in depth order; one wave per tile.
__global__ __launch_bounds__(kThreads) void k_merge(const uint32_t* __restrict__ chunk_off,
                                                    const uint32_t* __restrict__ chunk_cnt,
                                                    const float4* __restrict__ partial, CompositeArgs a,
                                                    float* __restrict__ out) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.x * (kThreads / 64) + wave;
    if (tile >= a.num_tiles) return;
    const uint32_t cnt = chunk_cnt[tile];
    if (cnt <= 1) return;
    const uint32_t c0 = chunk_off[tile];
    const int lane = __lane_id();
    const int tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const int x = tx * kTile + (lane & 15);
    if (x >= a.width) return;
    const size_t plane = (size_t)a.width * a.height;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int row = ty * kTile + 4 * k + (lane >> 4);
        float r = 0.f, g = 0.f, b = 0.f, T = 1.f;
        for (uint32_t c = 0; c < cnt; ++c) {
            const float4 q = partial[(size_t)(c0 + c) * 256 + k * 64 + lane];
            r += T * q.x;
            g += T * q.y;
            b += T * q.z;
            T *= q.w;
        }
        if (row >= a.height) continue;
        r += T * a.bg[0];
        g += T * a.bg[1];
        b += T * a.bg[2];
        const size_t pidx = (size_t)row * a.width + x;
        if (a.out_layout == 0) {
            out[pidx] = r;
            out[plane + pidx] = g;
            out[2 * plane + pidx] = b;
        } else {
            out[3 * pidx] = r;
            out[3 * pidx + 1] = g;
            out[3 * pidx + 2] = b;
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

static CompositeArgs make_args(const FrameUniforms& u, float t_min, const float* bg, int out_layout) {
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
    return a;
}

int launch_chunks(const uint2* ranges, int num_tiles, uint32_t chunk, uint32_t* chunk_cnt, uint32_t* chunk_off,
                  uint32_t* scan_tmp, uint32_t* n_chunks_dev, uint4* desc, hipStream_t s) {
    const unsigned g = (unsigned)((num_tiles + kThreads - 1) / kThreads);
    k_chunk_count<<<g, kThreads, 0, s>>>(ranges, num_tiles, chunk, chunk_cnt);
    GSR_LAUNCH_CHECK("chunk_count");
    int rc = scan_exclusive(chunk_cnt, chunk_off, (size_t)num_tiles, scan_tmp, n_chunks_dev, s);
    if (rc) return rc;
    k_chunk_write<<<g, kThreads, 0, s>>>(ranges, num_tiles, chunk, chunk_off, desc);
    GSR_LAUNCH_CHECK("chunk_write");
    return GSR_OK;
}

int launch_composite(const uint4* desc, const uint32_t* n_chunks_dev, uint32_t max_chunks, const uint32_t* chunk_off,
                     const uint32_t* chunk_cnt, const uint32_t* tile_vals, const SplatRec* recs,
                     const FrameUniforms& u, int frag_class, float t_min, const float* bg, int out_layout,
                     float* out, float4* partial, hipStream_t s) {
    const CompositeArgs a = make_args(u, t_min, bg, out_layout);
    const unsigned grid = (unsigned)((max_chunks + 3) / 4);
    switch (frag_class) {
        case kFragGauss:
            k_composite<kFragGauss><<<grid, kThreads, 0, s>>>(desc, n_chunks_dev, tile_vals, recs, a, out, partial);
            break;
        case kFragBillboard:
            k_composite<kFragBillboard><<<grid, kThreads, 0, s>>>(desc, n_chunks_dev, tile_vals, recs, a, out, partial);
            break;
        case kFragFlatBall:
            k_composite<kFragFlatBall><<<grid, kThreads, 0, s>>>(desc, n_chunks_dev, tile_vals, recs, a, out, partial);
            break;
        default:
            k_composite<kFragGaussBall><<<grid, kThreads, 0, s>>>(desc, n_chunks_dev, tile_vals, recs, a, out, partial);
            break;
    }
    GSR_LAUNCH_CHECK("composite");
    k_merge<<<(unsigned)((a.num_tiles + 3) / 4), kThreads, 0, s>>>(chunk_off, chunk_cnt, partial, a, out);
    GSR_LAUNCH_CHECK("merge");
    return GSR_OK;
}

}  // namespace gsr

// Per-Gaussian stage: box cull, view/projection + frustum cull, 3D->2D
// covariance (EWA), conic, quad rectangle, SH->RGB.  The arithmetic restates
// shaders/gau_vert.glsl:75-331 (and the fixed-function viewport transform)
// in float32 with a fixed left-to-right evaluation order and NO contraction
// (this file is compiled with -ffp-contract=off), so that per-splat values
// match the CPU oracle (oracle/gl_oracle.py) bit for bit.
//
// Two launches per frame:
//   k_cull        reads pos_op only (16 B/Gaussian), writes one visibility
//                 ballot + count per wave;  -> scan of the wave counts
//   k_preprocess  recomputes the cull for its lane, and for visible lanes
//                 loads rot/scale/SH planes (coalesced float4), writes the
//                 48-B SplatRec and the depth key at its compacted slot.
// Compaction slot = n_vis-1-(rank in Gaussian-index order), so a stable
// ascending depth sort resolves exact depth ties in DESCENDING index order:
// the exact reverse of the GL draw order (renderer_ogl.py:24, ascending z,
// ties by ascending index), i.e. front-to-back.
#pragma clang fp contract(off)
#include <cstdlib>

#include "gsr_internal.h"

#include <algorithm>

namespace gsr {
namespace {

constexpr int kThreads = 256;

// gau_vert.glsl:3-18
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f;
constexpr float SH_C2_1 = -1.0925484305920792f;
constexpr float SH_C2_2 = 0.31539156525252005f;
constexpr float SH_C2_3 = -1.0925484305920792f;
constexpr float SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f;
constexpr float SH_C3_1 = 2.890611442640554f;
constexpr float SH_C3_2 = -0.4570457994644658f;
constexpr float SH_C3_3 = 0.3731763325901154f;
constexpr float SH_C3_4 = -0.4570457994644658f;
constexpr float SH_C3_5 = 1.445305721320277f;
constexpr float SH_C3_6 = -0.5900435899266435f;

// isInsideRotatedCube (gau_vert.glsl:172-191)
__device__ __forceinline__ bool inside_box(float x, float y, float z, const FrameUniforms& u) {
    if (u.enable_obb == 1) {
        const float dx = x - u.pcenter[0], dy = y - u.pcenter[1], dz = z - u.pcenter[2];
        const float* M = u.obb_inv;
        const float t0 = (M[0] * dx + M[1] * dy) + M[2] * dz;
        const float t1 = (M[3] * dx + M[4] * dy) + M[5] * dz;
        const float t2 = (M[6] * dx + M[7] * dy) + M[8] * dz;
        return (t0 >= u.cmin[0]) & (t0 <= u.cmax[0]) & (t1 >= u.cmin[1]) & (t1 <= u.cmax[1]) &
               (t2 >= u.cmin[2]) & (t2 <= u.cmax[2]);
    }
    if (u.enable_aabb == 1) {
        const float t0 = x - u.pcenter[0], t1 = y - u.pcenter[1], t2 = z - u.pcenter[2];
        return (t0 >= u.pcenter[0] + u.cmin[0]) & (t0 <= u.pcenter[0] + u.cmax[0]) &
               (t1 >= u.pcenter[1] + u.cmin[1]) & (t1 <= u.pcenter[1] + u.cmax[1]) &
               (t2 >= u.pcenter[2] + u.cmin[2]) & (t2 <= u.pcenter[2] + u.cmax[2]);
    }
    return true;
}

struct Projected {
    float pv[4];
    float ndc[3];
    bool vis;
};

// gau_vert.glsl:209-218 + GL clip of |z_ndc| > 1 (all quad vertices share z).
__device__ __forceinline__ Projected project(float x, float y, float z, const FrameUniforms& u) {
    Projected o;
    const float* V = u.V;
    const float* P = u.P;
#pragma unroll
    for (int i = 0; i < 4; ++i) o.pv[i] = ((V[4 * i] * x + V[4 * i + 1] * y) + V[4 * i + 2] * z) + V[4 * i + 3];
    float pc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        pc[i] = ((P[4 * i] * o.pv[0] + P[4 * i + 1] * o.pv[1]) + P[4 * i + 2] * o.pv[2]) + P[4 * i + 3] * o.pv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) o.ndc[k] = pc[k] / pc[3];
    const float lim = 1.3f;
    o.vis = (fabsf(o.ndc[0]) <= lim) & (fabsf(o.ndc[1]) <= lim) & (fabsf(o.ndc[2]) <= lim) &
            (o.ndc[2] >= -1.0f) & (o.ndc[2] <= 1.0f);
    o.vis = o.vis & inside_box(x, y, z, u);
    return o;
}

// GL coverage of the quad's edges lo, hi (window coordinates): the vertices
// are snapped to 8 sub-pixel bits in the frame whose pixel centres are
// integers, L = rint((lo - 0.5) * 256), and pixel p is covered iff
// L <= 256 p < H (the top-left rule on an axis-aligned rectangle).  That is
// Mesa llvmpipe's rasteriser (FIXED_ORDER 8), which runs the reference's
// shaders in tests/golden/make_gl_golden.py; oracle/gl_oracle.py pixel_span.
// rintf rounds half to even, like the oracle's np.rint; L / 256 is exact.
__device__ __forceinline__ void pixel_span(float lo, float hi, int limit, int& p0, int& p1) {
    if (!(lo == lo) || !(hi == hi)) {
        p0 = limit;
        p1 = -1;
        return;
    }
    lo = fminf(fmaxf(lo, -1048576.f), 1048576.f);
    hi = fminf(fmaxf(hi, -1048576.f), 1048576.f);
    const float L = rintf((lo - 0.5f) * 256.0f), H = rintf((hi - 0.5f) * 256.0f);
    const int a = (int)ceilf(L * 0.00390625f);
    const int b = (int)ceilf(H * 0.00390625f) - 1;
    p0 = min(max(a, -1), limit);
    p1 = min(max(b, -1), limit);
}

// The fragment's alpha box (kFragGauss): the pixel rectangle outside which
// every fragment is discarded by alpha < 1/255 (gau_frag.glsl:42).  With the
// falloff pw = qa dx^2 + qb dx dy + qc dy^2 (power * log2 e, pixel offsets,
// negative definite) a pixel is kept only if pw >= thr = -log2(255 opacity);
// the set {pw >= thr} is an ellipse with half-extents
//   hx = sqrt(thr / (qa - qb^2 / (4 qc))),  hy = sqrt(thr / (qc - qb^2 / (4 qa))).
// The covered rectangle [x0, x1] x [r0, r1] (the 3-sigma quad, image rows) is
// intersected with that box widened by 0.2 % + 0.01 px (far above the float
// rounding of pw and of the box), so no kept fragment is ever dropped: the
// result only narrows the tiles and 16x4 slices a splat is composited over.
// opacity < 1/255 (thr > 0, or NaN): nothing is ever drawn, the rectangle is
// emptied.  Forms with disc = 4 qa qc - qb^2 <= 1e-2 * 4 qa qc (correlation
// |rho| > 0.995: needles) keep the quad unchanged.  Error budget (DESIGN.md,
// "alpha-box margin"): with disc / (4 qa qc) >= 1e-2 the cancellation in
// qa - qb^2 / (4 qc) amplifies the few-ulp rounding of the terms by at most
// 2 / 1e-2 = 200, i.e. <= ~1e-4 relative on hx^2, and the compositor's pw at a
// pixel carries a relative error of the same order; the margin is 2e-3
// relative + 0.01 px, an order of magnitude above both.
// Evaluated without contraction in this fixed order: tests/helpers.py
// (alpha_box_rects) mirrors it bit for bit.
__device__ __forceinline__ void alpha_box(float qa, float qb, float qc, float thr, float cx, float cy, int height,
                                          int& x0, int& x1, int& r0, int& r1) {
    if (!(thr <= 0.0f)) {
        x0 = 1;
        x1 = 0;
        return;
    }
    const float d4 = (4.0f * qa) * qc;
    const float disc = d4 - qb * qb;
    if (!(qa < 0.0f && qc < 0.0f && disc > 1e-2f * d4)) return;
    // half-extents of {q >= thr}: hx^2 = thr / (qa - qb^2 / 4qc) = qc * 4 thr / disc, and hy^2 likewise
    // with qa (one correctly rounded division instead of four; the margin covers the rounding)
    const float s4 = (4.0f * thr) / disc;
    const float hx = sqrtf(qc * s4) * 1.002f + 0.01f;
    const float hy = sqrtf(qa * s4) * 1.002f + 0.01f;
    if (!(hx < 65536.0f && hy < 65536.0f)) return;  // (cx, cy are within 1.3x of the viewport)
    // pixel p is a candidate if its centre p + 0.5 is within [c - h, c + h]
    const int bx0 = (int)ceilf((cx - hx) - 0.5f), bx1 = (int)floorf((cx + hx) - 0.5f);
    const int bj0 = (int)ceilf((cy - hy) - 0.5f), bj1 = (int)floorf((cy + hy) - 0.5f);  // window rows
    x0 = max(x0, bx0);
    x1 = min(x1, bx1);
    r0 = max(r0, (height - 1) - bj1);  // image rows
    r1 = min(r1, (height - 1) - bj0);
}

__device__ __forceinline__ uint32_t float_order_key(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// One view's visibility of the block's Gaussians: the wave's ballot and
// count, and the block's depth-key range {~kmin, kmax} of its visible ones.
// Ends with a barrier, so s_kr can be reused by the next view.
__device__ __forceinline__ void cull_view(const float4 p, bool in_range, int64_t i, const FrameUniforms& u,
                                          uint64_t* __restrict__ vis_mask, uint32_t* __restrict__ wave_counts,
                                          uint2* __restrict__ block_ranges, uint2* s_kr) {
    bool vis = false;
    uint32_t key = 0;
    if (in_range) {
        const Projected pr = project(p.x, p.y, p.z, u);
        vis = pr.vis;
        key = float_order_key(-pr.pv[2]);  // the depth key k_preprocess writes
    }
    const uint64_t m = __ballot(vis);
    if (__lane_id() == 0) {
        vis_mask[i >> 6] = m;
        wave_counts[i >> 6] = (uint32_t)__popcll(m);
    }
    // depth-key range of the visible Gaussians ({~kmin, kmax}, componentwise max)
    const uint32_t a = wave_reduce_max(vis ? ~key : 0u), b = wave_reduce_max(vis ? key : 0u);
    if (__lane_id() == 0) s_kr[threadIdx.x >> 6] = make_uint2(a, b);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint2 r = s_kr[0];
#pragma unroll
        for (int w = 1; w < kThreads / 64; ++w) r = make_uint2(max(r.x, s_kr[w].x), max(r.y, s_kr[w].y));
        block_ranges[blockIdx.x] = r;
    }
    __syncthreads();
}

// write-through (sc1) stores: several of these words are later updated by
// atomics, which act at the coherence point, not in this XCD's L2
__device__ __forceinline__ void clear_words(uint32_t* zero_words, uint32_t n_zero) {
    for (int64_t z = (int64_t)blockIdx.x * kThreads + threadIdx.x; z < (int64_t)n_zero;
         z += (int64_t)gridDim.x * kThreads)
        __hip_atomic_store(zero_words + z, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Also clears the frame's zero block (tile ranges, saturation words): they
// are first used several launches later, so no memset launch is needed.
__global__ __launch_bounds__(kThreads) void k_cull(const float4* __restrict__ pos_op, int64_t n, FrameUniforms u,
                                                   uint64_t* __restrict__ vis_mask, uint32_t* __restrict__ wave_counts,
                                                   uint2* __restrict__ block_ranges, uint32_t* __restrict__ zero_words,
                                                   uint32_t n_zero) {
    static_assert(kThreads == kCullBlock, "one key range per cull block");
    __shared__ uint2 s_kr[kThreads / 64];
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    clear_words(zero_words, n_zero);
    const float4 p = i < n ? pos_op[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    cull_view(p, i < n, i, u, vis_mask, wave_counts, block_ranges, s_kr);
}

// Several views of one scene (gsr_render_begin_views): each position is read
// once for all of them.
struct ViewCull {
    FrameUniforms u;
    uint64_t* vis_mask;
    uint32_t* wave_counts;
    uint2* block_ranges;
    uint32_t* zero_words;
    uint32_t n_zero;
};
struct ViewsCull {
    ViewCull v[kMaxViews];
    int32_t k;
};
static_assert(sizeof(ViewsCull) <= 3584, "kernel argument size");

__global__ __launch_bounds__(kThreads) void k_cull_views(const float4* __restrict__ pos_op, int64_t n, ViewsCull vc) {
    __shared__ uint2 s_kr[kThreads / 64];
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    for (int v = 0; v < vc.k; ++v) clear_words(vc.v[v].zero_words, vc.v[v].n_zero);
    const float4 p = i < n ? pos_op[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
    for (int v = 0; v < vc.k; ++v)
        cull_view(p, i < n, i, vc.v[v].u, vc.v[v].vis_mask, vc.v[v].wave_counts, vc.v[v].block_ranges, s_kr);
}

struct V3 {
    float x, y, z;
};

__device__ __forceinline__ V3 normalize3(float vx, float vy, float vz) {
    const float nn = sqrtf((vx * vx + vy * vy) + vz * vz);
    return V3{vx / nn, vy / nn, vz / nn};
}

// kNT: a frame alone reads the scene's attributes non-temporally.  They are
// read once per frame, and the default policy's L2/MALL allocations evicted
// what the depth sort and binning then re-read (their keys, ids and
// rectangles): C2 frame alone preprocess 66 -> 60 us, depth sort 52.4 -> 48.8,
// binning -2 (latency 0.326 -> 0.314 ms, profiles/r5_s50).  A group's frames
// keep the default (in flight no faster with it); the positions too (read by
// every lane, non-temporal no faster alone: r5_s51).
template <bool kNT = false>
__device__ __forceinline__ float4 load_stream(const float4* __restrict__ a, int64_t i) {
    if constexpr (kNT) {
        typedef float nt4 __attribute__((ext_vector_type(4)));
        const nt4 v = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(a) + i);
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return a[i];
    }
}

template <bool kNT = false>
__device__ __forceinline__ float4 load_plane(const float4* __restrict__ sh, int64_t n, int p, int64_t i) {
    return load_stream<kNT>(sh, (int64_t)p * n + i);
}

// SH floats needed at effective degree DEG (gau_vert.glsl:289-327 gates).
template <int DEG>
constexpr int sh_planes_for() {
    return DEG < 0 ? 0 : DEG == 0 ? 1 : DEG == 1 ? 3 : DEG == 2 ? 7 : 12;
}

// Colour varying, gau_vert.glsl:274-330, evaluated at effective degree DEG
// (the host picks DEG = what `sh_dim > 3/12/27 && render_mod >= 1/2/3`
// enables).  f[] holds the preloaded SH floats of this Gaussian.
template <int DEG>
__device__ __forceinline__ V3 sh_color(const float (&f)[48], float x, float y, float z, const FrameUniforms& u) {
    // dir = normalize(g_pos.xyz - cam_pos), rotateLightDirection
    V3 d = normalize3(x - u.campos[0], y - u.campos[1], z - u.campos[2]);
    float dx = d.x, dy = d.y, dz = d.z;
    {
        const float ry = dy * u.lcos[0] - dz * u.lsin[0];
        const float rz = dy * u.lsin[0] + dz * u.lcos[0];
        dy = ry;
        dz = rz;
    }
    {
        const float rx = dx * u.lcos[1] + dz * u.lsin[1];
        const float rz = -dx * u.lsin[1] + dz * u.lcos[1];
        dx = rx;
        dz = rz;
    }
    {
        const float rx = dx * u.lcos[2] - dy * u.lsin[2];
        const float ry = dx * u.lsin[2] + dy * u.lcos[2];
        dx = rx;
        dy = ry;
    }
#define G(k, c) f[3 * (k) + (c)]
    float col[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) col[c] = SH_C0 * G(0, c);
    if (DEG >= 1) {
        const float X = dx, Y = dy, Z = dz;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            col[c] = ((col[c] - (SH_C1 * Y) * G(1, c)) + (SH_C1 * Z) * G(2, c)) - (SH_C1 * X) * G(3, c);
            col[c] = col[c] * u.dc_factor;
        }
        if (DEG >= 2) {
            const float xx = X * X, yy = Y * Y, zz = Z * Z;
            const float xy = X * Y, yz = Y * Z, xz = X * Z;
            const float k4 = SH_C2_0 * xy, k5 = SH_C2_1 * yz, k6 = SH_C2_2 * ((2.0f * zz - xx) - yy);
            const float k7 = SH_C2_3 * xz, k8 = SH_C2_4 * (xx - yy);
#pragma unroll
            for (int c = 0; c < 3; ++c)
                col[c] = ((((col[c] + k4 * G(4, c)) + k5 * G(5, c)) + k6 * G(6, c)) + k7 * G(7, c)) + k8 * G(8, c);
            if (DEG >= 3) {
                const float k9 = (SH_C3_0 * Y) * (3.0f * xx - yy);
                const float k10 = (SH_C3_1 * xy) * Z;
                const float k11 = (SH_C3_2 * Y) * ((4.0f * zz - xx) - yy);
                const float k12 = (SH_C3_3 * Z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
                const float k13 = (SH_C3_4 * X) * ((4.0f * zz - xx) - yy);
                const float k14 = (SH_C3_5 * Z) * (xx - yy);
                const float k15 = (SH_C3_6 * X) * (xx - 3.0f * yy);
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    col[c] = ((((((col[c] + k9 * G(9, c)) + k10 * G(10, c)) + k11 * G(11, c)) + k12 * G(12, c)) +
                               k13 * G(13, c)) +
                              k14 * G(14, c)) +
                             k15 * G(15, c);
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) col[c] = col[c] * u.extra_factor;
        }
    }
#undef G
    V3 o;
    o.x = (col[0] + 0.5f) * u.cscale[0];
    o.y = (col[1] + 0.5f) * u.cscale[1];
    o.z = (col[2] + 0.5f) * u.cscale[2];
    return o;
}

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }

// The scene data of one Gaussian at effective SH degree DEG.
template <int DEG>
struct GaussLoad {
    float4 po, q1, sc4;
    float f[48];
};

// Issue every load of Gaussian i (all unconditional at this DEG), the ones
// needed first first: vmcnt waits are in issue order.
template <int DEG>
__device__ __forceinline__ void load_gaussian(GaussLoad<DEG>& g, const float4* __restrict__ pos_op,
                                              const float4* __restrict__ rot, const float4* __restrict__ scale,
                                              const float4* __restrict__ sh, int64_t n, int64_t i) {
    g.po = pos_op[i];
    g.q1 = rot[i];
    g.sc4 = scale[i];
#pragma unroll
    for (int p = 0; p < 12; ++p) {
        if (p < sh_planes_for<DEG>()) {
            const float4 t = load_plane(sh, n, p, i);
            g.f[4 * p + 0] = t.x;
            g.f[4 * p + 1] = t.y;
            g.f[4 * p + 2] = t.z;
            g.f[4 * p + 3] = t.w;
        } else {
            g.f[4 * p + 0] = g.f[4 * p + 1] = g.f[4 * p + 2] = g.f[4 * p + 3] = 0.f;
        }
    }
}

// The world-space covariance of a Gaussian: view-independent, so the views of
// a group (k_preprocess_views) compute it once per Gaussian.
struct Cov3 {
    float S[3][3];
};

__device__ __forceinline__ Cov3 cov3d(const float4 q1, const float4 sc4, const FrameUniforms& u) {
    // quatMultiply(g_rot, rot_modifier) (gau_vert.glsl:134-141, :224)
    const float q1x = q1.x, q1y = q1.y, q1z = q1.z, q1w = q1.w;
    const float q2x = u.rotmod[0], q2y = u.rotmod[1], q2z = u.rotmod[2], q2w = u.rotmod[3];
    const float qx = ((q1w * q2x + q1x * q2w) + q1y * q2z) - q1z * q2y;
    const float qy = ((q1w * q2y - q1x * q2z) + q1y * q2w) + q1z * q2x;
    const float qz = ((q1w * q2z + q1x * q2y) - q1y * q2x) + q1z * q2w;
    const float qw = ((q1w * q2w - q1x * q2x) - q1y * q2y) - q1z * q2z;

    // computeCov3D (gau_vert.glsl:75-95): (r,x,y,z) = q.xyzw
    const float s[3] = {sc4.x * u.gsf, sc4.y * u.gsf, sc4.z * u.gsf};
    const float r = qx, qx_ = qy, qy_ = qz, qz_ = qw;
    const float R[3][3] = {
        {1.0f - 2.0f * (qy_ * qy_ + qz_ * qz_), 2.0f * (qx_ * qy_ + r * qz_), 2.0f * (qx_ * qz_ - r * qy_)},
        {2.0f * (qx_ * qy_ - r * qz_), 1.0f - 2.0f * (qx_ * qx_ + qz_ * qz_), 2.0f * (qy_ * qz_ + r * qx_)},
        {2.0f * (qx_ * qz_ + r * qy_), 2.0f * (qy_ * qz_ - r * qx_), 1.0f - 2.0f * (qx_ * qx_ + qy_ * qy_)}};
    float M[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) M[a][b] = s[a] * R[a][b];
    float S[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = a; b < 3; ++b) {
            S[a][b] = (M[0][a] * M[0][b] + M[1][a] * M[1][b]) + M[2][a] * M[2][b];
            S[b][a] = S[a][b];
        }

    Cov3 c;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) c.S[a][b] = S[a][b];
    return c;
}

template <int DEG>
__device__ __forceinline__ uint32_t preprocess_compute(const GaussLoad<DEG>& g, const Cov3& S3, const FrameUniforms& u,
                                                       uint64_t m, int64_t i, uint32_t slot_base,
                                                       SplatRec* __restrict__ recs, uint32_t* __restrict__ depth_keys,
                                                       uint2* __restrict__ trect, int32_t* __restrict__ radii,
                                                       uint32_t& key);

// Per-Gaussian body of k_preprocess for a visible lane; returns the number of
// 16x16 tiles its covered pixel rectangle touches.
template <int DEG>
__device__ __forceinline__ uint32_t preprocess_one(const float4* __restrict__ pos_op, const float4* __restrict__ rot,
                                                  const float4* __restrict__ scale, const float4* __restrict__ sh,
                                                  int64_t n, const FrameUniforms& u, uint64_t m, int64_t i,
                                                  const uint32_t* __restrict__ wave_off,
                                                  const uint32_t* __restrict__ n_vis_dev, SplatRec* __restrict__ recs,
                                                  uint32_t* __restrict__ depth_keys, uint2* __restrict__ trect,
                                                  int32_t* __restrict__ radii) {
    GaussLoad<DEG> g;
    load_gaussian<DEG>(g, pos_op, rot, scale, sh, n, i);
    const uint32_t slot_base = n_vis_dev[0] - 1u - wave_off[i >> 6];
    // keep the compiler from sinking the loads below the arithmetic (it would
    // otherwise wait for pos/rot/scale before issuing the SH planes: two
    // dependent memory round trips per wave instead of one)
    __builtin_amdgcn_sched_barrier(0);
    uint32_t key;
    return preprocess_compute<DEG>(g, cov3d(g.q1, g.sc4, u), u, m, i, slot_base, recs, depth_keys, trect, radii, key);
}

// Everything after the loads: the vertex stage of one view for a visible lane
// (S3: the Gaussian's covariance, cov3d).
template <int DEG>
__device__ __forceinline__ uint32_t preprocess_compute(const GaussLoad<DEG>& g, const Cov3& S3, const FrameUniforms& u,
                                                       uint64_t m, int64_t i, uint32_t slot_base,
                                                       SplatRec* __restrict__ recs, uint32_t* __restrict__ depth_keys,
                                                       uint2* __restrict__ trect, int32_t* __restrict__ radii,
                                                       uint32_t& key) {
    const float4 po = g.po;
    const float x = po.x, y = po.y, z = po.z;
    const Projected pr = project(x, y, z, u);

    const float(&S)[3][3] = S3.S;

    // computeCov2D (gau_vert.glsl:97-122)
    const float fx = u.hfov[2], fy = u.hfov[2];
    float tx = pr.pv[0], ty = pr.pv[1];
    const float tz = pr.pv[2];
    const float limx = 1.3f * u.hfov[0];
    const float limy = 1.3f * u.hfov[1];
    const float txtz = tx / tz;
    const float tytz = ty / tz;
    tx = fminf(limx, fmaxf(-limx, txtz)) * tz;
    ty = fminf(limy, fmaxf(-limy, tytz)) * tz;
    const float tz2 = tz * tz;
    const float j0[3] = {fx / tz, 0.0f, -(fx * tx) / tz2};
    const float j1[3] = {0.0f, fy / tz, -(fy * ty) / tz2};
    const float* V = u.V;
    float uu[3], vv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        uu[k] = (V[0 + k] * j0[0] + V[4 + k] * j0[1]) + V[8 + k] * j0[2];
        vv[k] = (V[0 + k] * j1[0] + V[4 + k] * j1[1]) + V[8 + k] * j1[2];
    }
    float Su[3], Sv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        Su[k] = (S[k][0] * uu[0] + S[k][1] * uu[1]) + S[k][2] * uu[2];
        Sv[k] = (S[k][0] * vv[0] + S[k][1] * vv[1]) + S[k][2] * vv[2];
    }
    const float ca = ((uu[0] * Su[0] + uu[1] * Su[1]) + uu[2] * Su[2]) + 0.3f;
    const float cb = (vv[0] * Su[0] + vv[1] * Su[1]) + vv[2] * Su[2];
    const float cc = ((vv[0] * Sv[0] + vv[1] * Sv[1]) + vv[2] * Sv[2]) + 0.3f;

    // conic (gau_vert.glsl:235-240)
    const float det = ca * cc - cb * cb;
    const float det_inv = 1.0f / det;
    SplatRec rec;
    const float cA = cc * det_inv;
    const float cB = -cb * det_inv;
    const float cC = ca * det_inv;
    rec.opacity = po.w;

    // quad (gau_vert.glsl:225, 242-245) + viewport transform
    const float wh[2] = {(2.0f * u.hfov[0]) * u.hfov[2], (2.0f * u.hfov[1]) * u.hfov[2]};
    const float qs[2] = {3.0f * sqrtf(ca), 3.0f * sqrtf(cc)};
    const float half[2] = {(float)u.width * 0.5f, (float)u.height * 0.5f};
    float lo[2], hi[2], cw[2], sc[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float qn = qs[k] / wh[k] * 2.0f;
        const float off = qn * u.sdsf;
        lo[k] = (pr.ndc[k] + (-off)) * half[k] + half[k];
        hi[k] = (pr.ndc[k] + off) * half[k] + half[k];
        cw[k] = pr.ndc[k] * half[k] + half[k];
        sc[k] = qs[k] / ((hi[k] - lo[k]) * 0.5f);
    }
    rec.cx = cw[0];
    rec.cy = cw[1];
    rec.qa = (((-0.5f * kLog2e) * cA) * sc[0]) * sc[0];
    rec.qb = (((-kLog2e) * cB) * sc[0]) * sc[1];
    rec.qc = (((-0.5f * kLog2e) * cC) * sc[1]) * sc[1];
    int x0, x1, j0i, j1i;
    pixel_span(lo[0], hi[0], u.width, x0, x1);
    pixel_span(lo[1], hi[1], u.height, j0i, j1i);
    x0 = max(x0, 0);
    x1 = min(x1, u.width - 1);
    j0i = max(j0i, 0);
    j1i = min(j1i, u.height - 1);
    int r0 = (u.height - 1) - j1i, r1 = (u.height - 1) - j0i;
    const int mode = u.render_mod;
    const bool gauss = frag_class_of(mode) == kFragGauss;
    const float mid = gauss ? -0.5f * log2f(255.0f * po.w) : 0.f;
    if (gauss) alpha_box(rec.qa, rec.qb, rec.qc, 2.0f * mid, rec.cx, rec.cy, u.height, x0, x1, r0, r1);
    const bool nonempty = (x0 <= x1) && (r0 <= r1);
    rec.xspan = nonempty ? ((uint32_t)x0 | ((uint32_t)x1 << 16)) : 0xffffu;  // empty: x0 > x1
    rec.yspan = nonempty ? ((uint32_t)r0 | ((uint32_t)r1 << 16)) : 0xffffu;

    // colour varying
    V3 col;
    if (mode == -3) {  // depth (gau_vert.glsl:252-259)
        float d = -pr.pv[2];
        d = (d < 0.05f) ? 1.0f : d;
        d = 1.0f / d;
        col = V3{d, d, d};
    } else if (mode == -2 || mode == -1) {
        // -2: normal colour (gau_vert.glsl:265-272); -1: billboard normal
        // fragment colour = 0.5*(normalize(approxNormal)+1) (gau_frag.glsl:23-27)
        V3 nrm = normalize3(u.campos[0] - x, u.campos[1] - y, u.campos[2] - z);
        if (mode == -1) nrm = normalize3(nrm.x, nrm.y, nrm.z);
        col = V3{0.5f * (nrm.x + 1.0f), 0.5f * (nrm.y + 1.0f), 0.5f * (nrm.z + 1.0f)};
    } else {
        col = sh_color<DEG < 0 ? 0 : DEG>(g.f, x, y, z, u);
    }
    if (mode != -6) {  // unorm target clamps the fragment colour
        col.x = clamp01(col.x);
        col.y = clamp01(col.y);
        col.z = clamp01(col.z);
    }
    rec.r = col.x;
    rec.g = col.y;
    rec.b = col.z;
    rec.mid = u.plain_rec ? 0.f : mid;
    if (gauss && !u.plain_rec) {  // interval form (gsr_internal.h, SplatRec)
        rec.opacity = sqrtf(po.w / 255.0f) / 0.99f;
        rec.r = 0.99f * col.x;
        rec.g = 0.99f * col.y;
        rec.b = 0.99f * col.z;
    }

    const uint32_t slot = slot_base - (uint32_t)__popcll(m & lanemask_lt());
    float4* dst = reinterpret_cast<float4*>(recs + slot);
    dst[0] = make_float4(rec.cx, rec.cy, rec.opacity, __uint_as_float(rec.xspan));
    dst[1] = make_float4(rec.qa, rec.qb, rec.qc, __uint_as_float(rec.yspan));
    dst[2] = make_float4(rec.r, rec.g, rec.b, rec.mid);
    key = float_order_key(-pr.pv[2]);
    depth_keys[slot] = key;
    if (radii) {
        const float rr = ceilf(fmaxf(qs[0], qs[1]));
        radii[i] = (rr >= 0.f && rr < 2147483520.f) ? (int32_t)rr : 0;
    }
    uint32_t tiles = 0;
    uint2 tr = make_uint2(0xffffu, 0u);  // empty: tx0 > tx1
    if (nonempty) {
        const uint32_t tx0 = x0 >> 4, tx1 = x1 >> 4, ty0 = r0 >> 4, ty1 = r1 >> 4;
        tr = make_uint2(tx0 | (tx1 << 16), ty0 | (ty1 << 16));
        tiles = (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
    }
    trect[slot] = tr;
    return tiles;
}

#ifdef GSR_PRE_WPE
#define GSR_PRE_OCC __attribute__((amdgpu_waves_per_eu(GSR_PRE_WPE, 8)))
#else
#define GSR_PRE_OCC
#endif
template <int DEG>
__global__ __launch_bounds__(kThreads) GSR_PRE_OCC void k_preprocess(const float4* __restrict__ pos_op, const float4* __restrict__ rot,
                                                         const float4* __restrict__ scale, const float4* __restrict__ sh,
                                                         int64_t n, FrameUniforms u,
                                                         const uint64_t* __restrict__ vis_mask,
                                                         const uint32_t* __restrict__ wave_off,
                                                         const uint32_t* __restrict__ n_vis_dev,
                                                         SplatRec* __restrict__ recs, uint32_t* __restrict__ depth_keys,
                                                         uint2* __restrict__ trect, uint32_t* __restrict__ counters,
                                                         unsigned long long* __restrict__ done_ctr,
                                                         uint32_t* __restrict__ host_counters, uint32_t seq,
                                                         int32_t* __restrict__ radii) {
    __shared__ uint32_t s_cnt[kThreads / 64];
    uint32_t tiles = 0;
    // Grid-stride over blocks of kThreads Gaussians with a grid of ~4 blocks per
    // CU: the waves drift out of phase, so one wave's loads overlap another's
    // arithmetic.  (With one block per 256 Gaussians the resident waves ran in
    // lock-step rounds of load-then-compute: 67 -> 63.5 us at 1M.)
    for (int64_t i0 = (int64_t)blockIdx.x * kThreads; i0 < n; i0 += (int64_t)gridDim.x * kThreads) {
        const int64_t i = i0 + threadIdx.x;
        const uint64_t m = (i < n) ? vis_mask[i >> 6] : 0ull;
        const bool vis = (m >> __lane_id()) & 1ull;
        if (vis) tiles += preprocess_one<DEG>(pos_op, rot, scale, sh, n, u, m, i, wave_off, n_vis_dev, recs, depth_keys,
                                             trect, radii);
        else if (i < n && radii) radii[i] = 0;
    }
    // instance total for the frame (sizes the tile sort without waiting for it)
    const uint32_t ws = wave_reduce_sum(tiles);
    if (__lane_id() == 0) s_cnt[threadIdx.x >> 6] = ws;
    __syncthreads();
    if (threadIdx.x == 0) {
        // One 64-bit atomic carries both this block's instance count (low 40
        // bits) and its completion (high bits), so the block whose add
        // completes the grid holds the frame's total without any fence.  It
        // publishes (V, D) to the device counters and, with the frame's
        // sequence number last, to host-mapped memory (the host sizes the
        // tile sort from them while the GPU runs the depth sort), and re-arms
        // the counter for the next frame.
        const uint32_t b = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        const unsigned long long old = atomicAdd(done_ctr, (1ull << 40) | (unsigned long long)b);
        if ((old >> 40) == (unsigned long long)(gridDim.x - 1)) {
            const unsigned long long d64 = (old & ((1ull << 40) - 1)) + b;
            const uint32_t n_dup = (uint32_t)d64;
            const uint32_t n_vis = n_vis_dev[0];
            counters[1] = n_dup;
            __hip_atomic_store(host_counters + 0, n_vis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_counters + 1, n_dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_counters + 3, (uint32_t)(d64 >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_counters + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(done_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}


// Several views of one scene (gsr_render_begin_views): each Gaussian's scene
// data is loaded once and run through the vertex stage of every view it is
// visible in.  Per view, the same outputs, slots and publication protocol as
// k_preprocess.
struct ViewPre {
    FrameUniforms u;
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
struct ViewsPre {
    ViewPre v[kMaxViews];
    int32_t k;
};
static_assert(sizeof(ViewsPre) <= 3584, "kernel argument size");

template <int DEG>
__global__ __launch_bounds__(kThreads) GSR_PRE_OCC void k_preprocess_views(const float4* __restrict__ pos_op,
                                                                           const float4* __restrict__ rot,
                                                                           const float4* __restrict__ scale,
                                                                           const float4* __restrict__ sh, int64_t n,
                                                                           ViewsPre vs) {
    __shared__ uint32_t s_cnt[kMaxViews][kThreads / 64];
    const int wave = threadIdx.x >> 6;
    const int lane = __lane_id();
    if (threadIdx.x < kMaxViews * (kThreads / 64)) s_cnt[threadIdx.x / (kThreads / 64)][threadIdx.x % (kThreads / 64)] = 0u;
    __syncthreads();
    for (int64_t i0 = (int64_t)blockIdx.x * kThreads; i0 < n; i0 += (int64_t)gridDim.x * kThreads) {
        const int64_t i = i0 + threadIdx.x;
        bool any = false;
        for (int v = 0; v < vs.k; ++v) any |= i < n && ((vs.v[v].vis_mask[i >> 6] >> lane) & 1ull);
        GaussLoad<DEG> g;
        Cov3 S3;
        if (any) {
            load_gaussian<DEG>(g, pos_op, rot, scale, sh, n, i);
            S3 = cov3d(g.q1, g.sc4, vs.v[0].u);  // (the group shares rot_modifier and the scale factor)
        }
#pragma unroll 1
        for (int v = 0; v < vs.k; ++v) {
            const ViewPre& V = vs.v[v];
            const uint64_t m = i < n ? V.vis_mask[i >> 6] : 0ull;
            uint32_t tiles = 0;
            if ((m >> lane) & 1ull) {
                const uint32_t slot_base = V.n_vis_dev[0] - 1u - V.wave_off[i >> 6];
                uint32_t key;
                tiles = preprocess_compute<DEG>(g, S3, V.u, m, i, slot_base, V.recs, V.depth_keys, V.trect, V.radii,
                                                key);
            } else if (i < n && V.radii) {
                V.radii[i] = 0;
            }
            const uint32_t ws = wave_reduce_sum(tiles);
            if (lane == 0) s_cnt[v][wave] += ws;
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)vs.k) {  // one thread per view: k_preprocess's completion protocol
        const ViewPre& V = vs.v[threadIdx.x];
        const uint32_t b = s_cnt[threadIdx.x][0] + s_cnt[threadIdx.x][1] + s_cnt[threadIdx.x][2] + s_cnt[threadIdx.x][3];
        const unsigned long long old = atomicAdd(V.done_ctr, (1ull << 40) | (unsigned long long)b);
        if ((old >> 40) == (unsigned long long)(gridDim.x - 1)) {
            const unsigned long long d64 = (old & ((1ull << 40) - 1)) + b;
            const uint32_t n_dup = (uint32_t)d64;
            const uint32_t n_vis = V.n_vis_dev[0];
            V.counters[1] = n_dup;
            __hip_atomic_store(V.host_counters + 0, n_vis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(V.host_counters + 1, n_dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(V.host_counters + 3, (uint32_t)(d64 >> 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(V.host_counters + 2, V.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(V.done_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------ culling fused in
// The frame in one launch, without k_cull and the scan (GSR_FUSED_CULL): each
// lane projects its Gaussian itself and loads the rest of the scene data only
// when it is visible.  Slots are not compacted: Gaussian i owns slot n-1-i in
// recs / depth_keys / trect (the same descending-index order as the compacted
// slots, so the stable depth sort still resolves ties front to back), and a
// culled slot holds the key 0xffffffff and an empty rectangle; the depth
// sort's first pass runs over all n slots and drops every key outside the
// frame's key range (PassArgs::drop), later passes see only the V visible.
// Per frame, beside the completion word done_ctr[0] (blocks << 40 | D), in
// 64 shards (block b updates shard b mod 64: at most 16 blocks per address
// instead of the whole grid; a single word under 1024 blocks' atomics cost
// ~9 us of the frame):
//   done_ctr[kKeyShards0 + s]         (seq << 32) | kmax
//   done_ctr[kKeyShards0 + 64 + s]    (seq << 32) | ~kmin
//   done_ctr[kKeyShards0 + 128 + s]   the shard's visible count
// The key shards are tagged with the frame's sequence number, so they never
// need clearing: a frame's first max replaces any older frame's entry.  The
// block completing the grid reduces all of them with one wave, publishes as
// before, and zeroes the count shards and the completion word.  (Completion
// counted in two levels, per shard then per grid, measured no faster.)
constexpr int kKeyShards = 64;
constexpr int kKeyShards0 = 1;

// The rest of Gaussian i's data (its position is already loaded).
template <int DEG, bool kNT>
__device__ __forceinline__ void load_attrs(GaussLoad<DEG>& g, const float4 po, const float4* __restrict__ rot,
                                           const float4* __restrict__ scale, const float4* __restrict__ sh, int64_t n,
                                           int64_t i) {
    g.po = po;
    g.q1 = load_stream<kNT>(rot, i);
    g.sc4 = load_stream<kNT>(scale, i);
#pragma unroll
    for (int p = 0; p < 12; ++p) {
        if (p < sh_planes_for<DEG>()) {
            const float4 t = load_plane<kNT>(sh, n, p, i);
            g.f[4 * p + 0] = t.x;
            g.f[4 * p + 1] = t.y;
            g.f[4 * p + 2] = t.z;
            g.f[4 * p + 3] = t.w;
        } else {
            g.f[4 * p + 0] = g.f[4 * p + 1] = g.f[4 * p + 2] = g.f[4 * p + 3] = 0.f;
        }
    }
}

__device__ __forceinline__ void culled_slot(uint32_t slot, uint32_t* __restrict__ depth_keys,
                                            uint2* __restrict__ trect) {
    depth_keys[slot] = 0xffffffffu;
    trect[slot] = make_uint2(0xffffu, 0u);
}

// One frame's block results: counts and the key range of its visible
// Gaussians.  Thread 0 only; returns true in the block that completed the grid.
__device__ __forceinline__ bool block_done(unsigned long long* __restrict__ done_ctr, uint32_t seq, uint32_t tiles,
                                           uint32_t nvis, uint32_t kmax, uint32_t nkmin, unsigned long long& n_dup) {
    if (nvis) {
        const int sh = kKeyShards0 + (int)(blockIdx.x % kKeyShards);
        const unsigned long long tag = (unsigned long long)seq << 32;
        const unsigned long long r0 =
            __hip_atomic_fetch_max(done_ctr + sh, tag | kmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long r1 =
            __hip_atomic_fetch_max(done_ctr + sh + kKeyShards, tag | nkmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long r2 = __hip_atomic_fetch_add(done_ctr + sh + 2 * kKeyShards, (unsigned long long)nvis,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // Returned (so performed at the coherence point, where device-scope
        // atomics act) before the completion add below is issued: the block
        // that completes the grid sees every block's contributions, with no
        // cache write-back.  (The asm consumes the results: the atomics stay
        // the returning kind, and the compiler waits for them here.)
        asm volatile("" ::"v"(r0), "v"(r1), "v"(r2) : "memory");
    }
    const unsigned long long old = atomicAdd(done_ctr, (1ull << 40) | (unsigned long long)tiles);
    n_dup = (old & ((1ull << 40) - 1)) + tiles;
    return (old >> 40) == (unsigned long long)(gridDim.x - 1);
}

// The completing block's publication, by one whole wave: the frame's key
// range from the shards, V and D to the device counters and (V, D, seq) to
// host-mapped memory; the counters are re-armed for the next frame.
__device__ __forceinline__ void publish_frame(unsigned long long* __restrict__ done_ctr, uint32_t seq,
                                              unsigned long long n_dup64,
                                              uint32_t* __restrict__ key_range, uint32_t* __restrict__ counters,
                                              uint32_t* __restrict__ host_counters) {
    const int lane = __lane_id();
    const unsigned long long a =
        __hip_atomic_load(done_ctr + kKeyShards0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b =
        __hip_atomic_load(done_ctr + kKeyShards0 + kKeyShards + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long c =
        __hip_atomic_load(done_ctr + kKeyShards0 + 2 * kKeyShards + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t kmax = wave_reduce_max((uint32_t)(a >> 32) == seq ? (uint32_t)a : 0u);
    const uint32_t nkmin = wave_reduce_max((uint32_t)(b >> 32) == seq ? (uint32_t)b : 0u);
    const uint32_t n_vis = wave_reduce_sum((uint32_t)c);
    __hip_atomic_store(done_ctr + kKeyShards0 + 2 * kKeyShards + lane, 0ull, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
        key_range[0] = nkmin;  // {0, 0} when nothing is visible, like the scan's
        key_range[1] = kmax;
        const uint32_t n_dup = (uint32_t)n_dup64;
        counters[0] = n_vis;
        counters[1] = n_dup;
        __hip_atomic_store(host_counters + 0, n_vis, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_counters + 1, n_dup, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // instances beyond 32 bits: the host refuses the frame (GSR_ERR_OVERFLOW)
        __hip_atomic_store(host_counters + 3, (uint32_t)(n_dup64 >> 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_counters + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(done_ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One launch for the views of a group (k = 1: a frame alone): a position is
// projected for every view and the rest of the Gaussian loaded once when any
// view sees it.  (A separate one-view kernel with the uniforms as a plain
// kernel argument needed 164 VGPRs at DEG 3 against 119 here: the compiler
// hoisted every uniform out of the grid-stride loop and, out of SGPRs, kept
// them in VGPRs; indexed by the runtime view they are re-read each iteration.)
struct ViewPreFc {
    FrameUniforms u;
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
struct ViewsPreFc {
    ViewPreFc v[kMaxViews];
    int32_t k;
};
static_assert(sizeof(ViewsPreFc) <= 3584, "kernel argument size");

// kAlone: the same code, instantiated separately for the launches of a frame
// alone (k = 1) so that profiles tell them from the groups' launches.
template <int DEG, bool kAlone>
__global__ __launch_bounds__(kThreads) GSR_PRE_OCC void k_preprocess_fc_views(const float4* __restrict__ pos_op,
                                                                              const float4* __restrict__ rot,
                                                                              const float4* __restrict__ scale,
                                                                              const float4* __restrict__ sh,
                                                                              int64_t n, ViewsPreFc vs) {
    static_assert(kMaxViews * 4 * (kThreads / 64) <= kThreads, "one thread per LDS word");
    __shared__ uint32_t s_red[kMaxViews][4][kThreads / 64];
    __shared__ uint32_t s_last[kMaxViews];
    __shared__ unsigned long long s_dup[kMaxViews];
    const int wave = threadIdx.x >> 6;
    const int lane = __lane_id();
    for (int v = 0; v < vs.k; ++v) clear_words(vs.v[v].zero_words, vs.v[v].n_zero);
    if (threadIdx.x < kMaxViews * 4 * (kThreads / 64)) (&s_red[0][0][0])[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    const int64_t first = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    float4 pnext = first < n ? pos_op[first] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = first; i - threadIdx.x < n; i += stride) {
        const float4 p = pnext;
        pnext = i + stride < n ? pos_op[i + stride] : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool in = i < n;
        uint32_t vm = 0;  // the views that see Gaussian i
#pragma unroll 1
        for (int v = 0; v < vs.k; ++v)
            if (in && project(p.x, p.y, p.z, vs.v[v].u).vis) vm |= 1u << v;
        GaussLoad<DEG> g;
        Cov3 S3;
        if (vm) {
            load_attrs<DEG, kAlone>(g, p, rot, scale, sh, n, i);
            S3 = cov3d(g.q1, g.sc4, vs.v[0].u);  // (the group shares rot_modifier and the scale factor)
        }
        const uint32_t slot = (uint32_t)(n - 1 - i);
#pragma unroll 1
        for (int v = 0; v < vs.k; ++v) {
            const ViewPreFc& V = vs.v[v];
            uint32_t tiles = 0, key = 0;
            const bool vis = (vm >> v) & 1u;
            if (vis) {
                tiles =
                    preprocess_compute<DEG>(g, S3, V.u, 0ull, i, slot, V.recs, V.depth_keys, V.trect, V.radii, key);
            } else if (in) {
                culled_slot(slot, V.depth_keys, V.trect);
                if (V.radii) V.radii[i] = 0;
            }
            const uint32_t a = wave_reduce_sum(tiles);
            const uint32_t b = (uint32_t)__popcll(__ballot(vis));
            const uint32_t c = wave_reduce_max(vis ? key : 0u), d = wave_reduce_max(vis ? ~key : 0u);
            if (lane == 0) {
                s_red[v][0][wave] += a;
                s_red[v][1][wave] += b;
                s_red[v][2][wave] = max(s_red[v][2][wave], c);
                s_red[v][3][wave] = max(s_red[v][3][wave], d);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)vs.k) {  // one thread per view: the block's results
        const int v = threadIdx.x;
        uint32_t t = 0, nv = 0, kx = 0, kn = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; ++w)
            t += s_red[v][0][w], nv += s_red[v][1][w], kx = max(kx, s_red[v][2][w]), kn = max(kn, s_red[v][3][w]);
        unsigned long long n_dup;
        s_last[v] = block_done(vs.v[v].done_ctr, vs.v[v].seq, t, nv, kx, kn, n_dup) ? 1u : 0u;
        s_dup[v] = n_dup;
    }
    __syncthreads();
    for (int v = wave; v < vs.k; v += kThreads / 64)
        if (s_last[v])
            publish_frame(vs.v[v].done_ctr, vs.v[v].seq, s_dup[v], vs.v[v].key_range, vs.v[v].counters,
                          vs.v[v].host_counters);
}

__global__ __launch_bounds__(kThreads) void k_depth_keys_all(const float4* __restrict__ pos_op, int64_t n, float v8,
                                                             float v9, float v10, float v11, uint32_t* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = pos_op[i];
    keys[i] = float_order_key(((v8 * p.x + v9 * p.y) + v10 * p.z) + v11);
}

}  // namespace

// Grid-stride blocks: ~4 resident blocks per CU (92 VGPRs: 5 waves/SIMD fit)
// for a group's views; 3 for a frame alone (fused kernel with k = 1), whose
// preprocess measured 68.3 -> 66.1 us with 3 (2: 66.7, 16 = one thread per
// Gaussian: 82.4; a group's kernel was no faster with 3 or 2, profiles/r4_s27).
static unsigned preprocess_grid(int64_t n, bool alone = false) {
    static const int cus = [] {
        int dev = 0, c = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    // (measured: profiles/r4_s8, r4_s27; 6 or 12 per CU for C3's 6M alone: no change, r5_s28; with the
    // non-temporal scene reads 2 / 4 / 6 alone: preprocess 62.4 / 62.4 / 66 us against 60.5 for 3, r5_s53)
#ifndef GSR_PRE_PER_CU_ALONE  // build knob for A/B
#define GSR_PRE_PER_CU_ALONE 3
#endif
    const unsigned per_cu = alone ? (unsigned)GSR_PRE_PER_CU_ALONE : 4u;
    return std::max(1u, std::min((unsigned)((n + kThreads - 1) / kThreads), per_cu * (unsigned)cus));
}

static int effective_deg(const FrameUniforms& u) {
    // effective SH degree: the gates of gau_vert.glsl:289-313; -1 = colour not from SH
    const int m = u.render_mod;
    int deg = (u.sh_dim > 27 && m >= 3) ? 3 : (u.sh_dim > 12 && m >= 2) ? 2 : (u.sh_dim > 3 && m >= 1) ? 1 : 0;
    if (m == -3 || m == -2 || m == -1) deg = -1;
    return deg;
}

int launch_cull(const SceneData& sd, const FrameUniforms& u, uint64_t* vis_mask, uint32_t* wave_counts,
                uint2* block_ranges, uint32_t* zero_words, uint32_t n_zero, hipStream_t s) {
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_cull<<<grid, kThreads, 0, s>>>(sd.pos_op, sd.n, u, vis_mask, wave_counts, block_ranges, zero_words, n_zero);
    GSR_LAUNCH_CHECK("cull");
    return GSR_OK;
}

int launch_preprocess(const SceneData& sd, const FrameUniforms& u, const uint64_t* vis_mask,
                      const uint32_t* wave_off, const uint32_t* n_vis_dev, SplatRec* recs, uint32_t* depth_keys,
                      uint2* trect, uint32_t* counters, unsigned long long* done_ctr, uint32_t* host_counters,
                      uint32_t seq, int32_t* radii, hipStream_t s) {
    const unsigned grid = preprocess_grid(sd.n);
    const int deg = effective_deg(u);
#define GSR_PRE(D)                                                                                                  \
    k_preprocess<D><<<grid, kThreads, 0, s>>>(sd.pos_op, sd.rot, sd.scale, sd.sh, sd.n, u, vis_mask, wave_off,    \
                                              n_vis_dev, recs, depth_keys, trect, counters, done_ctr,            \
                                              host_counters, seq, radii)
    switch (deg) {
        case -1: GSR_PRE(-1); break;
        case 0: GSR_PRE(0); break;
        case 1: GSR_PRE(1); break;
        case 2: GSR_PRE(2); break;
        default: GSR_PRE(3); break;
    }
#undef GSR_PRE
    GSR_LAUNCH_CHECK("preprocess");
    return GSR_OK;
}

int launch_cull_views(const SceneData& sd, const ViewCullArgs* views, int k, hipStream_t s) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "cull_views: view count out of range");
    ViewsCull vc{};
    vc.k = k;
    for (int v = 0; v < k; ++v) {
        const ViewCullArgs& a = views[v];
        vc.v[v] = ViewCull{*a.u, a.vis_mask, a.wave_counts, a.block_ranges, a.zero_words, a.n_zero};
    }
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_cull_views<<<grid, kThreads, 0, s>>>(sd.pos_op, sd.n, vc);
    GSR_LAUNCH_CHECK("cull_views");
    return GSR_OK;
}

int launch_preprocess_views(const SceneData& sd, const ViewPreArgs* views, int k, hipStream_t s) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "preprocess_views: view count out of range");
    ViewsPre vp{};
    vp.k = k;
    const int deg = effective_deg(*views[0].u);
    for (int v = 0; v < k; ++v) {
        const ViewPreArgs& a = views[v];
        if (effective_deg(*a.u) != deg) return set_error(GSR_ERR_INVALID, "preprocess_views: views differ in SH degree");
        vp.v[v] = ViewPre{*a.u, a.vis_mask, a.wave_off, a.n_vis_dev, a.recs, a.depth_keys, a.trect,
                          a.counters, a.done_ctr, a.host_counters, a.radii, a.seq};
    }
    const unsigned grid = preprocess_grid(sd.n);
#define GSR_PREV(D) k_preprocess_views<D><<<grid, kThreads, 0, s>>>(sd.pos_op, sd.rot, sd.scale, sd.sh, sd.n, vp)
    switch (deg) {
        case -1: GSR_PREV(-1); break;
        case 0: GSR_PREV(0); break;
        case 1: GSR_PREV(1); break;
        case 2: GSR_PREV(2); break;
        default: GSR_PREV(3); break;
    }
#undef GSR_PREV
    GSR_LAUNCH_CHECK("preprocess_views");
    return GSR_OK;
}

static_assert(kDoneCtrWords >= (size_t)(kKeyShards0 + 3 * kKeyShards), "completion words");

int launch_preprocess_fc(const SceneData& sd, const FrameUniforms& u, SplatRec* recs, uint32_t* depth_keys,
                         uint2* trect, uint32_t* counters, uint32_t* key_range, uint32_t* zero_words, uint32_t n_zero,
                         unsigned long long* done_ctr, uint32_t* host_counters, uint32_t seq, int32_t* radii,
                         hipStream_t s) {
    const ViewPreFcArgs a{&u, recs, depth_keys, trect, counters, key_range, zero_words, done_ctr, host_counters, radii,
                          n_zero, seq};
    return launch_preprocess_fc_views(sd, &a, 1, s);
}

int launch_preprocess_fc_views(const SceneData& sd, const ViewPreFcArgs* views, int k, hipStream_t s) {
    if (k < 1 || k > kMaxViews) return set_error(GSR_ERR_INVALID, "preprocess_views: view count out of range");
    if ((uint64_t)sd.n > 0xffffffffull) return set_error(GSR_ERR_OVERFLOW, "preprocess: too many Gaussians");
    ViewsPreFc vp{};
    vp.k = k;
    const int deg = effective_deg(*views[0].u);
    for (int v = 0; v < k; ++v) {
        const ViewPreFcArgs& a = views[v];
        if (effective_deg(*a.u) != deg) return set_error(GSR_ERR_INVALID, "preprocess_views: views differ in SH degree");
        vp.v[v] = ViewPreFc{*a.u,         a.recs,      a.depth_keys, a.trect,         a.counters, a.key_range,
                            a.zero_words, a.done_ctr,  a.host_counters, a.radii,      a.n_zero,   a.seq};
    }
    const unsigned grid = preprocess_grid(sd.n, k == 1);
#define GSR_PREV(D)                                                                                             \
    (k == 1 ? k_preprocess_fc_views<D, true> : k_preprocess_fc_views<D, false>)<<<grid, kThreads, 0, s>>>(        \
        sd.pos_op, sd.rot, sd.scale, sd.sh, sd.n, vp)
    switch (deg) {
        case -1: GSR_PREV(-1); break;
        case 0: GSR_PREV(0); break;
        case 1: GSR_PREV(1); break;
        case 2: GSR_PREV(2); break;
        default: GSR_PREV(3); break;
    }
#undef GSR_PREV
    GSR_LAUNCH_CHECK("preprocess_fc_views");
    return GSR_OK;
}

int launch_depth_keys_all(const SceneData& sd, const float* V, uint32_t* keys, hipStream_t s) {
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_depth_keys_all<<<grid, kThreads, 0, s>>>(sd.pos_op, sd.n, V[8], V[9], V[10], V[11], keys);
    GSR_LAUNCH_CHECK("depth_keys_all");
    return GSR_OK;
}

}  // namespace gsr

// Scene creation: one-time repack of the GaussianData arrays into SoA float4
// planes so that every per-frame load is a coalesced 16-B-per-lane access.
//
// Input layouts (reference):
//   fields: xyz[n,3], rot[n,4], scale[n,3], opacity[n,1], sh[n,sh_dim]
//           (util_gau.py:10-42; GaussianDataCUDA renderer_cuda.py:60-101)
//   flat  : [n, 11+sh_dim] = [xyz, rot, scale, opacity, sh]  (util_gau.py:40-42,
//           SSBO layout gau_vert.glsl:28-42)
// HBM layout (this library): pos_op[n] (x,y,z,opacity), rot[n] (w,x,y,z),
//   scale[n] (sx,sy,sz,0), sh plane p = floats [4p, 4p+4) of each Gaussian's
//   SH vector at sh + p*n (zero padded).
#include "gsr_internal.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void k_repack_fields(const float* __restrict__ xyz, const float* __restrict__ rot,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ opacity,
                                                            const float* __restrict__ sh, int64_t n, int sh_dim,
                                                            int planes, float4* __restrict__ pos_op,
                                                            float4* __restrict__ rot_o, float4* __restrict__ scale_o,
                                                            float4* __restrict__ sh_o) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    pos_op[i] = make_float4(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], opacity[i]);
    rot_o[i] = make_float4(rot[4 * i], rot[4 * i + 1], rot[4 * i + 2], rot[4 * i + 3]);
    scale_o[i] = make_float4(scale[3 * i], scale[3 * i + 1], scale[3 * i + 2], 0.f);
    const float* s = sh + (int64_t)sh_dim * i;
    for (int p = 0; p < planes; ++p) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (4 * p + k < sh_dim) ? s[4 * p + k] : 0.f;
        sh_o[(int64_t)p * n + i] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

__global__ __launch_bounds__(kThreads) void k_repack_flat(const float* __restrict__ flat, int64_t n, int sh_dim,
                                                          int planes, float4* __restrict__ pos_op,
                                                          float4* __restrict__ rot_o, float4* __restrict__ scale_o,
                                                          float4* __restrict__ sh_o) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float* f = flat + (int64_t)(11 + sh_dim) * i;
    pos_op[i] = make_float4(f[0], f[1], f[2], f[10]);
    rot_o[i] = make_float4(f[3], f[4], f[5], f[6]);
    scale_o[i] = make_float4(f[7], f[8], f[9], 0.f);
    const float* s = f + 11;
    for (int p = 0; p < planes; ++p) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (4 * p + k < sh_dim) ? s[4 * p + k] : 0.f;
        sh_o[(int64_t)p * n + i] = make_float4(v[0], v[1], v[2], v[3]);
    }
}


// ---- PLY load on the device (gsr_scene_load_ply): activations and
// scale_data on the raw rows the parser streamed into a flat [n, 11 + sh_dim]
// array, in the reference's float32 evaluation order, unfused.
//   load_ply (util_gau.py:297-303): rot / ||rot|| (((r0^2 + r1^2) + r2^2) + r3^2,
//     NumPy's order for a 4-wide row), exp(scale), 1 / (1 + exp(-opacity));
//   scale_data (util_gau.py:44-53): centre = (min + max) / 2, factor =
//     interval / max(max - min), xyz = (xyz - centre) * factor, rot
//     renormalised, scale *= factor.
// No contraction (#pragma clang fp contract(off) on plain operators; the
// __f*_rn intrinsics' own bodies may still be fused).  min /
// max are exact (order-preserving integer keys).  exp is the device's
// (within 1 ulp of exact); NumPy's float32 exp is a SIMD polynomial within
// ~2.5 ulp, so scale and opacity can differ from load_ply by a few ulps.
__device__ __forceinline__ void normalize_rot(float* r) {
#pragma clang fp contract(off)  // (operators, not __f*_rn: those intrinsics' bodies allow fusing)
    const float s = ((r[0] * r[0] + r[1] * r[1]) + r[2] * r[2]) + r[3] * r[3];
    const float nrm = sqrtf(s);
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = r[k] / nrm;
}

__device__ __forceinline__ uint32_t ord_key(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ float from_ord_key(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// keys[0..2] = ~min key, keys[3..5] = max key (both reduced with atomicMax; zero-initialised)
__global__ __launch_bounds__(kThreads) void k_ply_activate(float* __restrict__ flat, int64_t n, int rec,
                                                           uint32_t* __restrict__ keys) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    uint32_t lo[3] = {0u, 0u, 0u}, hi[3] = {0u, 0u, 0u};
    if (i < n) {
        float* f = flat + (int64_t)rec * i;
        float r[4] = {f[3], f[4], f[5], f[6]};
        normalize_rot(r);
#pragma unroll
        for (int k = 0; k < 4; ++k) f[3 + k] = r[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) f[7 + k] = expf(f[7 + k]);
        f[10] = 1.0f / (1.0f + expf(-f[10]));
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint32_t key = ord_key(f[k]);
            lo[k] = ~key;
            hi[k] = key;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = max(lo[k], (uint32_t)__shfl_xor((int)lo[k], o, 64));
            hi[k] = max(hi[k], (uint32_t)__shfl_xor((int)hi[k], o, 64));
        }
    }
    if (__lane_id() == 0 && keys) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            atomicMax(keys + k, lo[k]);
            atomicMax(keys + 3 + k, hi[k]);
        }
    }
}

// out[0..2] = centre, out[3] = factor (written by thread 0 of block 0)
__global__ __launch_bounds__(kThreads) void k_ply_scale_data(float* __restrict__ flat, int64_t n, int rec,
                                                             const uint32_t* __restrict__ keys, float interval,
                                                             float* __restrict__ out) {
#pragma clang fp contract(off)
    float c[3], mn[3], mx[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        mn[k] = from_ord_key(~keys[k]);
        mx[k] = from_ord_key(keys[3 + k]);
        c[k] = (mn[k] + mx[k]) / 2.0f;
    }
    const float ext = fmaxf(fmaxf(mx[0] - mn[0], mx[1] - mn[1]), mx[2] - mn[2]);
    const float factor = interval / ext;
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i == 0 && out) {
        out[0] = c[0], out[1] = c[1], out[2] = c[2], out[3] = factor;
    }
    if (i >= n) return;
    float* f = flat + (int64_t)rec * i;
#pragma unroll
    for (int k = 0; k < 3; ++k) f[k] = (f[k] - c[k]) * factor;
    float r[4] = {f[3], f[4], f[5], f[6]};
    normalize_rot(r);
#pragma unroll
    for (int k = 0; k < 4; ++k) f[3 + k] = r[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) f[7 + k] = f[7 + k] * factor;
}

__global__ __launch_bounds__(kThreads) void k_flat_xyz(const float* __restrict__ flat, int64_t n, int rec,
                                                       float* __restrict__ xyz) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float* f = flat + (int64_t)rec * i;
    xyz[3 * i] = f[0];
    xyz[3 * i + 1] = f[1];
    xyz[3 * i + 2] = f[2];
}

// The scene's SoA planes back to the flat layout (gsr_scene_read_flat).
__global__ __launch_bounds__(kThreads) void k_unpack_flat(const float4* __restrict__ pos_op,
                                                          const float4* __restrict__ rot, const float4* __restrict__ scale,
                                                          const float4* __restrict__ sh, int64_t n, int sh_dim,
                                                          float* __restrict__ flat) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    float* f = flat + (int64_t)(11 + sh_dim) * i;
    const float4 p = pos_op[i], r = rot[i], s = scale[i];
    f[0] = p.x, f[1] = p.y, f[2] = p.z, f[10] = p.w;
    f[3] = r.x, f[4] = r.y, f[5] = r.z, f[6] = r.w;
    f[7] = s.x, f[8] = s.y, f[9] = s.z;
    for (int k = 0; k < sh_dim; ++k) {
        const float4 q = sh[(int64_t)(k >> 2) * n + i];
        f[11 + k] = (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
    }
}

int alloc_scene(SceneData& sd) {
    const size_t n = (size_t)sd.n;
    const size_t bytes = n * sizeof(float4) * (3 + (size_t)sd.sh_planes);
    void* p = nullptr;
    if (hipMalloc(&p, bytes < 16 ? 16 : bytes) != hipSuccess)
        return set_error(GSR_ERR_NOMEM, "scene: hipMalloc of " + std::to_string(bytes) + " bytes failed");
    sd.block = p;
    float4* b = static_cast<float4*>(p);
    sd.pos_op = b;
    sd.rot = b + n;
    sd.scale = b + 2 * n;
    sd.sh = b + 3 * n;
    return GSR_OK;
}

}  // namespace

int scene_repack_from_fields(SceneData& sd, const float* xyz, const float* rot, const float* scale,
                             const float* opacity, const float* sh, hipStream_t s) {
    int rc = alloc_scene(sd);
    if (rc) return rc;
    if (sd.n == 0) return GSR_OK;
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_repack_fields<<<grid, kThreads, 0, s>>>(xyz, rot, scale, opacity, sh, sd.n, sd.sh_dim, sd.sh_planes,
                                              sd.pos_op, sd.rot, sd.scale, sd.sh);
    GSR_LAUNCH_CHECK("repack_fields");
    return GSR_OK;
}

int ply_activate_flat(float* flat, int64_t n, int sh_dim, float interval, uint32_t* keys, float* out4, float* xyz,
                      hipStream_t s) {
    if (n == 0) return GSR_OK;
    const unsigned grid = (unsigned)((n + kThreads - 1) / kThreads);
    const int rec = 11 + sh_dim;
    const bool rescale = interval > 0.f;
    if (rescale) GSR_HIP_CHECK(hipMemsetAsync(keys, 0, 6 * sizeof(uint32_t), s));
    k_ply_activate<<<grid, kThreads, 0, s>>>(flat, n, rec, rescale ? keys : nullptr);
    GSR_LAUNCH_CHECK("ply_activate");
    if (rescale) {
        k_ply_scale_data<<<grid, kThreads, 0, s>>>(flat, n, rec, keys, interval, out4);
        GSR_LAUNCH_CHECK("ply_scale_data");
    }
    k_flat_xyz<<<grid, kThreads, 0, s>>>(flat, n, rec, xyz);
    GSR_LAUNCH_CHECK("flat_xyz");
    return GSR_OK;
}

int scene_unpack_flat(const SceneData& sd, float* flat, hipStream_t s) {
    if (sd.n == 0) return GSR_OK;
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_unpack_flat<<<grid, kThreads, 0, s>>>(sd.pos_op, sd.rot, sd.scale, sd.sh, sd.n, sd.sh_dim, flat);
    GSR_LAUNCH_CHECK("unpack_flat");
    return GSR_OK;
}

int scene_repack_from_flat(SceneData& sd, const float* flat, hipStream_t s) {
    int rc = alloc_scene(sd);
    if (rc) return rc;
    if (sd.n == 0) return GSR_OK;
    const unsigned grid = (unsigned)((sd.n + kThreads - 1) / kThreads);
    k_repack_flat<<<grid, kThreads, 0, s>>>(flat, sd.n, sd.sh_dim, sd.sh_planes, sd.pos_op, sd.rot, sd.scale,
                                            sd.sh);
    GSR_LAUNCH_CHECK("repack_flat");
    return GSR_OK;
}

}  // namespace gsr

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

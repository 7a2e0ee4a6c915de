// GPU box mask, bounding box and row compaction for export (include/gsr_io.h;
// SURVEY.md §8(f) row 3).  Restates util_gau.export_ply's filter
// (util_gau.py:389-413) and gsconverter's crop_by_bbox
// (tools/gsconverter/utils/base_converter.py:175-184):
//
//   k_center_seq   points_center = np.mean(xyz, axis=0).  For a C-contiguous
//                  float32 [n,3] array NumPy sums row after row in float32 and
//                  divides in float32.  One wave reproduces that order
//                  exactly: chunks of rows are staged through LDS (the next
//                  chunk is prefetched in registers), and lanes 0..2 each add
//                  their column sequentially.
//   k_box_mask     the export_ply predicate on xyz - center in float64
//                  (NumPy promotes against the float64 thresholds).  Masked
//                  points are counted, and min/max of the as-loaded xyz are
//                  reduced through order-preserving integer keys (exact).
//   k_crop_flag / scan / k_crop_write
//                  rows of the as-loaded xyz inside the box (inclusive), kept
//                  in ascending order: a stable compaction through the
//                  exclusive scan.
#include "gsr_internal.h"
#include "gsr_io.h"

namespace gsr {
namespace {

constexpr int kThreads = 256;
constexpr int kSeqChunk = 256;  // rows staged per step of the sequential mean

__global__ __launch_bounds__(64) void k_center_seq(const float* __restrict__ xyz, int64_t n, float* __restrict__ center) {
    __shared__ float rows[kSeqChunk * 3];
    const int lane = threadIdx.x;
    constexpr int kPer = kSeqChunk * 3 / 64;  // floats per lane per chunk
    float pre[kPer];
    auto fetch = [&](int64_t r0) {
        const int64_t base = r0 * 3;
        const int64_t lim = n * 3;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int64_t i = base + k * 64 + lane;
            pre[k] = i < lim ? xyz[i] : 0.f;
        }
    };
    fetch(0);
    float s = 0.f;  // lane c < 3: running float32 sum of column c
    for (int64_t r0 = 0; r0 < n; r0 += kSeqChunk) {
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < kPer; ++k) rows[k * 64 + lane] = pre[k];
        __builtin_amdgcn_wave_barrier();
        if (r0 + kSeqChunk < n) fetch(r0 + kSeqChunk);
        const int m = (int)min<int64_t>(kSeqChunk, n - r0);
        if (lane < 3)
            for (int r = 0; r < m; ++r) s = __fadd_rn(s, rows[r * 3 + lane]);
    }
    if (lane < 3) center[lane] = __fdiv_rn(s, (float)n);
}

__device__ __forceinline__ uint32_t ord_key(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

inline float from_ord_key(uint32_t k) {  // host side
    const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    float f;
    __builtin_memcpy(&f, &b, 4);
    return f;
}

struct BoxArgs {
    int mode;
    double lo[3], hi[3];  // AABB: center + cube_min/max; OBB: cube_min/max
    double m[9];          // OBB: row-major inverse rotation
    float c[3];           // points_center
};

// stats: [0] count, [1..3] min keys, [4..6] max keys
__global__ __launch_bounds__(kThreads) void k_box_mask(const float* __restrict__ cur, const float* __restrict__ orig,
                                                       int64_t n, BoxArgs a, uint32_t* __restrict__ stats) {
    __shared__ uint32_t red[7][kThreads / 64];
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    bool in = false;
    float o[3] = {0.f, 0.f, 0.f};
    if (i < n) {
        double t[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) t[k] = (double)__fsub_rn(cur[i * 3 + k], a.c[k]);  // float32 subtract, promoted
        if (a.mode == GSR_BOX_NONE) {
            in = true;
        } else if (a.mode == GSR_BOX_OBB) {
            in = true;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double r = __dadd_rn(__dadd_rn(__dmul_rn(a.m[3 * k], t[0]), __dmul_rn(a.m[3 * k + 1], t[1])),
                                           __dmul_rn(a.m[3 * k + 2], t[2]));
                in = in && (r >= a.lo[k]) && (r <= a.hi[k]);
            }
        } else {
            in = true;
#pragma unroll
            for (int k = 0; k < 3; ++k) in = in && (t[k] >= a.lo[k]) && (t[k] <= a.hi[k]);
        }
        if (in)
#pragma unroll
            for (int k = 0; k < 3; ++k) o[k] = orig[i * 3 + k];
    }
    uint32_t v[7];
    v[0] = in ? 1u : 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        v[1 + k] = in ? ord_key(o[k]) : 0xffffffffu;
        v[4 + k] = in ? ord_key(o[k]) : 0u;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v[0] += __shfl_xor(v[0], off, 64);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            v[1 + k] = min(v[1 + k], (uint32_t)__shfl_xor(v[1 + k], off, 64));
            v[4 + k] = max(v[4 + k], (uint32_t)__shfl_xor(v[4 + k], off, 64));
        }
    }
    const int w = threadIdx.x >> 6;
    if (__lane_id() == 0)
#pragma unroll
        for (int k = 0; k < 7; ++k) red[k][w] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = 0, mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0u, 0u, 0u};
        for (int j = 0; j < kThreads / 64; ++j) {
            c += red[0][j];
            for (int k = 0; k < 3; ++k) {
                mn[k] = min(mn[k], red[1 + k][j]);
                mx[k] = max(mx[k], red[4 + k][j]);
            }
        }
        if (c) {
            atomicAdd(stats, c);
            for (int k = 0; k < 3; ++k) {
                atomicMin(stats + 1 + k, mn[k]);
                atomicMax(stats + 4 + k, mx[k]);
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_crop_flag(const float* __restrict__ orig, int64_t n, float x0, float y0,
                                                        float z0, float x1, float y1, float z1,
                                                        uint32_t* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float x = orig[i * 3], y = orig[i * 3 + 1], z = orig[i * 3 + 2];
    flag[i] = (x >= x0 && x <= x1 && y >= y0 && y <= y1 && z >= z0 && z <= z1) ? 1u : 0u;
}

// after the in-place exclusive scan of the flags: rows[off] = i for kept rows
__global__ __launch_bounds__(kThreads) void k_crop_write(const float* __restrict__ orig, int64_t n, float x0, float y0,
                                                         float z0, float x1, float y1, float z1,
                                                         const uint32_t* __restrict__ off, int64_t* __restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float x = orig[i * 3], y = orig[i * 3 + 1], z = orig[i * 3 + 2];
    if (x >= x0 && x <= x1 && y >= y0 && y <= y1 && z >= z0 && z <= z1) rows[off[i]] = i;
}

__global__ __launch_bounds__(kThreads) void k_iota64(int64_t n, int64_t* __restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i < n) rows[i] = i;
}

template <typename T>
struct Tmp {
    T* p = nullptr;
    ~Tmp() {
        if (p) (void)hipFree(p);
    }
    int alloc(size_t n) {
        if (hipMalloc(&p, (n ? n : 1) * sizeof(T)) != hipSuccess) {
            p = nullptr;
            return set_error(GSR_ERR_NOMEM, "export: hipMalloc failed");
        }
        return GSR_OK;
    }
};

}  // namespace

int launch_points_center(const float* xyz, int64_t n, float* out3, hipStream_t s) {
    if (n <= 0) return set_error(GSR_ERR_INVALID, "points_center: empty point set");
    k_center_seq<<<1, 64, 0, s>>>(xyz, n, out3);
    GSR_LAUNCH_CHECK("center_seq");
    return GSR_OK;
}

}  // namespace gsr

using namespace gsr;

extern "C" int gsr_points_center(const float* xyz_dev, int64_t n, float center[3], void* stream) {
    if (!xyz_dev || !center || n <= 0) return set_error(GSR_ERR_INVALID, "points_center: bad argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    Tmp<float> c;
    int rc = c.alloc(3);
    if (rc) return rc;
    k_center_seq<<<1, 64, 0, s>>>(xyz_dev, n, c.p);
    GSR_LAUNCH_CHECK("center_seq");
    GSR_HIP_CHECK(hipMemcpyAsync(center, c.p, 3 * sizeof(float), hipMemcpyDeviceToHost, s));
    GSR_HIP_CHECK(hipStreamSynchronize(s));
    return GSR_OK;
}

extern "C" int gsr_export_select(const float* xyz_cur_dev, const float* xyz_orig_dev, int64_t n, const float center[3],
                                 const gsr_box* box, int64_t* rows_dev, int64_t* n_rows, float bbox[6],
                                 int32_t* has_bbox, void* stream) {
    if (!xyz_cur_dev || !xyz_orig_dev || !center || !box || !rows_dev || !n_rows || !bbox || !has_bbox || n < 0)
        return set_error(GSR_ERR_INVALID, "export_select: bad argument");
    if (box->mode < GSR_BOX_NONE || box->mode > GSR_BOX_OBB) return set_error(GSR_ERR_INVALID, "export_select: bad box mode");
    if (n > 0xfffffffell) return set_error(GSR_ERR_OVERFLOW, "export_select: more than 2^32 points");
    hipStream_t s = static_cast<hipStream_t>(stream);
    *n_rows = 0;
    *has_bbox = 0;
    if (n == 0) return GSR_OK;
    BoxArgs a;
    a.mode = box->mode;
    for (int k = 0; k < 3; ++k) {
        a.lo[k] = box->cube_min[k];
        a.hi[k] = box->cube_max[k];
        a.c[k] = center[k];
    }
    for (int k = 0; k < 9; ++k) a.m[k] = box->rot_inv[k];
    Tmp<uint32_t> stats;
    int rc = stats.alloc(7);
    if (rc) return rc;
    uint32_t init[7] = {0u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    GSR_HIP_CHECK(hipMemcpyAsync(stats.p, init, sizeof(init), hipMemcpyHostToDevice, s));
    const unsigned g = (unsigned)((n + kThreads - 1) / kThreads);
    k_box_mask<<<g, kThreads, 0, s>>>(xyz_cur_dev, xyz_orig_dev, n, a, stats.p);
    GSR_LAUNCH_CHECK("box_mask");
    uint32_t h[7];
    GSR_HIP_CHECK(hipMemcpyAsync(h, stats.p, sizeof(h), hipMemcpyDeviceToHost, s));
    GSR_HIP_CHECK(hipStreamSynchronize(s));
    if (h[0] == 0) {  // bbox=None: gsconverter crops nothing
        k_iota64<<<g, kThreads, 0, s>>>(n, rows_dev);
        GSR_LAUNCH_CHECK("iota64");
        GSR_HIP_CHECK(hipStreamSynchronize(s));
        *n_rows = n;
        return GSR_OK;
    }
    for (int k = 0; k < 3; ++k) {
        bbox[k] = from_ord_key(h[1 + k]);
        bbox[3 + k] = from_ord_key(h[4 + k]);
    }
    *has_bbox = 1;
    Tmp<uint32_t> flag, tmp, total;
    if ((rc = flag.alloc((size_t)n)) || (rc = tmp.alloc(scan_tmp_elems((size_t)n))) || (rc = total.alloc(1))) return rc;
    k_crop_flag<<<g, kThreads, 0, s>>>(xyz_orig_dev, n, bbox[0], bbox[1], bbox[2], bbox[3], bbox[4], bbox[5], flag.p);
    GSR_LAUNCH_CHECK("crop_flag");
    if ((rc = scan_exclusive(flag.p, flag.p, (size_t)n, tmp.p, total.p, s))) return rc;
    k_crop_write<<<g, kThreads, 0, s>>>(xyz_orig_dev, n, bbox[0], bbox[1], bbox[2], bbox[3], bbox[4], bbox[5], flag.p,
                                        rows_dev);
    GSR_LAUNCH_CHECK("crop_write");
    uint32_t cnt = 0;
    GSR_HIP_CHECK(hipMemcpyAsync(&cnt, total.p, sizeof(cnt), hipMemcpyDeviceToHost, s));
    GSR_HIP_CHECK(hipStreamSynchronize(s));
    *n_rows = cnt;
    return GSR_OK;
}

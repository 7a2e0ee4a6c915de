// Calibration of the FETCH_SIZE counter for the compositor's access pattern
// (MI355X_MICROARCH.md, HBM section: FETCH_SIZE is calibrated only for wide
// streaming reads, where it reports half the bytes; "other access widths are
// uncalibrated").  Measurement tooling, not product code.
//
// Kernels (each one launch, known distinct bytes):
//   k_stream     float4 per lane, coalesced, over B bytes            -> B bytes
//   k_gather48   48-B records (three float4 loads per lane) at random
//                ids, every record exactly once (a permutation)      -> 48 N bytes,
//                                                                       each 128-B line shared by 2-3 records
//   k_gather48r  the compositor's pattern: 1.76 M ids with repeats over
//                1 M records, in tile-list order (random here)
// Run under: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// Build: hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ void k_stream(const float4* __restrict__ in, size_t n, float* __restrict__ out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 123.456f) out[0] = acc;  // keep the loads
}

template <int KIND>  // 0: permutation, 1: with repeats (distinct kernel names in the trace)
__global__ void k_gather48(const float4* __restrict__ recs, const uint32_t* __restrict__ ids, size_t n,
                           float* __restrict__ out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4* r = recs + 3 * (size_t)ids[i];
        const float4 a = r[0], b = r[1], c = r[2];
        acc += a.x + b.y + c.z + a.w + b.w + c.w;
    }
    if (acc == 123.456f) out[0] = acc;
}

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

int main() {
    const size_t n_rec = 1000000, n_inst = 1756533;
    const size_t stream_bytes = (size_t)256 << 20;
    float4* buf;
    float4* recs;
    uint32_t *perm, *rep;
    float* out;
    CHECK(hipMalloc(&buf, stream_bytes));
    CHECK(hipMalloc(&recs, n_rec * 48));
    CHECK(hipMalloc(&perm, n_rec * 4));
    CHECK(hipMalloc(&rep, n_inst * 4));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(buf, 0, stream_bytes));
    CHECK(hipMemset(recs, 0, n_rec * 48));
    std::vector<uint32_t> p(n_rec), r(n_inst);
    std::mt19937 g(1);
    for (size_t i = 0; i < n_rec; ++i) p[i] = (uint32_t)i;
    std::shuffle(p.begin(), p.end(), g);
    for (size_t i = 0; i < n_inst; ++i) r[i] = (uint32_t)(g() % n_rec);
    CHECK(hipMemcpy(perm, p.data(), n_rec * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(rep, r.data(), n_inst * 4, hipMemcpyHostToDevice));
    const int grid = 4096, block = 256;
    for (int it = 0; it < 3; ++it) {
        k_stream<<<grid, block>>>(buf, stream_bytes / 16, out);
        k_gather48<0><<<grid, block>>>(recs, perm, n_rec, out);
        k_gather48<1><<<grid, block>>>(recs, rep, n_inst, out);
    }
    CHECK(hipDeviceSynchronize());
    std::printf("known bytes: stream %zu | gather48 perm: records %zu + ids %zu | gather48 rep: records %zu "
                "(distinct lines <= %zu) + ids %zu\n",
                stream_bytes, n_rec * 48, n_rec * 4, n_inst * 48, n_rec * 48, n_inst * 4);
    return 0;
}

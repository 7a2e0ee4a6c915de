// Reference point for the radix sorts on MI355X: hipCUB DeviceRadixSort::SortPairs
// (rocPRIM underneath) on the shapes of our two sorts.  Measurement tooling, not
// product code: the product's sorts are the hand-written kernels in
// gsviewer_amd/csrc/radix_sort.hip.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 sort_ref.hip -o sort_ref
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void run(const char* name, size_t n, int end_bit, uint32_t mask) {
    std::vector<uint32_t> hk(n), hv(n);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        hk[i] = (uint32_t)x & mask;
        hv[i] = (uint32_t)i;
    }
    uint32_t *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, n * 4)); CK(hipMalloc(&k1, n * 4)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
    CK(hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
    size_t tmp_bytes = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, v0, v1, (int)n, 0, end_bit));
    void* tmp;
    CK(hipMalloc(&tmp, tmp_bytes));
    for (int i = 0; i < 3; ++i) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, (int)n, 0, end_bit));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int iters = 50;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) CK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, (int)n, 0, end_bit));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-28s n=%zu bits=%d: %.1f us per sort\n", name, n, end_bit, 1e3 * ms / iters);
    CK(hipFree(tmp)); CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(v0)); CK(hipFree(v1));
}

int main() {
    run("depth keys (32-bit)", 1000000, 32, 0xffffffffu);
    run("depth keys (32-bit)", 800000, 32, 0xffffffffu);
    run("tile keys (13-bit)", 1817600, 13, 0x1fffu);
    run("tile keys (15-bit, 4K)", 4000000, 15, 0x7fffu);
    return 0;
}

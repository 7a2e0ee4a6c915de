// Checks the DPP wave scan / reduce of gsr_internal.h against a serial scan
// on random data (one wave per 64 values).  Prints the mismatch count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
#include "gsr_internal.h"

__global__ void k_check(const uint32_t* in, uint32_t* inc_out, uint32_t* red_out, uint32_t* max_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = in[i];
    inc_out[i] = gsr::wave_inclusive_scan(v);
    red_out[i] = gsr::wave_reduce_sum(v);
    max_out[i] = gsr::wave_reduce_max(v * 40503u);  // spread over the full 32-bit range
}

int main() {
    const int n = 64 * 4096;
    std::vector<uint32_t> h(n), inc(n), red(n), mx(n);
    srand(7);
    for (int i = 0; i < n; ++i) h[i] = (i % 7 == 0) ? 0u : (uint32_t)(rand() % 100000);
    uint32_t *d, *di, *dr, *dm;
    if (hipMalloc(&d, n * 4) || hipMalloc(&di, n * 4) || hipMalloc(&dr, n * 4) || hipMalloc(&dm, n * 4)) return 2;
    if (hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice)) return 2;
    k_check<<<n / 256, 256>>>(d, di, dr, dm);
    if (hipDeviceSynchronize()) return 3;
    if (hipMemcpy(inc.data(), di, n * 4, hipMemcpyDeviceToHost) || hipMemcpy(red.data(), dr, n * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(mx.data(), dm, n * 4, hipMemcpyDeviceToHost)) return 2;
    long bad_inc = 0, bad_red = 0, bad_max = 0;
    for (int w = 0; w < n / 64; ++w) {
        uint32_t run = 0, tot = 0, m = 0;
        for (int l = 0; l < 64; ++l) {
            tot += h[w * 64 + l];
            m = std::max(m, h[w * 64 + l] * 40503u);
        }
        for (int l = 0; l < 64; ++l) {
            run += h[w * 64 + l];
            if (inc[w * 64 + l] != run) ++bad_inc;
            if (red[w * 64 + l] != tot) ++bad_red;
            if (mx[w * 64 + l] != m) ++bad_max;
        }
    }
    printf("dpp_scan_check: %d values, inclusive-scan mismatches %ld, reduce mismatches %ld, max mismatches %ld\n", n,
           bad_inc, bad_red, bad_max);
    return (bad_inc || bad_red || bad_max) ? 1 : 0;
}

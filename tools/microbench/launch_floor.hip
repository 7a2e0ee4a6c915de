// The cost of a dependent kernel launch on one stream (measurement tooling,
// not product code): why every kernel of a frame alone costs >= ~5 us.
// Each case runs REPS launches back to back on one stream; wall time per
// launch from events around the whole run:
//   empty         1 block, no memory access
//   empty_wide    512 blocks of 256 threads, no memory access
//   write         512 blocks, each writes 1 KB (plain stores)
//   read_write    512 blocks, each reads the previous launch's 1 KB of another
//                 block and writes its own (a dependent chain like the sorts')
//   rows          the radix offsets kernel's shape: 512 blocks of 4 waves, each
//                 wave scans a row of 489 counts and stores it back
//   rows_graph    the same, 100 launches captured in a HIP graph and replayed
// Build: hipcc --offload-arch=gfx950 -O3 launch_floor.hip -o launch_floor
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_empty() {}

__global__ void k_write(uint32_t* out, uint32_t v) { out[blockIdx.x * 256 + threadIdx.x] = v + threadIdx.x; }

__global__ void k_read_write(const uint32_t* in, uint32_t* out) {
    const uint32_t src = ((blockIdx.x * 97u + 13u) % gridDim.x) * 256u + threadIdx.x;
    out[blockIdx.x * 256 + threadIdx.x] = in[src] + 1u;
}

__global__ void k_rows(uint32_t* hist, uint32_t ntiles) {
    const uint32_t d = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t* row = hist + (size_t)d * ntiles;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t per = (ntiles + 63) / 64;
    uint32_t c[8], s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t i = lane * per + k;
        c[k] = (k < (int)per && i < ntiles) ? row[i] : 0u;
        s += c[k];
    }
    // (no cross-lane scan: the memory round trip and the kernel boundary are what is measured)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t i = lane * per + k;
        if (k < (int)per && i < ntiles) row[i] = s;
        s += c[k];
    }
}

int main() {
    const int REPS = 2000;
    uint32_t *a, *b, *h;
    if (hipMalloc(&a, 512 * 256 * 4) || hipMalloc(&b, 512 * 256 * 4) || hipMalloc(&h, 2048 * 489 * 4)) return 2;
    hipMemset(a, 0, 512 * 256 * 4);
    hipMemset(h, 0, 2048 * 489 * 4);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 50; ++i) launch(i);
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int i = 0; i < REPS; ++i) launch(i);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-12s %7.2f us per launch\n", name, 1e3 * ms / REPS);
    };
    run("empty", [&](int) { k_empty<<<1, 64, 0, s>>>(); });
    run("empty_wide", [&](int) { k_empty<<<512, 256, 0, s>>>(); });
    run("write", [&](int i) { k_write<<<512, 256, 0, s>>>(a, (uint32_t)i); });
    run("read_write", [&](int i) {
        if (i & 1) k_read_write<<<512, 256, 0, s>>>(b, a);
        else k_read_write<<<512, 256, 0, s>>>(a, b);
    });
    run("rows", [&](int) { k_rows<<<512, 256, 0, s>>>(h, 489u); });
    // the same chain of `rows` launches captured once in a HIP graph and replayed
    {
        const int G = 100;
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int i = 0; i < G; ++i) k_rows<<<512, 256, 0, s>>>(h, 489u);
        hipStreamEndCapture(s, &g);
        if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return 4;
        for (int i = 0; i < 3; ++i) hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        hipEventRecord(e0, s);
        for (int i = 0; i < REPS / G; ++i) hipGraphLaunch(ge, s);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-12s %7.2f us per launch\n", "rows_graph", 1e3 * ms / (REPS / G * G));
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 3;
}

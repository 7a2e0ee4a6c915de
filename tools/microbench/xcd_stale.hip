// Cross-XCD visibility of a hand-off whose reader already holds the lines
// (measurement tooling, not product code): the question behind the tail
// merge's partial and saturation-word reads (composite.hip).
//
// in-launch: one launch of 16 one-wave blocks; block 0 (reader) first loads
//   two 256-B regions, A with plain loads and B with sc1 loads, so its CU's
//   L1 / its XCD's L2 may hold them; block 1 (another XCD: blocks are dealt
//   round-robin) then rewrites both with sc1 stores, waits, and adds to a
//   counter; the reader, after its atomic poll of the counter sees the add,
//   reads both regions again by one of the read forms below and counts the
//   lanes that still see the old value.
// cross-launch: launch 1 every block reads A and B (plain / sc1), launch 2
//   block 1 rewrites them (sc1 stores), launch 3 every block reads them by the
//   read form; stale lanes counted on the blocks whose XCD is not the writer's.
// Read forms: 0 plain, 1 agent acquire + plain, 2 sc1 load, 3 agent acquire +
// sc1 load, 4 atomic (fetch_max 0).
// Build: hipcc --offload-arch=gfx950 -O3 xcd_stale.hip -o xcd_stale
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); }

// plain: no cache-policy bits (a C++ volatile load is emitted with sc0 sc1, i.e. uncached)
__device__ __forceinline__ uint32_t ld_plain(const uint32_t* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t ld_atomic(uint32_t* p) {
    return __hip_atomic_fetch_max(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t read_form(uint32_t* p, int form) {
    switch (form) {
        case 0: return ld_plain(p);
        case 1:
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return ld_plain(p);
        case 2: return ld_sc1(p);
        case 3:
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            return ld_sc1(p);
        default: return ld_atomic(p);
    }
}

// ctl: [0] reader ready, [1] writer done, [2] reader xcc, [3] writer xcc
__global__ void k_inlaunch(uint32_t* A, uint32_t* B, uint32_t* C, uint32_t* ctl, uint32_t* stale, uint32_t epoch,
                           int form) {
    const uint32_t lane = threadIdx.x;
    uint32_t* a = A + lane * 32;  // one lane per 128-B line
    uint32_t* b = B + lane * 32;
    uint32_t* cc = C + lane * 32;
    if (blockIdx.x == 0) {
        uint32_t keep = ld_plain(a) + ld_sc1(b) + ld_sc1(cc);
        asm volatile("" ::"v"(keep));
        if (lane == 0) {
            ctl[2] = xcc_id();
            __hip_atomic_store(ctl + 0, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_atomic(ctl + 1) != epoch && __builtin_amdgcn_s_memrealtime() - t0 < 10000000ull)
                __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t ra = read_form(a, form), rb = read_form(b, form), rc = read_form(cc, form);
        if (ra != epoch) atomicAdd(stale + 0, 1u);
        if (rb != epoch) atomicAdd(stale + 1, 1u);
        if (rc != epoch) atomicAdd(stale + 2, 1u);
    } else if (blockIdx.x == 1) {
        if (lane == 0) {
            ctl[3] = xcc_id();
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (ld_atomic(ctl + 0) != epoch && __builtin_amdgcn_s_memrealtime() - t0 < 10000000ull)
                __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_wave_barrier();
        st_sc1(a, epoch);
        st_sc1(b, epoch);
        __hip_atomic_fetch_max(cc, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_exchange(ctl + 1, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_touch(uint32_t* A, uint32_t* B) {  // every block reads A plain and B sc1
    const uint32_t lane = threadIdx.x;
    uint32_t keep = ld_plain(A + lane * 32) + ld_sc1(B + lane * 32);
    asm volatile("" ::"v"(keep));
}
__global__ void k_write(uint32_t* A, uint32_t* B, uint32_t* ctl, uint32_t epoch) {
    if (blockIdx.x != 1) return;
    const uint32_t lane = threadIdx.x;
    st_sc1(A + lane * 32, epoch);
    st_sc1(B + lane * 32, epoch);
    if (lane == 0) ctl[3] = xcc_id();
}
__global__ void k_read(uint32_t* A, uint32_t* B, uint32_t* ctl, uint32_t* stale, uint32_t epoch, int form) {
    const uint32_t lane = threadIdx.x;
    const uint32_t ra = read_form(A + lane * 32, form), rb = read_form(B + lane * 32, form);
    if (xcc_id() == ctl[3]) return;  // (ctl[3]: written by the previous launch)
    if (ra != epoch) atomicAdd(stale + 0, 1u);
    if (rb != epoch) atomicAdd(stale + 1, 1u);
}

int main() {
    uint32_t *A, *B, *C, *ctl, *stale;
    hipMalloc(&A, 64 * 128);
    hipMalloc(&B, 64 * 128);
    hipMalloc(&C, 64 * 128);
    hipMemset(C, 0, 64 * 128);
    hipMalloc(&ctl, 64);
    hipMalloc(&stale, 12);
    hipMemset(A, 0, 64 * 128);
    hipMemset(B, 0, 64 * 128);
    hipMemset(ctl, 0, 64);
    const char* names[5] = {"plain", "acquire+plain", "sc1", "acquire+sc1", "atomic"};
    const int reps = 400;
    uint32_t epoch = 1;
    for (int form = 0; form < 5; ++form) {
        hipMemset(stale, 0, 12);
        uint32_t same_xcc = 0;
        for (int r = 0; r < reps; ++r, ++epoch) {
            k_inlaunch<<<16, 64>>>(A, B, C, ctl, stale, epoch, form);
            uint32_t c[4];
            hipMemcpy(c, ctl, 16, hipMemcpyDeviceToHost);
            same_xcc += c[2] == c[3];
        }
        uint32_t s[3];
        hipMemcpy(s, stale, 12, hipMemcpyDeviceToHost);
        printf("in-launch    %-14s stale lanes: A(plain-cached, sc1 store) %u / %d, B(sc1-cached, sc1 store) %u / %d, "
               "C(sc1-cached, atomic max) %u / %d (same-XCD runs %u)\n",
               names[form], s[0], reps * 64, s[1], reps * 64, s[2], reps * 64, same_xcc);
    }
    for (int form = 0; form < 5; ++form) {
        hipMemset(stale, 0, 8);
        for (int r = 0; r < reps; ++r, ++epoch) {
            k_touch<<<16, 64>>>(A, B);
            k_write<<<16, 64>>>(A, B, ctl, epoch);
            k_read<<<16, 64>>>(A, B, ctl, stale, epoch, form);
        }
        uint32_t s[2];
        hipMemcpy(s, stale, 8, hipMemcpyDeviceToHost);
        printf("cross-launch %-14s stale lanes: A(plain-cached) %u / %d, B(sc1-cached) %u / %d\n", names[form], s[0],
               reps * 64 * 14, s[1], reps * 64 * 14);
    }
    return 0;
}

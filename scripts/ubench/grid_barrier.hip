// Microbenchmark for the persistent-learner question: what a
// grid-wide barrier inside one persistent kernel costs on MI355X, against what a
// kernel boundary costs on one stream (the learner step is a ~65-launch dependent
// chain with a ~4 us median gap, profiles/r05/learner/timeline).
//
//   mode barrier: one launch of G workgroups (256 threads, all resident: G <= CUs)
//                 that passes N grid barriers back to back -- a global arrival
//                 counter and a generation word, agent-scope release/acquire, the
//                 arriving workgroup's thread 0 spins (s_sleep) on the generation;
//                 reported: wall time per barrier (HIP events over the launch)
//   mode barrier2: the same with a two-level barrier (8 group counters, then one)
//   mode chain:   N launches of the same G-workgroup kernel doing nothing but its
//                 entry/exit, back to back on one stream: wall time per launch
//   mode chain_work: as chain, each launch touching 64 KiB (a BN-sized pass)
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/grid_barrier.hip -o scripts/ubench/grid_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

// count[0] = arrivals, count[1] = generation; the last arrival resets the count and
// bumps the generation.  Every wave of the workgroup waits at the workgroup barrier;
// thread 0 alone talks to memory.  The spin is bounded (the grid is sized to be
// resident; a bound keeps a mis-sized launch from hanging the device).
__device__ __forceinline__ bool grid_barrier(unsigned *count, unsigned G) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned a = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (a == G - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(count + 1, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(count + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 24)) {
                    ok = false;
                    break;
                }
            }
        }
    }
    __syncthreads();
    return ok;
}

// two-level: the workgroups of group b % 8 (one group per XCD when the dispatcher
// places workgroups round-robin, as MI355X does; correct for any placement) arrive on
// their group's counter (own 128-B line); each group's last arrival arrives on the
// global counter, whose last arrival bumps the generation.  c[32 g] = group g,
// c[256] = global, c[288] = generation.
__device__ __forceinline__ bool grid_barrier2(unsigned *c, unsigned G) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const unsigned grp = blockIdx.x % 8, gsize = G / 8 + (grp < G % 8 ? 1u : 0u), ngroups = G < 8 ? G : 8;
        const unsigned g = __hip_atomic_load(c + 288, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool last = false;
        if (__hip_atomic_fetch_add(c + 32 * grp, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
            __hip_atomic_store(c + 32 * grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = __hip_atomic_fetch_add(c + 256, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        }
        if (last) {
            __hip_atomic_store(c + 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(c + 288, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(c + 288, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 24)) {
                    ok = false;
                    break;
                }
            }
        }
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(256) void k_barriers2(unsigned *c, unsigned G, int n, unsigned *fail) {
    for (int i = 0; i < n; ++i)
        if (!grid_barrier2(c, G)) {
            if (threadIdx.x == 0) atomicAdd(fail, 1u);
            return;
        }
}

__global__ __launch_bounds__(256) void k_barriers(unsigned *count, unsigned G, int n, unsigned *fail) {
    for (int i = 0; i < n; ++i)
        if (!grid_barrier(count, G)) {
            if (threadIdx.x == 0) atomicAdd(fail, 1u);
            return;
        }
}

__global__ __launch_bounds__(256) void k_empty(float *p) {
    if (p && threadIdx.x == 1024) p[0] = 1.f;   // never true: keeps the kernel non-trivial
}

__global__ __launch_bounds__(256) void k_touch(float *p, int per_wg) {
    float *q = p + (size_t)blockIdx.x * per_wg;
    for (int i = threadIdx.x; i < per_wg; i += 256) q[i] = q[i] * 0.5f + 1.f;
}

int main(int argc, char **argv) {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    unsigned *count, *fail;
    float *buf;
    CK(hipMalloc(&count, 2048));
    CK(hipMalloc(&fail, 4));
    CK(hipMalloc(&buf, (size_t)64 << 20));
    CK(hipMemset(count, 0, 2048));
    CK(hipMemset(fail, 0, 4));
    CK(hipMemset(buf, 0, (size_t)64 << 20));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grids[] = {64, 128, cus};
    std::printf("device %s, %d CUs\n", prop.name, cus);
    for (int G : grids) {
        if (G > cus) continue;
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 2000;
            k_barriers<<<G, 256, 0, st>>>(count, (unsigned)G, 10, fail);   // warm
            CK(hipEventRecord(a, st));
            k_barriers<<<G, 256, 0, st>>>(count, (unsigned)G, n, fail);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            unsigned hf = 0;
            CK(hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost));
            std::printf("barrier    G %4d: %7.3f us per grid barrier (%d barriers in one launch)%s\n", G,
                        ms * 1e3 / n, n, hf ? "  SPIN BOUND HIT" : "");
            if (hf) return 2;
        }
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 2000;
            unsigned *c2 = count + 64;   // its own lines, past the flat barrier's words
            k_barriers2<<<G, 256, 0, st>>>(c2, (unsigned)G, 10, fail);   // warm
            CK(hipEventRecord(a, st));
            k_barriers2<<<G, 256, 0, st>>>(c2, (unsigned)G, n, fail);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            unsigned hf = 0;
            CK(hipMemcpy(&hf, fail, 4, hipMemcpyDeviceToHost));
            std::printf("barrier2   G %4d: %7.3f us per grid barrier (two-level: 8 groups, then global)%s\n", G,
                        ms * 1e3 / n, hf ? "  SPIN BOUND HIT" : "");
            if (hf) return 2;
        }
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 2000;
            for (int i = 0; i < 20; ++i) k_empty<<<G, 256, 0, st>>>(nullptr);
            CK(hipEventRecord(a, st));
            for (int i = 0; i < n; ++i) k_empty<<<G, 256, 0, st>>>(nullptr);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("chain      G %4d: %7.3f us per launch (empty kernel, %d back to back)\n", G, ms * 1e3 / n, n);
        }
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 2000, per = (64 << 10) / 4 / G;
            CK(hipEventRecord(a, st));
            for (int i = 0; i < n; ++i) k_touch<<<G, 256, 0, st>>>(buf, per);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("chain_work G %4d: %7.3f us per launch (64 KiB read+write per launch)\n", G, ms * 1e3 / n);
        }
    }
    CK(hipStreamSynchronize(st));
    return 0;
}

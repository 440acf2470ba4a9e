// Microbenchmark: per-CU rate of streaming an L2-resident weight set (the C4
// forward's 1 KiB MFMA A-fragments) into a CU, by load kind and depth.
//   mode 0: global_load_dwordx4 -> VGPRs, each wave its own fragment (4 KiB unique / CU / step)
//   mode 1: global_load_dwordx4 -> VGPRs, all 4 waves the same fragment (1 KiB unique / CU / step)
//   mode 2: global_load_lds_dwordx4 -> LDS ring, each wave its own fragment
// Reports bytes per shader cycle per CU (s_memtime) over K steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kFrag = 1024;     // bytes per wave-instruction
constexpr int kNF = 1024;       // fragments in the set (1 MiB)
constexpr int kSteps = 4096;

template <int MODE, int D>
__global__ __launch_bounds__(256) void k_stream(const uint4 *__restrict__ w, unsigned long long *cyc, uint4 *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8 * kFrag];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4 acc = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE < 2) {
        uint4 r[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int f = MODE == 0 ? (i * 4 + wave + blockIdx.x * 7) % kNF : (i + blockIdx.x * 7) % kNF;
            r[i] = w[f * 64 + lane];
        }
        for (int s = 0; s < kSteps; s += D) {
#pragma unroll
            for (int i = 0; i < D; ++i) {
                acc.x ^= r[i].x; acc.y += r[i].y; acc.z ^= r[i].z; acc.w += r[i].w;
                const int f = MODE == 0 ? ((s + D + i) * 4 + wave + blockIdx.x * 7) % kNF
                                        : (s + D + i + blockIdx.x * 7) % kNF;
                r[i] = w[f * 64 + lane];
            }
        }
#pragma unroll
        for (int i = 0; i < D; ++i) { acc.x ^= r[i].x; acc.y += r[i].y; }
    } else {
        uint8_t *base = lds + wave * 8 * kFrag;
        for (int s = 0; s < kSteps; ++s) {
            const int f = (s * 4 + wave + blockIdx.x * 7) % kNF;
            __builtin_amdgcn_global_load_lds((const void *)(w + f * 64 + lane), (__attribute__((address_space(3))) void *)(base + (s % 8) * kFrag), 16, 0, 0);
            if (s >= D) {
                if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else if constexpr (D == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                const uint4 v = *(const uint4 *)(base + ((s - D) % 8) * kFrag + lane * 16);
                acc.x ^= v.x; acc.y += v.y;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
    if (acc.x == 0x12345678u && acc.y == 7u) sink[threadIdx.x] = acc;
}

template <int MODE, int D>
void run(const uint4 *w, unsigned long long *cyc, uint4 *sink, int grid, const char *name) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) k_stream<MODE, D><<<grid, 256>>>(w, cyc, sink);
    hipEventRecord(a);
    k_stream<MODE, D><<<grid, 256>>>(w, cyc, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(grid * 4);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0, sum = 0;
    for (auto v : h) { mx = v > mx ? v : mx; sum += v; }
    const double bytes_cu = (double)kSteps * (MODE == 1 ? kFrag : 4 * kFrag);   // unique bytes into the CU
    const double loaded_cu = (double)kSteps * 4 * kFrag;                          // bytes the waves load
    printf("%-34s grid %4d D %d: %.1f us, mean %.0f cyc/wave, %.1f B/clk/CU unique, %.1f B/clk/CU loaded, clk %.2f GHz\n",
           name, grid, D, ms * 1e3, sum / h.size(), bytes_cu / (sum / h.size()), loaded_cu / (sum / h.size()),
           sum / h.size() / (ms * 1e3) * 1e-3);
}

int main() {
    uint4 *w, *sink;
    unsigned long long *cyc;
    hipMalloc(&w, kNF * kFrag);
    hipMalloc(&sink, 256 * 16);
    hipMalloc(&cyc, 2048 * 4 * 8);
    hipMemset(w, 1, kNF * kFrag);
    for (int grid : {256, 1}) {
        run<0, 2>(w, cyc, sink, grid, "vgpr, per-wave fragments");
        run<0, 4>(w, cyc, sink, grid, "vgpr, per-wave fragments");
        run<0, 8>(w, cyc, sink, grid, "vgpr, per-wave fragments");
        run<0, 16>(w, cyc, sink, grid, "vgpr, per-wave fragments");
        run<1, 4>(w, cyc, sink, grid, "vgpr, shared fragment (L1 reuse)");
        run<1, 8>(w, cyc, sink, grid, "vgpr, shared fragment (L1 reuse)");
        run<2, 2>(w, cyc, sink, grid, "lds-dma, per-wave fragments");
        run<2, 4>(w, cyc, sink, grid, "lds-dma, per-wave fragments");
        run<2, 6>(w, cyc, sink, grid, "lds-dma, per-wave fragments");
    }
    return 0;
}

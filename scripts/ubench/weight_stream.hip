// Microbenchmark: per-CU rate of streaming an L2-resident weight set (the C4
// forward's 1 KiB MFMA A-fragments, 1 MiB in all) into a CU's registers.
//   mode 0: every wave loads its own fragment per step (4 KiB unique / CU / step)
//   mode 1: all 4 waves load the same fragment (1 KiB unique, 4 KiB loaded)
//   mode 2: as mode 0 with nontemporal loads
//   mode 3: wave 0 alone loads 4 fragments per step (the others idle)
// D = loads in flight per wave.  Reports loaded bytes per shader cycle per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kNF = 1024;
constexpr int kSteps = 4096;

template <int MODE>
__device__ __forceinline__ uint4 ld(const uint4 *p) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (MODE == 2) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}

template <int MODE, int D>
__global__ __launch_bounds__(256) void k_stream(const uint4 *__restrict__ w, unsigned long long *cyc, uint4 *sink) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (MODE == 3 && wave) return;
    const int per = MODE == 3 ? 4 : 1;   // fragments per step per loading wave
    uint4 acc = make_uint4(0, 0, 0, 0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    uint4 r[D];
    auto frag = [&](int i) {   // fragment of load number i of this wave
        const int s = i / per, k = i % per;
        return MODE == 1 ? (s + blockIdx.x * 7) & (kNF - 1)
                         : (s * 4 + (MODE == 3 ? k : wave) + blockIdx.x * 7) & (kNF - 1);
    };
#pragma unroll
    for (int i = 0; i < D; ++i) r[i] = ld<MODE>(w + frag(i) * 64 + lane);
    for (int s = 0; s < kSteps * per; s += D) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            acc.x ^= r[i].x; acc.y += r[i].y; acc.z ^= r[i].z; acc.w += r[i].w;
            r[i] = ld<MODE>(w + frag(s + D + i) * 64 + lane);
        }
    }
#pragma unroll
    for (int i = 0; i < D; ++i) { acc.x ^= r[i].x; acc.y += r[i].y; acc.z ^= r[i].z; acc.w += r[i].w; }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int MODE, int D>
void run(const uint4 *w, unsigned long long *cyc, uint4 *sink, int grid, const char *name) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; ++rep) k_stream<MODE, D><<<grid, 256>>>(w, cyc, sink);
    (void)hipEventRecord(a);
    k_stream<MODE, D><<<grid, 256>>>(w, cyc, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(grid);
    (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double sum = 0;
    for (auto v : h) sum += v;
    const double mean = sum / h.size();
    const double loaded = (double)kSteps * 4 * 1024;   // bytes loaded into the CU
    printf("%-36s grid %3d D %2d: %7.1f us, %8.0f cyc, %5.1f B/clk/CU loaded (%4.1f KiB in flight/CU), clk %.2f GHz\n",
           name, grid, D, ms * 1e3, mean, loaded / mean, (MODE == 3 ? 1 : 4) * D * 1.0, mean / (ms * 1e3) * 1e-3);
}

int main() {
    uint4 *w, *sink;
    unsigned long long *cyc;
    (void)hipMalloc(&w, kNF * 1024);
    (void)hipMalloc(&sink, 256 * 16);
    (void)hipMalloc(&cyc, 2048 * 8);
    (void)hipMemset(w, 1, kNF * 1024);
    for (int grid : {256, 1}) {
        run<0, 1>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 2>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 3>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 4>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 6>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 8>(w, cyc, sink, grid, "own fragment per wave");
        run<0, 12>(w, cyc, sink, grid, "own fragment per wave");
        run<1, 2>(w, cyc, sink, grid, "shared fragment (L1 reuse)");
        run<1, 4>(w, cyc, sink, grid, "shared fragment (L1 reuse)");
        run<1, 8>(w, cyc, sink, grid, "shared fragment (L1 reuse)");
        run<2, 2>(w, cyc, sink, grid, "own fragment, nontemporal");
        run<2, 4>(w, cyc, sink, grid, "own fragment, nontemporal");
        run<2, 8>(w, cyc, sink, grid, "own fragment, nontemporal");
        run<3, 4>(w, cyc, sink, grid, "wave 0 loads all 4");
        run<3, 8>(w, cyc, sink, grid, "wave 0 loads all 4");
        run<3, 16>(w, cyc, sink, grid, "wave 0 loads all 4");
    }
    return 0;
}

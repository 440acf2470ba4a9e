// Microbenchmark for the C4 forward's epilogue question (profiles/r06/README.md: the
// epilogue's LDS stores cost ~750-900 cycles per trunk conv at S = 8 whatever their
// bank pattern, count or MFMA overlap window).  What does an LDS store cost a wave that
// is issuing MFMAs back to back, and does it depend on the bytes or the instruction?
//
// One workgroup of 4 waves per CU (one wave per SIMD, as k_forward), 256 workgroups.
// Each wave loops over blocks of 8 independent v_mfma_f32_16x16x32_bf16 (128 cycles of
// MFMA issue) with NST LDS stores of W bytes per lane and NRD ds_read_b128 per block
// interleaved; the reads feed the next block's B operands (as the forward's B ring).
// Reported: s_memtime cycles per block per wave (mean over waves) and the extra cycles
// per store against the store-free block with the same reads.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/ubench/lds_store_mfma.hip -o scripts/ubench/lds_store_mfma
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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaveBytes = 16384;   // each wave's own 16 KB of LDS (4 waves: 64 KB)

template <int W> struct St;
template <> struct St<4> {
    static __device__ __forceinline__ void put(char *p, unsigned v) { *(unsigned *)p = v; }
};
template <> struct St<8> {
    static __device__ __forceinline__ void put(char *p, unsigned v) { *(u32x2 *)p = u32x2{v, v ^ 1u}; }
};
template <> struct St<16> {
    static __device__ __forceinline__ void put(char *p, unsigned v) { *(u32x4 *)p = u32x4{v, v ^ 1u, v ^ 2u, v ^ 3u}; }
};

template <int NST, int W, int NRD, int SFIRST = 0>
__global__ __launch_bounds__(256) void k_mix(float *out, unsigned long long *cyc, int iters) {
    __shared__ __attribute__((aligned(16))) char lds[4 * kWaveBytes];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char *mine = lds + wave * kWaveBytes;
    // seed the read area (first 8 KB of the wave's region) so reads return defined bits
    for (int i = lane; i < kWaveBytes / 16; i += 64) ((u32x4 *)mine)[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
    __syncthreads();
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 av = u32x4{0x3f803f80u ^ (unsigned)lane, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    u32x4 rb[NRD > 0 ? NRD : 1];
#pragma unroll
    for (int r = 0; r < (NRD > 0 ? NRD : 1); ++r) rb[r] = av;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        u32x4 nb[NRD > 0 ? NRD : 1];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                             __builtin_bit_cast(bf16x8, rb[m % (NRD > 0 ? NRD : 1)]),
                                                             acc[m], 0, 0, 0);
            // slot m of the block: reads in the first NRD slots and stores in the last NST
            // (SFIRST = 0), or stores first and reads last (SFIRST = 1)
            const int rs = SFIRST ? m - (8 - NRD) : m, ss = SFIRST ? m : m - (8 - NST);
            const bool rd = rs >= 0 && rs < NRD, st = ss >= 0 && ss < NST;
            if (rd)   // reads from the first 8 KB, a different 1 KB each read
                nb[rs] = ((const u32x4 *)(mine + ((it * NRD + rs) & 7) * 1024))[lane];
            if (st)   // stores into the second 8 KB
                St<W>::put(mine + 8192 + ((it * NST + ss) * 64 * W) % 8192 + lane * W, (unsigned)(it + m));
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (rd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (st) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
#pragma unroll
        for (int r = 0; r < NRD; ++r) rb[r] = nb[r];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
    __syncthreads();
    s += (float)((const unsigned *)(mine + 8192))[lane];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int NST, int W, int NRD, int SFIRST = 0>
static double run(float *out, unsigned long long *cyc, unsigned long long *h, int grid, int iters) {
    k_mix<NST, W, NRD, SFIRST><<<grid, 256>>>(out, cyc, iters);   // warm
    CK(hipDeviceSynchronize());
    k_mix<NST, W, NRD, SFIRST><<<grid, 256>>>(out, cyc, iters);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * grid * 4, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < grid * 4; ++i) s += (double)h[i];
    return s / (grid * 4) / iters;
}

template <int NST, int W, int NRD, int SFIRST = 0>
static void line(float *out, unsigned long long *cyc, unsigned long long *h, int grid, int iters, double base) {
    const double c = run<NST, W, NRD, SFIRST>(out, cyc, h, grid, iters);
    std::printf("stores %d x %2d B/lane (%4d B/wave/block), reads %d x b128, %s: %7.1f cycles per 8-MFMA block",
                NST, W, NST * W * 64, NRD, SFIRST ? "stores first" : "reads first ", c);
    if (NST > 0 && base > 0) std::printf("  (+%.1f per store, %.2f B/cycle/wave of the extra)", (c - base) / NST,
                                         (c - base) > 1 ? NST * W * 64 / (c - base) : 0.0);
    std::printf("\n");
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 4096;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount;
    std::printf("device %s, %d CUs, grid %d x 4 waves, %d blocks of 8 MFMAs per wave (s_memtime cycles)\n",
                prop.name, prop.multiProcessorCount, grid, iters);
    float *out;
    unsigned long long *cyc, *h = (unsigned long long *)std::malloc(sizeof(unsigned long long) * grid * 4);
    CK(hipMalloc(&out, sizeof(float) * grid * 256));
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * grid * 4));
    for (int rep = 0; rep < 2; ++rep) {
        const double b0 = run<0, 8, 0>(out, cyc, h, grid, iters);
        line<0, 8, 0>(out, cyc, h, grid, iters, 0);
        line<1, 8, 0>(out, cyc, h, grid, iters, b0);
        line<2, 8, 0>(out, cyc, h, grid, iters, b0);
        line<4, 8, 0>(out, cyc, h, grid, iters, b0);
        line<8, 8, 0>(out, cyc, h, grid, iters, b0);
        line<2, 4, 0>(out, cyc, h, grid, iters, b0);
        line<4, 4, 0>(out, cyc, h, grid, iters, b0);
        line<8, 4, 0>(out, cyc, h, grid, iters, b0);
        line<1, 16, 0>(out, cyc, h, grid, iters, b0);
        line<2, 16, 0>(out, cyc, h, grid, iters, b0);
        line<4, 16, 0>(out, cyc, h, grid, iters, b0);
        const double b3 = run<0, 8, 3>(out, cyc, h, grid, iters);
        line<0, 8, 3>(out, cyc, h, grid, iters, 0);
        line<1, 8, 3>(out, cyc, h, grid, iters, b3);
        line<2, 8, 3>(out, cyc, h, grid, iters, b3);
        line<4, 8, 3>(out, cyc, h, grid, iters, b3);
        line<2, 16, 3>(out, cyc, h, grid, iters, b3);
        line<1, 8, 3, 1>(out, cyc, h, grid, iters, b3);
        line<2, 8, 3, 1>(out, cyc, h, grid, iters, b3);
        line<4, 8, 3, 1>(out, cyc, h, grid, iters, b3);
        const double b6 = run<0, 8, 6>(out, cyc, h, grid, iters);
        line<0, 8, 6>(out, cyc, h, grid, iters, 0);
        line<2, 8, 6>(out, cyc, h, grid, iters, b6);
        line<4, 8, 6>(out, cyc, h, grid, iters, b6);
        line<2, 8, 6, 1>(out, cyc, h, grid, iters, b6);
    }
    CK(hipFree(out));
    CK(hipFree(cyc));
    std::free(h);
    return 0;
}

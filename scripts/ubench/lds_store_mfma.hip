// Microbenchmark for the C4 forward's epilogue question (profiles/r06/README.md: the
// epilogue's LDS stores cost ~750-900 cycles per trunk conv at S = 8 whatever their
// bank pattern, count or MFMA overlap window).  What does an LDS store cost a wave that
// is issuing MFMAs back to back, and does it depend on the bytes or the instruction?
//
// One workgroup of 4 waves per CU (one wave per SIMD, as k_forward); one workgroup
// (no clock throttling) or one per CU.  Each wave loops over blocks of NM
// v_mfma_f32_16x16x32_bf16 on 8 accumulators with NST LDS stores of W bytes per lane,
// spread over the block or bunched at its end; or (modes 2 / 3) one ds_read_b128 issued
// behind / ahead of the stores and waited for kLag MFMAs later (lgkmcnt counts LDS
// operations in issue order, so a read behind stores completes after them).  Reported: s_memtime cycles per block
// per wave (mean over waves), per MFMA, and the extra cycles per store against the
// store-free block.
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

// the block is written in inline asm so that the compiler neither reorders it nor
// shuffles the loop-carried accumulators; the stores' address and data registers are
// loop-invariant, so the loop holds only MFMAs, stores and the loop counter
template <int W> struct St;
template <> struct St<4> {
    static __device__ __forceinline__ void put(unsigned addr, const u32x4 &v) {
        asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v[0]) : "memory");
    }
};
template <> struct St<8> {
    static __device__ __forceinline__ void put(unsigned addr, const u32x4 &v) {
        const u32x2 d = u32x2{v[0], v[1]};
        asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(d) : "memory");
    }
};
template <> struct St<16> {
    static __device__ __forceinline__ void put(unsigned addr, const u32x4 &v) {
        asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
    }
};
__device__ __forceinline__ void mfma(f32x4 &acc, const u32x4 &a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, %0" : "+a"(acc) : "v"(a));
}

// NM MFMAs per block, NST stores of W bytes per lane; MODE 0 spreads the stores over
// the block (one after every NM / NST-th MFMA), MODE 1 issues them back to back after the
// block's last MFMA.  No reads: B = A, so the loop carries only the accumulators.
constexpr int kLag = 6;   // MFMAs between the read's issue and its wait (modes 2 / 3)

template <int NM, int NST, int W, int MODE>
__global__ __launch_bounds__(256) void k_mix(float *out, unsigned long long *cyc, int iters) {
    __shared__ __attribute__((aligned(16))) char lds[4 * kWaveBytes];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    char *mine = lds + wave * kWaveBytes;
    f32x4 acc[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    const u32x4 av = u32x4{0x3f803f80u ^ (unsigned)lane, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
    // per-store LDS addresses (the wave's own 16 KB; 64 W-byte lanes per store): `lds` is
    // the kernel's only LDS object, so it starts at LDS address 0
    const unsigned base = (unsigned)(wave * kWaveBytes + lane * W);
    const unsigned rbase = (unsigned)(wave * kWaveBytes + kWaveBytes / 2 + lane * 16);   // reads: the upper 8 KB
    u32x4 rsink = av;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            mfma(acc[m % 8], av);
            if constexpr (MODE >= 2) {   // one ds_read_b128 behind (2) or ahead of (3) NST stores, waited kLag MFMAs later
                constexpr int rd_at = MODE == 2 ? NST : 0, st0 = MODE == 2 ? 0 : 1, wait_at = (MODE == 2 ? NST : NST + 1) + kLag;
                static_assert(wait_at < NM, "the wait must sit inside the block");
                if (m >= st0 && m < st0 + NST) St<W>::put(base + (((m - st0) * 64 * W) & (kWaveBytes / 2 - 1)), av);
                if (m == rd_at) asm volatile("ds_read_b128 %0, %1" : "=v"(rsink) : "v"(rbase) : "memory");
                if (m == wait_at) {
                    if (MODE == 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    else asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NST) : "memory");
                }
            }
            if (MODE == 0 && NST > 0 && (m + 1) % (NM / (NST > 0 ? NST : 1)) == 0) {
                const int ss = (m + 1) / (NM / (NST > 0 ? NST : 1)) - 1;
                St<W>::put(base + ((ss * 64 * W) & (kWaveBytes - 1)), av);
            }
        }
        if (MODE == 1) {
#pragma unroll
            for (int ss = 0; ss < NST; ++ss) St<W>::put(base + ((ss * 64 * W) & (kWaveBytes - 1)), av);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    (void)rsink;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 8; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
    __syncthreads();
    s += (float)((const unsigned *)mine)[lane];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
}

template <int NM, int NST, int W, int MODE>
static double run(float *out, unsigned long long *cyc, unsigned long long *h, int grid, int iters) {
    k_mix<NM, NST, W, MODE><<<grid, 256>>>(out, cyc, iters);   // warm
    CK(hipDeviceSynchronize());
    k_mix<NM, NST, W, MODE><<<grid, 256>>>(out, cyc, iters);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * grid * 4, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < grid * 4; ++i) s += (double)h[i];
    return s / (grid * 4) / iters;
}

template <int NM, int NST, int W, int MODE>
static void line(float *out, unsigned long long *cyc, unsigned long long *h, int grid, int iters, double base) {
    const double c = run<NM, NST, W, MODE>(out, cyc, h, grid, iters);
    static const char *mode[] = {"spread ", "bunched", "read behind the stores", "read ahead of the stores"};
    std::printf("grid %3d  %2d MFMA + %2d stores x %2d B/lane %s: %7.1f cycles per block, %5.1f per MFMA", grid, NM, NST,
                W, mode[MODE], c, c / NM);
    if (NST > 0 && base > 0) std::printf("  (+%.1f per store)", (c - base) / NST);
    std::printf("\n");
}

template <int NM>
static void sweep(float *out, unsigned long long *cyc, unsigned long long *h, int grid, int iters) {
    const double b = run<NM, 0, 8, 0>(out, cyc, h, grid, iters);
    line<NM, 0, 8, 0>(out, cyc, h, grid, iters, 0);
    line<NM, 1, 8, 0>(out, cyc, h, grid, iters, b);
    line<NM, 2, 8, 0>(out, cyc, h, grid, iters, b);
    line<NM, 4, 8, 0>(out, cyc, h, grid, iters, b);
    line<NM, 8, 8, 0>(out, cyc, h, grid, iters, b);
    line<NM, 2, 8, 1>(out, cyc, h, grid, iters, b);
    line<NM, 4, 8, 1>(out, cyc, h, grid, iters, b);
    line<NM, 8, 8, 1>(out, cyc, h, grid, iters, b);
    line<NM, 4, 4, 0>(out, cyc, h, grid, iters, b);
    line<NM, 2, 16, 0>(out, cyc, h, grid, iters, b);
    line<NM, 4, 16, 0>(out, cyc, h, grid, iters, b);
    line<NM, 4, 16, 1>(out, cyc, h, grid, iters, b);
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
    for (int g : {1, grid}) {   // a read waited kLag MFMAs after its issue, behind or ahead of the stores
        const double r = run<16, 0, 8, 2>(out, cyc, h, g, iters);
        line<16, 0, 8, 2>(out, cyc, h, g, iters, 0);
        line<16, 1, 8, 2>(out, cyc, h, g, iters, r);
        line<16, 2, 8, 2>(out, cyc, h, g, iters, r);
        line<16, 4, 8, 2>(out, cyc, h, g, iters, r);
        line<16, 1, 8, 3>(out, cyc, h, g, iters, r);
        line<16, 2, 8, 3>(out, cyc, h, g, iters, r);
        line<16, 4, 8, 3>(out, cyc, h, g, iters, r);
    }
    for (int g : {1, grid}) {
        sweep<8>(out, cyc, h, g, iters);
        sweep<16>(out, cyc, h, g, iters);
        sweep<32>(out, cyc, h, g, iters);
    }
    CK(hipFree(out));
    CK(hipFree(cyc));
    std::free(h);
    return 0;
}

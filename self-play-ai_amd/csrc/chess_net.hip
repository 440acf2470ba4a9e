// chess_net.hip — chess policy/value ResNet forward (model/chess.rs:48-77,
// model/mod.rs:152-184) as ONE fused HIP kernel per evaluation batch.
//
// Net: stem conv3x3 19->256 + BN + ReLU; `blocks` residual blocks
// relu(x + BN(conv(relu(BN(conv(x)))))) at 256 channels; policy head conv1x1
// 256->256 + ReLU + conv1x1 256->73 (flattened NCHW: index = ch*64 + cell, the
// Policy layout of chess.rs:252-257); value head conv1x1 256->1 + ReLU +
// linear 64->256 + ReLU + linear 256->1 + tanh.  BN (eval) folded into the convs.
//
// MI355X design:
//  * one workgroup = 4 waves (one per SIMD) = 2 positions' whole forward.  Both boards' 128
//    cells x 256 channels stay in LDS for every layer (two bf16 buffers of
//    64 KiB: layer input and output; the residual is the input buffer, updated
//    in place), so activations never touch HBM; only weights stream (L2).
//  * every conv is an implicit GEMM on v_mfma_f32_16x16x32_bf16, D[co][cell] =
//    W[co][k] X[k][cell], k = tap*256 + ci.  Wave w owns co tiles 4w..4w+3 (64
//    output channels) over all 8 cell tiles (two boards), so a k-step is 32
//    MFMAs on 4 weight fragments (global, pre-packed in exact fragment order:
//    one coalesced 1 KiB load each, issued 3 k-steps ahead and pinned there by
//    a scheduling barrier) and 8 activation fragments (ds_read_b128, immediate
//    offsets).
//    A whole board is inside the workgroup, so a 3x3 tap is a row shift;
//    off-board taps read a zero row.
//  * LDS rows hold [cell][256 ch] bf16 at a 544-B pitch: for every tap shift the
//    16 lanes of each ds_read_b128 lane group hit 16 distinct bank quads
//    (row_chunk), and a k-step's read is the tap's row base + a constant.
//  * bias is the first MFMA's C operand; epilogues fuse ReLU and the residual.
// Algorithmic FLOPs per position at 20 blocks: 3,036,348,928.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "chess_engine.h"
#include "philox.h"

namespace spai {
namespace chess {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

constexpr int kHid = 256;
#ifndef SPAI_CHESS_WAVES
#define SPAI_CHESS_WAVES 4   // 8 (two per SIMD) measured equal: 2.101 vs 2.101 ms
#endif
constexpr int kWaves = SPAI_CHESS_WAVES;     // 4: one wave per SIMD; 8: two
constexpr int kCPW = 16 / kWaves;             // co tiles (of 16 channels) per wave
constexpr int kThreads = 64 * kWaves;
constexpr int kPos = 2;                       // positions per workgroup
constexpr int kRows = kPos * 64;              // LDS rows (cells)
constexpr int kRowB = kHid * 2;               // 512 B of channels per row
constexpr int kStride = kRowB + 32;           // 544 B row pitch (see row_chunk)
constexpr int kBufA = 0;
constexpr int kBufB = kRows * kStride;        // 69632
constexpr int kZero = 2 * kRows * kStride;    // 139264: zeros for off-board taps
constexpr int kZeroB = 768;
constexpr int kSmem = kZero + kZeroB;         // 140032 B
constexpr int kCT = kHid / 16;                // 16 co tiles
constexpr int kPolCT = 5;                     // 73 policy channels -> 80
constexpr int kFrag = 64;                     // uint4 per fragment (1 KiB)
constexpr int kMaxBlocks = 40;

struct NetW {
    const uint4 *w_stem, *w_res, *w_p1, *w_p2;
    const float *b_stem, *b_res, *b_p1, *b_p2;
    const float *v_w, *v_b, *l1_w, *l1_b, *l2_w, *l2_b;
    int blocks;
};

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint32_t pack_relu_bf16x2(float a, float b) {
    const i16x2 h = __builtin_bit_cast(i16x2, __builtin_convertvector((f32x2){a, b}, bf16x2));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, (i16x2){0, 0}));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// byte offset of 16-B chunk `c` (channels 8c..8c+7) of row `v` inside a buffer.
// The 544-B pitch puts row v's chunk c in bank quad (2v + c) mod 16: the 16 lanes
// of a ds_read_b128 lane group (two k-groups q of opposite parity, 8 consecutive
// rows each, for any tap shift) land in 16 distinct bank quads, and a k-step's
// address is the tap's row base plus a compile-time offset.
__device__ __forceinline__ int row_chunk(int v, int c) { return v * kStride + (c << 4); }

// Implicit-GEMM conv over the LDS buffer at IN: TAPS (9 = 3x3 pad 1, 1 = 1x1)
// x CB channel blocks of 32.  acc[c][t]: co tile 4*wave + c, cell tile t.
// Software pipeline (fully unrolled, so every ring slot is static): weight
// fragments (global/L2) DA-1 k-steps ahead, activation fragments (LDS) one
// k-step ahead; the first k-step takes the bias as its C operand.
#ifndef SPAI_CHESS_DA
#define SPAI_CHESS_DA 4   // weight ring: 3 k-steps ahead (measured: 2 -> 3.40 ms, 8 -> 2.19 ms at 4 waves)
#endif
#ifndef SPAI_CHESS_DB
#define SPAI_CHESS_DB 2
#endif
#ifndef SPAI_CHESS_SCHED
#define SPAI_CHESS_SCHED 0
#endif
#ifndef SPAI_CHESS_PIN
#define SPAI_CHESS_PIN 1
#endif
#ifndef SPAI_CHESS_TAP_UNROLL
#define SPAI_CHESS_TAP_UNROLL 9   // taps per iteration of the tap loop (9: fully unrolled, 1.92 vs 1.99 ms)
#endif
// SPAI_CHESS_PREFETCH (experiment): at a conv's start every wave loads its
// share of the NEXT conv's weight fragments (the 128 waves of an XCD split the
// layer's 72 x 16 fragments), so that layer's ring loads hit the XCD's L2
// instead of going to the Infinity Cache one k-step window ahead; the loads'
// values feed a never-taken store, so they are waited for once, early in this conv.
template <int TAPS, int CB, int NT>
__device__ __forceinline__ void conv(const uint8_t *smem, int in, const uint4 *__restrict__ w,
                                     const float *__restrict__ bias, int wave, int lane, f32x4 (&acc)[kCPW][NT],
                                     const uint4 *__restrict__ wnext = nullptr, float *__restrict__ sink = nullptr) {
    constexpr int DA = SPAI_CHESS_DA;
#ifdef SPAI_CHESS_PREFETCH
    uint32_t pf = 0;
    if (wnext) {
        const int g = (int)((blockIdx.x >> 3) & 31u) * kWaves + wave;   // blocks b, b + 8, ... share an XCD
#pragma unroll
        for (int j = 0; j < (72 * kCT + 127) / 128; ++j) {
            const int f = g + 128 * j;
            if (f < 72 * kCT) pf ^= wnext[(size_t)f * kFrag + lane].x;
        }
    }
#else
    (void)wnext;
    (void)sink;
#endif
    const int q = lane >> 4, col = lane & 15;
    f32x4 bv[kCPW];
#pragma unroll
    for (int c = 0; c < kCPW; ++c) {
        const float4 b = *(const float4 *)(bias + (kCPW * wave + c) * 16 + 4 * q);
        bv[c] = f32x4{b.x, b.y, b.z, b.w};
    }
    const uint4 *wl = w + (size_t)(kCPW * wave) * kFrag + lane;
    constexpr int KS = TAPS * CB;
    constexpr int DB = (CB % SPAI_CHESS_DB == 0) ? SPAI_CHESS_DB : 2;
    uint4 A[DA][kCPW], B[DB > 2 ? DB : 2][NT];
    int rowoff[NT];
    auto geo = [&](int tap) {
        const int dy = TAPS == 9 ? tap / 3 - 1 : 0, dx = TAPS == 9 ? tap % 3 - 1 : 0;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int cell = (t & 3) * 16 + col;
            const int y = (cell >> 3) + dy, x = (cell & 7) + dx;
            const int v = (t >> 2) * 64 + y * 8 + x;
            const bool ok = (unsigned)y < 8u && (unsigned)x < 8u;
            // an off-board tap reads zeros in the bank quad its row would use
            rowoff[t] = (ok ? in + v * kStride : kZero + ((v & 7) << 5)) + (q << 4);
        }
    };
    auto load_a = [&](int ks, uint4 (&a)[kCPW]) {
#pragma unroll
        for (int c = 0; c < kCPW; ++c) a[c] = wl[((size_t)ks * kCT + c) * kFrag];
    };
    auto load_b = [&](int ks, uint4 (&b)[NT]) {
        const int cb = ks % CB;
#pragma unroll
        for (int t = 0; t < NT; ++t) b[t] = *(const uint4 *)(smem + rowoff[t] + (cb << 6));
    };
#pragma unroll
    for (int c = 0; c < kCPW; ++c)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[c][t] = bv[c];
#pragma unroll
    for (int k = 0; k < DA - 1; ++k)
        if (k < KS) load_a(k, A[k]);
    geo(0);
    if constexpr (CB % DA == 0 && CB % DB == 0) {
        // taps as a runtime loop, channel blocks unrolled: ring slots stay static
#pragma unroll
        for (int k = 0; k < DB - 1; ++k) load_b(k, B[k]);
#pragma unroll SPAI_CHESS_TAP_UNROLL
        for (int tap = 0; tap < TAPS; ++tap) {
#pragma unroll
            for (int cb = 0; cb < CB; ++cb) {
                const int ks = tap * CB + cb;
                if (ks + DA - 1 < KS) load_a(ks + DA - 1, A[(cb + DA - 1) % DA]);
                const int kb = cb + DB - 1;   // next activation k-step to fetch
                if (kb < CB) {
                    load_b(kb, B[kb % DB]);
                } else if (tap + 1 < TAPS) {
                    if (kb == CB) geo(tap + 1);   // every fetch of this tap is already issued
                    load_b(kb - CB, B[kb % DB]);
                }
#if SPAI_CHESS_PIN
                // keep the prefetches here: the scheduler would otherwise sink them
                // next to their MFMAs and expose the full L2 latency every k-step
                __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
                for (int c = 0; c < kCPW; ++c)
#pragma unroll
                    for (int t = 0; t < NT; ++t)
                        acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[cb % DA][c]),
                                                                            as_bf16x8(B[cb % DB][t]), acc[c][t], 0, 0, 0);
#if SPAI_CHESS_SCHED
                // issue order: each MFMA followed by up to one LDS read, one weight load, two VALU
#pragma unroll
                for (int i = 0; i < kCPW * 8; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    if (i < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    if (i < 4) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
#endif
            }
        }
    } else {
        load_b(0, B[0]);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + DA - 1 < KS) load_a(ks + DA - 1, A[(ks + DA - 1) % DA]);
            if (ks + 1 < KS) {
                if ((ks + 1) % CB == 0) geo((ks + 1) / CB);
                load_b(ks + 1, B[(ks + 1) & 1]);
            }
#pragma unroll
            for (int c = 0; c < kCPW; ++c)
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[ks % DA][c]),
                                                                        as_bf16x8(B[ks & 1][t]), acc[c][t], 0, 0, 0);
        }
    }
#ifdef SPAI_CHESS_PREFETCH
    if (wnext && pf == 0x9E3779B9u && acc[0][0][0] == -1234.5678f) sink[lane] = (float)pf;   // never taken
#endif
}

// relu(acc [+ residual at OUT]) -> bf16 at OUT (in place over the residual)
template <bool RES, int NT>
__device__ __forceinline__ void epilogue(uint8_t *smem, int out, int wave, int lane, const f32x4 (&acc)[kCPW][NT]) {
    const int q = lane >> 4, col = lane & 15;
#pragma unroll
    for (int c = 0; c < kCPW; ++c)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int v = (t >> 2) * 64 + (t & 3) * 16 + col;
            const int chunk = (kCPW * wave + c) * 2 + (q >> 1);
            uint2 *p = (uint2 *)(smem + out + row_chunk(v, chunk) + (q & 1) * 8);
            f32x4 a = acc[c][t];
            if (RES) {
                const uint2 r = *p;
                a[0] += bf_lo(r.x);
                a[1] += bf_hi(r.x);
                a[2] += bf_lo(r.y);
                a[3] += bf_hi(r.y);
            }
            *p = make_uint2(pack_relu_bf16x2(a[0], a[1]), pack_relu_bf16x2(a[2], a[3]));
        }
}

// Residual add as one identity MFMA per (co tile, cell tile): acc += I * x with
// B = the (untapped) fragment of the 32-channel block holding the co tile, read
// from the conv's output buffer (which still holds x), and A selecting the co
// tile's 16 channels.  One exact product plus zeros and a single fp32 rounding:
// the value of the VALU add it replaces.  Wave w owns co tiles 4w..4w+3, i.e.
// whole 32-channel blocks, so no other wave writes them meanwhile.
#ifndef SPAI_CHESS_RES_MFMA
#define SPAI_CHESS_RES_MFMA 1
#endif
template <int NT>
__device__ __forceinline__ void residual_mfma(const uint8_t *smem, int out, int wave, int lane,
                                              f32x4 (&acc)[kCPW][NT]) {
    const int m = lane & 15, q = lane >> 4, col = lane & 15;
    uint4 id[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = 16 * h + m - 8 * q;   // this lane's k slot that holds the 1, if any
        uint32_t w[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = j == 2 * e ? 0x3F80u : j == 2 * e + 1 ? 0x3F800000u : 0u;
        id[h] = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int c = 0; c < kCPW; ++c) {
        const int ct = kCPW * wave + c;
        uint4 b[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int v = (t >> 2) * 64 + (t & 3) * 16 + col;
            b[t] = *(const uint4 *)(smem + out + row_chunk(v, (ct >> 1) * 4 + q));
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
            acc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(id[ct & 1]), as_bf16x8(b[t]), acc[c][t], 0,
                                                               0, 0);
    }
}

// the forward of P positions (slots slot0 .. slot0+P-1) by one workgroup
template <int P>
__device__ __forceinline__ void forward_body(uint8_t *smem, uint32_t count, uint32_t slot0,
                                             const uint16_t *__restrict__ x, const NetW &W, float *__restrict__ logits,
                                             float *__restrict__ value, int tid_in, int lane_in, int wave) {
    constexpr int NT = 4 * P, ROWS = 64 * P, TPW = NT / kWaves;
    // hide the thread id from loop-invariant code motion: the per-lane addresses of
    // every layer hoisted out of the pass loop stayed live across it and were
    // spilled to scratch (~100 8-byte slots stored per wave and launch, reloaded
    // every pass); recomputed per pass they cost a few VALU
    int tid = tid_in;
    asm volatile("" : "+v"(tid));
    tid &= kThreads - 1;
    const int lane = tid & 63;
    (void)lane_in;
    // stage the input planes (bf16 [cell][32]) into buffer B, chunks 0..3 of each row; zero row
    for (int i = tid; i < ROWS * 4; i += kThreads) {
        const int v = i >> 2, c = i & 3;
        const uint32_t slot = slot0 + (v >> 6);
        uint4 d = make_uint4(0, 0, 0, 0);
        if (slot < count) d = *(const uint4 *)(x + ((size_t)slot * 64 + (v & 63)) * kInCh + c * 8);
        *(uint4 *)(smem + kBufB + row_chunk(v, c)) = d;
    }
    for (int i = tid; i < kZeroB / 16; i += kThreads) *(uint4 *)(smem + kZero + i * 16) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    f32x4 acc[kCPW][NT];
    conv<9, 1, NT>(smem, kBufB, W.w_stem, W.b_stem, wave, lane, acc);
    epilogue<false, NT>(smem, kBufA, wave, lane, acc);
    __syncthreads();
    for (int l = 0; l < W.blocks; ++l) {
#ifdef SPAI_CHESS_EXP_FIXW   // timing experiment (wrong results): every block reads block 0's weights (L2-resident)
        const size_t l1 = 0, l2 = 1;
#else
        const size_t l1 = 2 * l, l2 = 2 * l + 1;
#endif
        conv<9, 8, NT>(smem, kBufA, W.w_res + l1 * 72 * kCT * kFrag, W.b_res + l1 * kHid, wave, lane, acc,
                       W.w_res + l2 * 72 * kCT * kFrag, value);
        epilogue<false, NT>(smem, kBufB, wave, lane, acc);
        __syncthreads();
        conv<9, 8, NT>(smem, kBufB, W.w_res + l2 * 72 * kCT * kFrag, W.b_res + l2 * kHid, wave, lane, acc,
                       l + 1 < W.blocks ? W.w_res + (l2 + 1) * 72 * kCT * kFrag : nullptr, value);
        if (SPAI_CHESS_RES_MFMA) {
            residual_mfma<NT>(smem, kBufA, wave, lane, acc);
            epilogue<false, NT>(smem, kBufA, wave, lane, acc);
        } else {
            epilogue<true, NT>(smem, kBufA, wave, lane, acc);
        }
        __syncthreads();
    }
    // ---- policy head: conv1x1 256->256 + ReLU -> buffer B
    conv<1, 8, NT>(smem, kBufA, W.w_p1, W.b_p1, wave, lane, acc);
    epilogue<false, NT>(smem, kBufB, wave, lane, acc);
    // ---- value head (VALU, fp32): conv1x1 256->1 + ReLU per cell, from buffer A
    __syncthreads();
    {
        // conv1x1 256->256 output in B; torso output still in A.  Value conv
        // over A: 2 threads per cell, 128 channels each (the same reduction
        // order whatever P is, so a position's value never depends on its batch).
        constexpr int TPC = 2, CPT = 32 / TPC;
        const int v = tid / TPC, part = tid % TPC;
        float s = 0.f;
#pragma unroll 4
        for (int k = 0; k < CPT; ++k) {
            if (v >= ROWS) break;
            const int c = part * CPT + k;
            const uint4 d = *(const uint4 *)(smem + kBufA + row_chunk(v, c));
            const float4 w0 = *(const float4 *)(W.v_w + c * 8), w1 = *(const float4 *)(W.v_w + c * 8 + 4);
            s += bf_lo(d.x) * w0.x + bf_hi(d.x) * w0.y + bf_lo(d.y) * w0.z + bf_hi(d.y) * w0.w;
            s += bf_lo(d.z) * w1.x + bf_hi(d.z) * w1.y + bf_lo(d.w) * w1.z + bf_hi(d.w) * w1.w;
        }
#pragma unroll
        for (int o = 1; o < TPC; o <<= 1) s += __shfl_xor(s, o, 64);
        __syncthreads();   // every wave is done reading A (conv1x1 above, value conv here)
        float *vcell = (float *)(smem + kBufA);           // [128] value-conv features
        float *hid = (float *)(smem + kBufA + 1024);      // [2][256]
        float *red = (float *)(smem + kBufA + 4096);      // [2][4] wave partials
        if (part == 0 && v < ROWS) vcell[v] = fmaxf(s + W.v_b[0], 0.f);
        __syncthreads();
        {
            const int j = tid & 255;   // linear 64 -> 256 + ReLU, then the 256 -> 1 partial
            const float *wr = W.l1_w + (size_t)j * 64;
            for (int sp = tid >> 8; sp < P; sp += kThreads / 256) {
                float h = W.l1_b[j];
                for (int c = 0; c < 64; ++c) h += wr[c] * vcell[sp * 64 + c];
                h = fmaxf(h, 0.f);
                hid[sp * 256 + j] = h;
                float pr = W.l2_w[j] * h;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) pr += __shfl_xor(pr, o, 64);
                if (lane == 0) red[sp * 4 + (j >> 6)] = pr;
            }
        }
        __syncthreads();
        if (tid < P) {
            const uint32_t slot = slot0 + tid;
            const float *r = red + 4 * tid;
            if (slot < count) value[slot] = tanhf(W.l2_b[0] + ((r[0] + r[1]) + (r[2] + r[3])));
        }
    }
    // ---- policy conv1x1 256->73 over B -> logits [slot][ch*64 + cell]
    {
        const int q = lane >> 4, col = lane & 15;
        f32x4 pa[kPolCT][TPW];
#pragma unroll
        for (int c = 0; c < kPolCT; ++c) {
            const float4 b = *(const float4 *)(W.b_p2 + c * 16 + 4 * q);
#pragma unroll
            for (int u = 0; u < TPW; ++u) pa[c][u] = f32x4{b.x, b.y, b.z, b.w};
        }
#pragma unroll 2
        for (int ks = 0; ks < 8; ++ks) {
            uint4 a[kPolCT], b[TPW];
#pragma unroll
            for (int c = 0; c < kPolCT; ++c) a[c] = W.w_p2[((size_t)ks * kPolCT + c) * kFrag + lane];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int t = TPW * wave + u;
                const int v = (t >> 2) * 64 + (t & 3) * 16 + col;
                b[u] = *(const uint4 *)(smem + kBufB + row_chunk(v, 4 * ks + q));
            }
#pragma unroll
            for (int c = 0; c < kPolCT; ++c)
#pragma unroll
                for (int u = 0; u < TPW; ++u)
                    pa[c][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[c]), as_bf16x8(b[u]), pa[c][u], 0,
                                                                       0, 0);
        }
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            const int t = TPW * wave + u;
            const uint32_t slot = slot0 + (t >> 2);
            const int cell = (t & 3) * 16 + col;
            if (slot < count) {
                float *lg = logits + (size_t)slot * kPolicy;
#pragma unroll
                for (int c = 0; c < kPolCT; ++c)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int co = c * 16 + 4 * q + i;
                        if (co < 73) lg[co * 64 + cell] = pa[c][u][i];
                    }
            }
        }
    }
}

// Up to n_cu workgroups, one per CU (140 KiB of LDS each).  With no more
// positions than CUs, one position per workgroup (P = 1).  Otherwise, with
// m = ceil(count / n_cu) positions on the busiest CU:
//  * m even: P = 2 passes over slots 2w, 2w + 2 n_cu, ... (m / 2 passes);
//  * m odd: the count is split evenly (q or q + 1 positions per workgroup),
//    run as P = 2 passes plus one P = 1 pass: 600 positions take a P = 2 and a
//    P = 1 pass instead of two P = 2 passes (+25 % at 520-700 positions;
//    profiles/r02/chess/split_ab.txt).  For even m the even split measured
//    slower (-7..-11 %: more workgroups stream the weights for no fewer passes).
// A position's results do not depend on P or on its workgroup.
__global__ void __launch_bounds__(kThreads, 1)
    k_chess_forward(const uint32_t *__restrict__ d_count, uint32_t max_n, uint32_t n_cu,
                    const uint16_t *__restrict__ x, NetW W, float *__restrict__ logits, float *__restrict__ value) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kSmem];
    const uint32_t count = d_count ? min(*d_count, max_n) : max_n;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t w = blockIdx.x;
    if (count <= n_cu) {
        if (w >= count) return;
        forward_body<1>(smem, count, w, x, W, logits, value, tid, lane, wave);
        return;
    }
    if (w >= n_cu) return;
    const uint32_t m = (count + n_cu - 1) / n_cu;
    if ((m & 1) == 0) {
        for (uint32_t slot0 = 2 * w; slot0 < count; slot0 += 2 * n_cu) {
            forward_body<2>(smem, count, slot0, x, W, logits, value, tid, lane, wave);
            __syncthreads();   // the next pass restages the LDS
        }
        return;
    }
    const uint32_t q = count / n_cu, r = count % n_cu;
    uint32_t lo = w * q + min(w, r);
    const uint32_t hi = lo + q + (w < r ? 1u : 0u);
    for (; lo + 2 <= hi; lo += 2) {
        forward_body<2>(smem, count, lo, x, W, logits, value, tid, lane, wave);
        __syncthreads();
    }
    if (lo < hi) forward_body<1>(smem, count, lo, x, W, logits, value, tid, lane, wave);
}

// f32 [n][19][8][8] -> bf16 [n][64][kInCh]
__global__ void k_pack_input(const float *__restrict__ x, uint32_t n, uint16_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * 64) return;
    const uint32_t s = i >> 6, cell = i & 63;
    uint16_t v[kInCh];
#pragma unroll
    for (int c = 0; c < kInCh; ++c) {
        const float f = c < kPlanes ? x[((size_t)s * kPlanes + c) * 64 + cell] : 0.f;
        v[c] = __builtin_bit_cast(uint16_t, (__bf16)f);
    }
#pragma unroll
    for (int c = 0; c < kInCh; c += 8)
        *(uint4 *)(out + (size_t)i * kInCh + c) = *(const uint4 *)(v + c);
}

// ---------------------------------------------------------------- host packing
uint16_t f2bf(float f) {   // round to nearest even
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)((u >> 16) | ((u & 0xFFFF) ? 0x40 : 0));
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// w [co][ci][k][k] (k = 1 or 3), BN scale per co (or 1) -> A fragments
// [ks = tap*CB + cb][ct][lane][8] with ci padded to CB*32 and co to CT*16
void pack_conv(const float *w, const std::vector<double> &scale, int co, int ci, int k, int CB, int CT,
               std::vector<uint16_t> &out) {
    const int taps = k * k;
    const size_t base = out.size();
    out.resize(base + (size_t)taps * CB * CT * 64 * 8, 0);
    for (int tap = 0; tap < taps; ++tap)
        for (int cb = 0; cb < CB; ++cb)
            for (int ct = 0; ct < CT; ++ct)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 8; ++j) {
                        const int o = ct * 16 + (l & 15), i = cb * 32 + (l >> 4) * 8 + j;
                        float v = 0.f;
                        if (o < co && i < ci) v = (float)((double)w[((size_t)o * ci + i) * taps + tap] * scale[o]);
                        out[base + ((((size_t)(tap * CB + cb) * CT + ct) * 64 + l) * 8 + j)] = f2bf(v);
                    }
}

float philox_unit(uint64_t seed, uint32_t tensor, uint64_t idx) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), tensor, 0xC4E55u};
    uint32_t o[4];
    philox4x32(ctr, key, o);
    return (float)(o[0] >> 8) * (1.0f / 16777216.0f);
}

}  // namespace

size_t net_num_params(int blocks) {
    auto conv = [](size_t ci, size_t co, size_t k) { return co * ci * k * k + co; };
    size_t n = conv(19, kHid, 3) + 4 * kHid;
    n += (size_t)blocks * 2 * (conv(kHid, kHid, 3) + 4 * kHid);
    n += conv(kHid, 256, 1) + conv(256, 73, 1);
    n += conv(kHid, 1, 1) + (64 * 256 + 256) + (256 + 1);
    return n;
}

// tch 0.13 default init (as spai_net_init_params): conv / linear weights
// Kaiming-uniform bound sqrt(6 / fan_in), conv bias 0, linear bias
// U(+-1/sqrt(fan_in)), BN gamma U(0,1), beta 0, running mean 0, var 1.
void net_init_params(int blocks, uint64_t seed, float *params) {
    uint32_t t = 0;
    float *p = params;
    auto uni = [&](size_t n, float lo, float hi) {
        for (size_t i = 0; i < n; ++i) p[i] = lo + (hi - lo) * philox_unit(seed, t, i);
        p += n;
        ++t;
    };
    auto cst = [&](size_t n, float v) {
        for (size_t i = 0; i < n; ++i) p[i] = v;
        p += n;
        ++t;
    };
    auto conv = [&](int ci, int co, int k) {
        const float b = (float)std::sqrt(6.0 / (double)(ci * k * k));
        uni((size_t)co * ci * k * k, -b, b);
        cst(co, 0.f);
    };
    auto bn = [&](int c) {
        uni(c, 0.f, 1.f);
        cst(c, 0.f);
        cst(c, 0.f);
        cst(c, 1.f);
    };
    auto lin = [&](int in, int out) {
        const float b = (float)std::sqrt(6.0 / (double)in), bb = (float)(1.0 / std::sqrt((double)in));
        uni((size_t)out * in, -b, b);
        uni(out, -bb, bb);
    };
    conv(19, kHid, 3);
    bn(kHid);
    for (int i = 0; i < blocks; ++i) {
        conv(kHid, kHid, 3);
        bn(kHid);
        conv(kHid, kHid, 3);
        bn(kHid);
    }
    conv(kHid, 256, 1);
    conv(256, 73, 1);
    conv(kHid, 1, 1);
    lin(64, 256);
    lin(256, 1);
}

int net_create(spai_chess *e, int blocks, const float *params, size_t n, spai_chess_net **out) {
    SPAI_CHECK(blocks >= 0 && blocks <= kMaxBlocks, SPAI_ERR_UNSUPPORTED, "chess net: 0..%d blocks (got %d)",
               kMaxBlocks, blocks);
    SPAI_CHECK(params && n == net_num_params(blocks), SPAI_ERR_INVALID, "expected %zu params, got %zu",
               net_num_params(blocks), n);
    const float *p = params;
    std::vector<uint16_t> w_stem, w_res, w_p1, w_p2;
    std::vector<float> b_stem, b_res, b_p1, b_p2;
    // conv + BN (eval): w' = w * g / sqrt(var + eps), b' = (b - mu) * g / sqrt(var + eps) + beta
    auto conv_bn = [&](int ci, std::vector<uint16_t> &wout, std::vector<float> &bout, int CB) {
        const float *w = p, *b = p + (size_t)kHid * ci * 9, *bn = b + kHid;
        p = bn + 4 * kHid;
        std::vector<double> sc(kHid);
        for (int o = 0; o < kHid; ++o) {
            sc[o] = (double)bn[o] / std::sqrt((double)bn[3 * kHid + o] + 1e-5);
            bout.push_back((float)(((double)b[o] - (double)bn[2 * kHid + o]) * sc[o] + (double)bn[kHid + o]));
        }
        pack_conv(w, sc, kHid, ci, 3, CB, kCT, wout);
    };
    conv_bn(19, w_stem, b_stem, 1);
    for (int i = 0; i < 2 * blocks; ++i) conv_bn(kHid, w_res, b_res, 8);
    {
        std::vector<double> one(256, 1.0);
        pack_conv(p, one, 256, kHid, 1, 8, kCT, w_p1);
        p += 256 * kHid;
        b_p1.assign(p, p + 256);
        p += 256;
        pack_conv(p, one, 73, 256, 1, 8, kPolCT, w_p2);
        p += 73 * 256;
        b_p2.assign(80, 0.f);
        std::copy(p, p + 73, b_p2.begin());
        p += 73;
    }
    std::vector<float> v_w(p, p + kHid), v_b(p + kHid, p + kHid + 1);
    p += kHid + 1;
    std::vector<float> l1_w(p, p + 64 * 256), l1_b(p + 64 * 256, p + 64 * 256 + 256);
    p += 64 * 256 + 256;
    std::vector<float> l2_w(p, p + 256), l2_b(p + 256, p + 257);
    p += 257;
    SPAI_CHECK((size_t)(p - params) == n, SPAI_ERR_INVALID, "parameter walk mismatch");
    if (blocks == 0) w_res.assign(8, 0), b_res.assign(4, 0.f);   // keep the buffers non-empty

    spai_chess_net *net = new spai_chess_net();
    net->eng = e;
    net->blocks = blocks;
    auto up16 = [&](DevBuf<uint16_t> &d, const std::vector<uint16_t> &h) -> int {
        SPAI_TRY(d.alloc(h.size()));
        SPAI_HIP(hipMemcpy(d.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        return SPAI_OK;
    };
    auto upf = [&](DevBuf<float> &d, const std::vector<float> &h) -> int {
        SPAI_TRY(d.alloc(h.size()));
        SPAI_HIP(hipMemcpy(d.p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        return SPAI_OK;
    };
    int rc = SPAI_OK;
    if (rc == SPAI_OK) rc = up16(net->w_stem, w_stem);
    if (rc == SPAI_OK) rc = up16(net->w_res, w_res);
    if (rc == SPAI_OK) rc = up16(net->w_p1, w_p1);
    if (rc == SPAI_OK) rc = up16(net->w_p2, w_p2);
    if (rc == SPAI_OK) rc = upf(net->b_stem, b_stem);
    if (rc == SPAI_OK) rc = upf(net->b_res, b_res);
    if (rc == SPAI_OK) rc = upf(net->b_p1, b_p1);
    if (rc == SPAI_OK) rc = upf(net->b_p2, b_p2);
    if (rc == SPAI_OK) rc = upf(net->v_w, v_w);
    if (rc == SPAI_OK) rc = upf(net->v_b, v_b);
    if (rc == SPAI_OK) rc = upf(net->l1_w, l1_w);
    if (rc == SPAI_OK) rc = upf(net->l1_b, l1_b);
    if (rc == SPAI_OK) rc = upf(net->l2_w, l2_w);
    if (rc == SPAI_OK) rc = upf(net->l2_b, l2_b);
    if (rc != SPAI_OK) {
        net_destroy(net);
        return rc;
    }
    *out = net;
    return SPAI_OK;
}

void net_destroy(spai_chess_net *net) {
    if (!net) return;
    for (auto *d : {&net->w_stem, &net->w_res, &net->w_p1, &net->w_p2, &net->io_x}) d->release();
    for (auto *d : {&net->b_stem, &net->b_res, &net->b_p1, &net->b_p2, &net->v_w, &net->v_b, &net->l1_w, &net->l1_b,
                    &net->l2_w, &net->l2_b, &net->io_logits, &net->io_value})
        d->release();
    net->io_count.release();
    delete net;
}

static NetW weights_of(const spai_chess_net *n) {
    NetW W;
    W.w_stem = (const uint4 *)n->w_stem.p;
    W.w_res = (const uint4 *)n->w_res.p;
    W.w_p1 = (const uint4 *)n->w_p1.p;
    W.w_p2 = (const uint4 *)n->w_p2.p;
    W.b_stem = n->b_stem.p;
    W.b_res = n->b_res.p;
    W.b_p1 = n->b_p1.p;
    W.b_p2 = n->b_p2.p;
    W.v_w = n->v_w.p;
    W.v_b = n->v_b.p;
    W.l1_w = n->l1_w.p;
    W.l1_b = n->l1_b.p;
    W.l2_w = n->l2_w.p;
    W.l2_b = n->l2_b.p;
    W.blocks = n->blocks;
    return W;
}

int net_eval(spai_chess_net *net, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint16_t *x,
             float *logits, float *value) {
    if (!max_n) return SPAI_OK;
    const uint32_t n_cu = (uint32_t)net->eng->n_cu;
    k_chess_forward<<<std::min(max_n, n_cu), kThreads, 0, st>>>(d_count, max_n, n_cu, x, weights_of(net), logits,
                                                               value);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

int net_forward_host(spai_chess_net *net, uint32_t n, const float *x, float *logits, float *value) {
    if (!n) return SPAI_OK;
    spai_chess *e = net->eng;
    if (net->io_cap < n) {
        SPAI_TRY(net->io_x.alloc((size_t)n * 64 * kInCh));
        SPAI_TRY(net->io_logits.alloc((size_t)n * kPolicy));
        SPAI_TRY(net->io_value.alloc(n));
        net->io_cap = n;
    }
    float *d_in = net->io_logits.p;   // f32 input staged in the logits buffer (n*1216 <= n*4672)
    SPAI_HIP(hipMemcpyAsync(d_in, x, sizeof(float) * n * kPlanes * 64, hipMemcpyHostToDevice, e->stream));
    k_pack_input<<<(n * 64 + 255) / 256, 256, 0, e->stream>>>(d_in, n, net->io_x.p);
    SPAI_HIP(hipGetLastError());
    SPAI_TRY(net_eval(net, e->stream, nullptr, n, net->io_x.p, net->io_logits.p, net->io_value.p));
    SPAI_HIP(hipMemcpyAsync(logits, net->io_logits.p, sizeof(float) * n * kPolicy, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(value, net->io_value.p, sizeof(float) * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

// Model::predict (model/mod.rs:36-98) over game slots [first, first+n): encode
// (with the slot's repetition count), forward, softmax, mask_invalid_actions,
// all on the device; only the priors and values cross to the host.
int net_predict(spai_chess_net *net, uint32_t first, uint32_t n, float *priors, float *values) {
    if (!n) return SPAI_OK;
    spai_chess *e = net->eng;
    SPAI_CHECK((uint64_t)first + n <= e->slots.n, SPAI_ERR_INVALID, "slots [%u, %u) out of range (%u)", first,
               first + n, e->slots.n);
    if (net->io_cap < n) {
        SPAI_TRY(net->io_x.alloc((size_t)n * 64 * kInCh));
        SPAI_TRY(net->io_logits.alloc((size_t)n * kPolicy));
        SPAI_TRY(net->io_value.alloc(n));
        net->io_cap = n;
    }
    float *d_enc = e->slots.f32.p, *d_pri = e->slots.f32b.p;
    SPAI_TRY(slots_encode_device(e, first, n, d_enc));
    k_pack_input<<<(n * 64 + 255) / 256, 256, 0, e->stream>>>(d_enc, n, net->io_x.p);
    SPAI_HIP(hipGetLastError());
    SPAI_TRY(net_eval(net, e->stream, nullptr, n, net->io_x.p, net->io_logits.p, net->io_value.p));
    SPAI_TRY(slots_softmax_mask_device(e, first, n, net->io_logits.p, d_pri));
    SPAI_HIP(hipMemcpyAsync(priors, d_pri, sizeof(float) * n * kPolicy, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(values, net->io_value.p, sizeof(float) * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

}  // namespace chess
}  // namespace spai

// learner.hip — the training step of the C4 policy/value ResNet on the device
// (SURVEY.md §8f.1): ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85)
// = Net::forward(x, train=true) (model/mod.rs:152-184, model/connect_four.rs:50-81),
// loss -(log_softmax(p)·π).sum()/B + MSE(v, z) (model/mod.rs:128-135), and
// tch's Adam::default() step (β1 0.9, β2 0.999, eps 1e-8, no weight decay,
// lr 1e-3; model/mod.rs:107).  BatchNorm runs in train mode: batch statistics
// over (B, 6, 7), running statistics updated with momentum 0.1 and the
// unbiased batch variance (tch/libtorch batch_norm semantics).
//
// Data-parallel learner: with a communicator set, the flat gradient is summed
// over ranks with RCCL (ncclAllReduce over xGMI) and scaled by 1/world before
// Adam, and the BN running statistics are averaged, so every rank holds the
// same parameters after every step.
//
// Layout: fp32 NCHW activations [B][C][42].  The convs (forward, data and
// weight gradients) run on the exact-f32 MFMA; every reduction has a fixed
// order and there are no float atomics, so a step is deterministic.
// Parameters, gradients and Adam moments share the flat construction-order
// layout of spai_net_create (conv w, b, BN γ, β, μ, σ²; linears w, b).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "spai_internal.h"

namespace spai {
namespace {

constexpr int kCells = 42, kRows = 6, kCols = 7;
constexpr int kPad = 72;          // (6+2) x (7+2) zero-padded plane
constexpr int kPlane = 73;        // its LDS stride (odd, so channels spread over the banks)
constexpr int kThreads = 256;
constexpr int kTickDbias = 8;     // BatchNorm hand-off counters: tick[0..7] channel slices, tick[8] the bias-gradient merge
constexpr int kTicks = 16;

// ------------------------------------------------------------------ conv 3x3 on f32 MFMA
// Every conv of the step is a GEMM on v_mfma_f32_16x16x4_f32 (exact f32: an
// fmaf chain per output element; 157 TF/s peak, the f32 vector rate).  The
// reduction index is tap-major, k = tap * cinp + c (cinp = input channels
// rounded up to 4), so one k-step of 4 stays inside one tap and a lane's LDS
// address is its position's tap offset plus the channel.
//   forward:  out[b][n][p] = bias[n] + sum_k X[b][p][k] * Wk[k][n]
//   data grad: the same with X = dz and Wk built from the flipped, transposed
//              weights (w'[ci][co][8 - tap] = w[co][ci][tap])
//   weight grad: part[b][n][k] = sum_p dz[b][n][p] * X[b][p][k], then a
//              fixed-order sum over the batch (deterministic, no atomics)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline int round4(int c) { return (c + 3) & ~3; }
__host__ __device__ inline int round16(int c) { return (c + 15) & ~15; }

// tap offset inside a zero-padded 8 x 9 plane
__device__ __forceinline__ int tap_off(int tap) { return (tap / 3 - 1) * 9 + (tap % 3 - 1); }

// stage a sample's input planes [c][kPlane], zero-padded (rows -1..6, cols -1..7), channels >= cin zero.
// All of a thread's loads are issued before its LDS stores, so the staging pays
// one memory round trip, not one per element.
constexpr int kStageMax = (64 * kPad + kThreads - 1) / kThreads;   // 18 elements per thread at 64 channels
__device__ __forceinline__ void load_planes(const float *__restrict__ xb, int cin, int cinp, float (&v)[kStageMax]) {
    const int n = cinp * kPad;
#pragma unroll
    for (int j = 0; j < kStageMax; ++j) {
        const int i = threadIdx.x + j * kThreads;
        const int c = i / kPad, r = i - c * kPad, h = r / 9 - 1, x = r % 9 - 1;
        v[j] = (i < n && c < cin && h >= 0 && h < kRows && x >= 0 && x < kCols) ? xb[c * kCells + h * kCols + x] : 0.f;
    }
}
__device__ __forceinline__ void store_planes(const float (&v)[kStageMax], int cinp, float *xs) {
    const int n = cinp * kPad;
#pragma unroll
    for (int j = 0; j < kStageMax; ++j) {
        const int i = threadIdx.x + j * kThreads;
        if (i < n) xs[(i / kPad) * kPlane + i % kPad] = v[j];
    }
}
constexpr int kDzMax = (64 * 44 + kThreads - 1) / kThreads;
__device__ __forceinline__ void load_dz(const float *__restrict__ dzb, int cout, int coutp, float (&v)[kDzMax]) {
#pragma unroll
    for (int j = 0; j < kDzMax; ++j) {
        const int i = threadIdx.x + j * kThreads, n = i / 44, p = i - n * 44;
        v[j] = (i < coutp * 44 && n < cout && p < kCells) ? dzb[n * kCells + p] : 0.f;
    }
}
__device__ __forceinline__ void store_dz(const float (&v)[kDzMax], int coutp, float *ds) {
#pragma unroll
    for (int j = 0; j < kDzMax; ++j) {
        const int i = threadIdx.x + j * kThreads;
        if (i < coutp * 44) ds[i] = v[j];
    }
}
__device__ __forceinline__ void stage_planes(const float *__restrict__ xb, int cin, int cinp, float *xs) {
    float v[kStageMax];
    const int n = cinp * kPad;
#pragma unroll
    for (int j = 0; j < kStageMax; ++j) {
        const int i = threadIdx.x + j * kThreads;
        const int c = i / kPad, r = i - c * kPad, h = r / 9 - 1, x = r % 9 - 1;
        v[j] = (i < n && c < cin && h >= 0 && h < kRows && x >= 0 && x < kCols) ? xb[c * kCells + h * kCols + x] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kStageMax; ++j) {
        const int i = threadIdx.x + j * kThreads;
        if (i < n) xs[(i / kPad) * kPlane + i % kPad] = v[j];
    }
}

// stage_planes without per-element index math: thread t < 252 owns cell t % 42
// of channels t / 42 + 6j (source and LDS offsets are the thread's base plus
// immediates), thread t < 240 zeroes border cell t % 30 of channels t / 30 + 8j;
// the two sets are disjoint, so one barrier after the call covers both.
template <int CINP>
__device__ __forceinline__ void stage_planes_fast(const float *__restrict__ xb, int cin, float *xs) {
    const int t = threadIdx.x;
    if (t < 252) {
        const int c0 = t / kCells, cell = t - c0 * kCells;
        float *dst = xs + c0 * kPlane + (cell / kCols + 1) * 9 + cell % kCols + 1;
        const float *src = xb + t;
        float v[(CINP + 5) / 6];
#pragma unroll
        for (int j = 0; j < (CINP + 5) / 6; ++j) v[j] = c0 + 6 * j < cin ? src[252 * j] : 0.f;
#pragma unroll
        for (int j = 0; j < (CINP + 5) / 6; ++j)
            if (c0 + 6 * j < CINP) dst[6 * kPlane * j] = v[j];
    }
    if (t < 240) {
        const int c0 = t / 30, bi = t - c0 * 30;
        const int k = bi - 18;
        const int off = bi < 9 ? bi : bi < 18 ? 63 + bi - 9 : 9 * (1 + k / 2) + ((k & 1) ? 8 : 0);
        float *dst = xs + c0 * kPlane + off;
#pragma unroll
        for (int j = 0; j < (CINP + 7) / 8; ++j)
            if (c0 + 8 * j < CINP) dst[8 * kPlane * j] = 0.f;
    }
}

// Wk[(tap * cinp + c) * coutp + n]: forward Wk = w[n][c][tap]; data gradient Wk = w[c][n][8 - tap].
// Every conv's forward and data-gradient matrices are packed in one launch per
// step (blockIdx.y = entry of the table built at learner_create):
//   desc[8 y ..] = {param offset, cin, cout, cinp, coutp, dgrad, packed offset, 0}
constexpr int kPackDesc = 8;
// (it also zeroes the BatchNorm hand-off counters ahead of the step's convs)
__global__ void k_pack_all(const float *__restrict__ P, const uint32_t *__restrict__ desc, float *__restrict__ wall,
                           unsigned *__restrict__ tick) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < kTicks) tick[threadIdx.x] = 0u;
    const uint32_t *d = desc + kPackDesc * blockIdx.y;
    const int cin = (int)d[1], cout = (int)d[2], cinp = (int)d[3], coutp = (int)d[4];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 9 * cinp * coutp) return;
    const float *w = P + d[0];
    const int n = i % coutp, k = i / coutp, tap = k / cinp, c = k - tap * cinp;
    float v = 0.f;
    if (c < cin && n < cout)
        v = d[5] ? w[((size_t)c * cout + n) * 9 + (8 - tap)] : w[((size_t)n * cin + c) * 9 + tap];
    wall[d[6] + i] = v;
}

// BatchNorm (train mode) of a conv's input, applied while the consumer conv
// stages it (MODE & kBnIn).  The producer conv (MODE & kStatsOut) leaves
// per-(channel, sample) partials {sum, centred sum of squares} over the 42 cells,
// and the last of its workgroups to finish a channel slice merges that slice's B
// partials in a fixed order (Chan's pairwise variance: N var = sum_b Q_b + 42
// sum_b (m_b - mean)^2) into the batch mean / invstd and the running statistics
// (momentum, unbiased variance) -- what k_bn_fwd did in a kernel of its own.  The
// consumer stages a = relu(gamma (z - mean) invstd + beta [+ res]) from those
// 4 x 64 floats; its slice-0 workgroups write a (the backward's mask and
// weight-gradient input).
//
// The hand-off inside the producer launch (cdna_hip_programming.md §6 Guideline
// 16, counter form): every partial is stored write-through (sc1), each storing
// wave drains, the workgroup barrier, then one lane's agent-scope ticket add; the
// workgroup that draws the slice's last ticket reads the partials with sc1 loads
// and resets the counter.  The merge order is fixed, so the result does not
// depend on which workgroup finishes last.
constexpr int kBnIn = 1, kStatsOut = 2, kBnGrad = 4, kGradStats = 8;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
struct BnIn {
    float2 *part;                 // [c][B] producer partials (kStatsOut)
    const float *gamma, *beta;
    const float *res;             // residual (block input) [B][cin][42], or null
    float *a_out;                 // activations [B][cin][42]
    float *mean, *invstd, *run_mean, *run_var;
    int B;
    float eps, momentum;
    unsigned *tick;               // the producer's slice counters
};
constexpr int kBnStatFloats = 5 * 64;   // LDS: per input channel 4 (forward) or 5 (backward) statistics
constexpr int kLdsFlags = 4;            // LDS: the ticket results

__device__ __forceinline__ void store_part(float2 *p, float x, float y) {   // write-through (sc1)
    const unsigned long long u = ((unsigned long long)__float_as_uint(y) << 32) | __float_as_uint(x);
    __hip_atomic_store((gu64 *)p, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 load_part(const float2 *p) {   // sc1: no stale L1 copy
    const unsigned long long u = __hip_atomic_load((gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32)));
}
__device__ __forceinline__ void store_part1(float *p, float x) {
    __hip_atomic_store((gu32 *)p, __float_as_uint(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float load_part1(const float *p) {
    return __uint_as_float(__hip_atomic_load((gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// sum over the tpc consecutive lanes of a channel (butterfly: the same value on each)
__device__ __forceinline__ float chan_sum(float v, int tpc) {
    for (int o = 1; o < tpc; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// the merge of channels [c0, c0 + ch) of a forward producer (ch = 16 or 64: 16 or
// 4 lanes per channel, samples strided over them)
__device__ __forceinline__ void fin_bn_fwd(const BnIn &bo, int c0, int ch, int cout) {
    const int tpc = kThreads / ch, c = c0 + threadIdx.x / tpc, q = threadIdx.x % tpc, B = bo.B;
    const bool ok = c < cout;
    const float2 *pp = bo.part + (size_t)c * B;
    float s = 0.f;
    if (ok)
        for (int b = q; b < B; b += tpc) s += load_part(pp + b).x;
    s = chan_sum(s, tpc);
    const int n = B * kCells;
    const float mu = s / (float)n;
    float q2 = 0.f;
    if (ok)
        for (int b = q; b < B; b += tpc) {
            const float2 v = load_part(pp + b);
            const float d = v.x / (float)kCells - mu;
            q2 += v.y + (float)kCells * (d * d);
        }
    q2 = chan_sum(q2, tpc);
    if (q == 0 && ok) {
        const float var = q2 / (float)n;
        bo.mean[c] = mu;
        bo.invstd[c] = 1.0f / sqrtf(var + bo.eps);
        bo.run_mean[c] = (1.0f - bo.momentum) * bo.run_mean[c] + bo.momentum * mu;
        bo.run_var[c] = (1.0f - bo.momentum) * bo.run_var[c] +
                        bo.momentum * (n > 1 ? var * (float)n / (float)(n - 1) : var);
    }
}

// The backward of a = relu(bn(z) [+ res]) fused the same way (kBnGrad): the
// producer of da (the data gradient of the layer above, kGradStats) leaves per
// (channel, sample) partials {sum dy, sum dy xhat} with dy = da [a > 0] and
// xhat = (z - mean) invstd, and its slice's last workgroup merges them into
// dbeta = sum dy and dgamma = sum dy xhat; the consumer (this layer's
// data-gradient conv) stages dz = gamma invstd / N (N dy - dbeta - xhat dgamma)
// (k_bn_bwd's arithmetic), writing dz for the weight gradient and dy for the
// residual's skip path from its slice-0 workgroups.  Those also leave per-sample
// sums of dz, merged by their last workgroup into the conv bias gradient.
struct BnGrad {
    const float *a, *z, *mean, *invstd, *gamma;
    const float *dgamma, *dbeta;  // merged by the producer of da
    float *dz_out, *dy_out;       // [B][c][42] (dy_out may be null)
    float *db_part, *dbias;       // [c][B] per-sample dz sums; the conv bias gradient
    unsigned *tick;
    int B;
};
struct GradStats {                // the partials for the layer whose da this conv produces
    const float *a, *z, *mean, *invstd;
    float2 *part;                 // [c][B]
    float *dgamma, *dbeta;        // that layer's merged gradients
    unsigned *tick;
};

__device__ __forceinline__ void fin_bn_grad(const GradStats &gs, int c0, int ch, int cout, int B) {
    const int tpc = kThreads / ch, c = c0 + threadIdx.x / tpc, q = threadIdx.x % tpc;
    const bool ok = c < cout;
    const float2 *pp = gs.part + (size_t)c * B;
    float s1 = 0.f, s2 = 0.f;
    if (ok)
        for (int b = q; b < B; b += tpc) {
            const float2 v = load_part(pp + b);
            s1 += v.x;
            s2 += v.y;
        }
    s1 = chan_sum(s1, tpc);
    s2 = chan_sum(s2, tpc);
    if (q == 0 && ok) {
        gs.dbeta[c] = s1;
        gs.dgamma[c] = s2;
    }
}

__device__ __forceinline__ void bn_grad_stats(const BnGrad &bg, int cin, float *st) {
    const int c = threadIdx.x;
    if (c < cin) {
        const float is = bg.invstd[c];
        st[c] = bg.dbeta[c];
        st[64 + c] = bg.dgamma[c];
        st[128 + c] = bg.mean[c];
        st[192 + c] = is;
        st[256 + c] = bg.gamma[c] * is / (float)(bg.B * kCells);
    }
}

// stage dz of this layer (k_bn_bwd's arithmetic) from da, a, z; slice 0 writes dz and dy
template <int CINP>
__device__ __forceinline__ void stage_planes_dz(const float *__restrict__ dab, int cin, const BnGrad &bg, size_t boff,
                                                const float *st, float *xs) {
    const int t = threadIdx.x;
    if (t < 252) {
        const int c0 = t / kCells, cell = t - c0 * kCells;
        float *dst = xs + c0 * kPlane + (cell / kCols + 1) * 9 + cell % kCols + 1;
        constexpr int J = (CINP + 5) / 6;
        float vd[J], va[J], vz[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const bool ok = c0 + 6 * j < cin;
            vd[j] = ok ? dab[t + 252 * j] : 0.f;
            va[j] = ok ? bg.a[boff + t + 252 * j] : 0.f;
            vz[j] = ok ? bg.z[boff + t + 252 * j] : 0.f;
        }
        const bool w = blockIdx.y == 0;
        const float n = (float)(bg.B * kCells);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int c = c0 + 6 * j;
            if (c < CINP) {
                float v = 0.f;
                if (c < cin) {
                    const float d = va[j] > 0.f ? vd[j] : 0.f;
                    const float x = (vz[j] - st[128 + c]) * st[192 + c];
                    v = st[256 + c] * (n * d - st[c] - x * st[64 + c]);
                    if (w) {
                        bg.dz_out[boff + t + 252 * j] = v;
                        if (bg.dy_out) bg.dy_out[boff + t + 252 * j] = d;
                    }
                }
                dst[6 * kPlane * j] = v;
            }
        }
    }
    if (t < 240) {
        const int c0 = t / 30, bi = t - c0 * 30;
        const int k = bi - 18;
        const int off = bi < 9 ? bi : bi < 18 ? 63 + bi - 9 : 9 * (1 + k / 2) + ((k & 1) ? 8 : 0);
        float *dst = xs + c0 * kPlane + off;
#pragma unroll
        for (int j = 0; j < (CINP + 7) / 8; ++j)
            if (c0 + 8 * j < CINP) dst[8 * kPlane * j] = 0.f;
    }
}

// per-channel statistics of the input (merged by its producer) -> LDS st[4][64]
__device__ __forceinline__ void bn_in_stats(const BnIn &bn, int cin, float *st) {
    const int c = threadIdx.x;
    if (c < cin) {
        st[c] = bn.mean[c];
        st[64 + c] = bn.invstd[c];
        st[128 + c] = bn.gamma[c];
        st[192 + c] = bn.beta[c];
    }
}

// stage_planes_fast of relu(bn(z) [+ res]) (k_bn_fwd's arithmetic); a written by the slice-0 workgroups
template <int CINP>
__device__ __forceinline__ void stage_planes_bn(const float *__restrict__ zb, int cin, const BnIn &bn, size_t boff,
                                                const float *st, float *xs) {
    const int t = threadIdx.x;
    if (t < 252) {
        const int c0 = t / kCells, cell = t - c0 * kCells;
        float *dst = xs + c0 * kPlane + (cell / kCols + 1) * 9 + cell % kCols + 1;
        float v[(CINP + 5) / 6], r[(CINP + 5) / 6];
#pragma unroll
        for (int j = 0; j < (CINP + 5) / 6; ++j) {
            v[j] = c0 + 6 * j < cin ? zb[t + 252 * j] : 0.f;
            r[j] = bn.res && c0 + 6 * j < cin ? bn.res[boff + t + 252 * j] : 0.f;
        }
        const bool wa = bn.a_out && blockIdx.y == 0;
#pragma unroll
        for (int j = 0; j < (CINP + 5) / 6; ++j) {
            const int c = c0 + 6 * j;
            if (c < CINP) {
                float a = 0.f;
                if (c < cin) {
                    float y = st[128 + c] * ((v[j] - st[c]) * st[64 + c]) + st[192 + c];
                    if (bn.res) y += r[j];
                    a = fmaxf(y, 0.f);
                    if (wa) bn.a_out[boff + t + 252 * j] = a;
                }
                dst[6 * kPlane * j] = a;
            }
        }
    }
    if (t < 240) {
        const int c0 = t / 30, bi = t - c0 * 30;
        const int k = bi - 18;
        const int off = bi < 9 ? bi : bi < 18 ? 63 + bi - 9 : 9 * (1 + k / 2) + ((k & 1) ? 8 : 0);
        float *dst = xs + c0 * kPlane + off;
#pragma unroll
        for (int j = 0; j < (CINP + 7) / 8; ++j)
            if (c0 + 8 * j < CINP) dst[8 * kPlane * j] = 0.f;
    }
}

// workgroup (sample, slice): 3 position tiles (48 rows, 42 real) x NT channel
// tiles of output channels [16 NT slice, 16 NT (slice + 1)); wave w owns channel
// tile w % NT and K part w / NT (KS = 4/NT parts, summed in LDS in a fixed
// order).  CINP (input channels padded to 4) and NT are compile-time, so the
// k-loop unrolls fully and the weight loads of a whole part are in flight
// together.  coutp_all = the packed matrix's row length (all output channels).
template <int CINP, int NT, int MODE = 0, int MTS = 3>
__global__ __launch_bounds__(kThreads) void k_conv_mfma(const float *__restrict__ in, int cin,
                                                        const float *__restrict__ wk, const float *__restrict__ bias,
                                                        int cout, int coutp_all, float *__restrict__ out,
                                                        int accumulate, BnIn bn, BnIn bo, BnGrad bg, GradStats gs) {
    constexpr int KS = 4 / NT, CSN = CINP / 4, KSTEPS = 9 * CSN, PER = KSTEPS / KS;
    static_assert(4 % NT == 0 && KSTEPS % KS == 0, "4 waves: NT channel tiles x KS whole K parts");
    extern __shared__ float sm[];
    float *xs = sm;                          // [CINP][kPlane]
    float *red = sm + CINP * kPlane;         // K-split partials [3 parts][3 mt][64 lanes][4] per channel tile
    const int b = blockIdx.x, lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nt = wave % NT, part = wave / NT;
    const int s0 = part * PER;
    const int row = lane & 15, kq = lane >> 4;
    // this wave's weights first: their loads are in flight while the planes stage
    const int co0 = MTS == 3 ? 16 * NT * (int)blockIdx.y : 0;
    const float *wl = wk + (size_t)(4 * s0 + kq) * coutp_all + co0 + nt * 16 + row;
    float bq[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) bq[i] = wl[(size_t)i * 4 * coutp_all];
    if constexpr ((MODE & kBnIn) != 0) {
        float *st = sm + CINP * kPlane + 2 * 2304;
        bn_in_stats(bn, cin, st);
        __syncthreads();
        stage_planes_bn<CINP>(in + (size_t)b * cin * kCells, cin, bn, (size_t)b * cin * kCells, st, xs);
    } else if constexpr ((MODE & kBnGrad) != 0) {
        float *st = sm + CINP * kPlane + 2 * 2304;
        bn_grad_stats(bg, cin, st);
        __syncthreads();
        stage_planes_dz<CINP>(in + (size_t)b * cin * kCells, cin, bg, (size_t)b * cin * kCells, st, xs);
    } else {
        stage_planes_fast<CINP>(in + (size_t)b * cin * kCells, cin, xs);
    }
    __syncthreads();
    // MTS = 3: the workgroup covers all 3 position tiles and blockIdx.y picks the
    // channel slice; MTS = 1: blockIdx.y picks the position tile (all channels)
    const int mt0 = MTS == 3 ? 0 : (int)blockIdx.y;
    // per-lane A base of each position tile, biased by the most negative tap
    // offset (-10) so every k-step's offset is a non-negative immediate.  Rows past
    // the 42 cells read cell 0: D row i depends only on A row i, and those rows are
    // never stored, so the k-loop has no select (a per-MFMA exec branch kept the
    // scheduler from running LDS reads ahead: one exposed LDS round trip per MFMA)
    const float *xb[MTS];
#pragma unroll
    for (int mt = 0; mt < MTS; ++mt) {
        const int p = (mt0 + mt) * 16 + row;
        const int pp = p < kCells ? p : 0;
        xb[mt] = xs + kq * kPlane + (pp / kCols + 1) * 9 + pp % kCols + 1 - 10;
    }
    f32x4 acc[MTS];
#pragma unroll
    for (int mt = 0; mt < MTS; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the wave's K part as a compile-time constant: every LDS offset is an immediate
    auto kloop = [&](auto part_c) {
        constexpr int s0c = decltype(part_c)::value * PER;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int s = s0c + i, tap = s / CSN, cs = s % CSN;
            const int off = 4 * cs * kPlane + tap_off(tap) + 10;
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[mt][off], bq[i], acc[mt], 0, 0, 0);
        }
    };
    if constexpr (KS == 1) {
        kloop(std::integral_constant<int, 0>{});
    } else if constexpr (KS == 2) {
        if (part == 0) kloop(std::integral_constant<int, 0>{});
        else kloop(std::integral_constant<int, 1>{});
    } else {
        if (part == 0) kloop(std::integral_constant<int, 0>{});
        else if (part == 1) kloop(std::integral_constant<int, 1>{});
        else if (part == 2) kloop(std::integral_constant<int, 2>{});
        else kloop(std::integral_constant<int, 3>{});
    }
    if (KS > 1) {   // fixed-order sum of the K parts
        if (part > 0) {
            float *dst = red + (((part - 1) * 3) * 64 + lane) * 4 + nt * (3 * 3 * 64 * 4);
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) dst[mt * 64 * 4 + r] = acc[mt][r];
        }
        __syncthreads();
        if (part == 0)
#pragma unroll
        for (int q = 1; q < KS; ++q) {
            const float *src = red + (((q - 1) * 3) * 64 + lane) * 4 + nt * (3 * 3 * 64 * 4);
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[mt][r] += src[mt * 64 * 4 + r];
        }
    }
    const int n = co0 + nt * 16 + row;   // D[row = 4 kq + r][col = lane & 15]: col = channel, row = position
    // the waves that hold a finished tile (part 0); no early return: every wave
    // reaches the hand-off's barriers below
    const bool live = (KS == 1 || part == 0) && n < cout;
    const int b0 = (int)gridDim.x;   // the partials' row length: the batch
    if (live) {
        const float bv = bias ? bias[n] : 0.f;
        float *ob = out + ((size_t)b * cout + n) * kCells;
        float fin[MTS][4];   // the stored values (kGradStats)
#pragma unroll
        for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = (mt0 + mt) * 16 + 4 * kq + r;
                fin[mt][r] = 0.f;
                if (p < kCells) {
                    const float v = acc[mt][r] + bv;
                    fin[mt][r] = accumulate ? ob[p] + v : v;
                    ob[p] = fin[mt][r];
                }
            }
        if constexpr ((MODE & kGradStats) != 0) {   // the next BN backward's partials of channel n, sample b
            static_assert(MTS == 3, "statistics need the whole board");
            const size_t base = ((size_t)b * cout + n) * kCells;
            const float mu = gs.mean[n], is = gs.invstd[n];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int p = (mt0 + mt) * 16 + 4 * kq + r;
                    if (p < kCells) {
                        const float d = gs.a[base + p] > 0.f ? fin[mt][r] : 0.f;
                        s1 += d;
                        s2 += d * ((gs.z[base + p] - mu) * is);
                    }
                }
            s1 += __shfl_xor(s1, 16, 64);
            s1 += __shfl_xor(s1, 32, 64);
            s2 += __shfl_xor(s2, 16, 64);
            s2 += __shfl_xor(s2, 32, 64);
            if (kq == 0) store_part(gs.part + (size_t)n * b0 + b, s1, s2);
        }
        if constexpr ((MODE & kStatsOut) != 0) {   // the consumer's BN partials of channel n, sample b
            static_assert(MTS == 3, "statistics need the whole board");
            float s = 0.f;
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if ((mt0 + mt) * 16 + 4 * kq + r < kCells) s += acc[mt][r] + bv;
            s += __shfl_xor(s, 16, 64);   // the 4 lanes of the channel, a fixed order, the same value on each
            s += __shfl_xor(s, 32, 64);
            const float m = s / (float)kCells;
            float q = 0.f;
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if ((mt0 + mt) * 16 + 4 * kq + r < kCells) {
                        const float d = (acc[mt][r] + bv) - m;
                        q += d * d;
                    }
            q += __shfl_xor(q, 16, 64);
            q += __shfl_xor(q, 32, 64);
            if (kq == 0) store_part(bo.part + (size_t)n * b0 + b, s, q);
        }
    }
    constexpr bool kStats = (MODE & (kStatsOut | kGradStats)) != 0, kDb = (MODE & kBnGrad) != 0;
    if constexpr (kStats || kDb) {
        static_assert(MTS == 3, "the hand-off counts whole-board workgroups");
        // kBnGrad: the slice-0 workgroups' per-sample bias-gradient partials, sum_p dz
        // over the staged planes (4 lanes per channel, a fixed order)
        const bool dbw = kDb && blockIdx.y == 0;
        if (dbw) {
            const int c = threadIdx.x >> 2, q = threadIdx.x & 3;
            float s = 0.f;
            if (c < cin)
                for (int p = q; p < kCells; p += 4) s += xs[c * kPlane + (p / kCols + 1) * 9 + p % kCols + 1];
            s = chan_sum(s, 4);
            if (q == 0 && c < cin) store_part1(bg.db_part + (size_t)c * b0 + b, s);
        }
        float *flag = sm + CINP * kPlane + 2 * 2304 + kBnStatFloats;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned *tick = kStats ? ((MODE & kStatsOut) ? bo.tick : gs.tick) : nullptr;
            float l1 = 0.f, l2 = 0.f;
            if (kStats) {
                const unsigned t = __hip_atomic_fetch_add((gu32 *)(tick + blockIdx.y), 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (t == gridDim.x - 1) {
                    l1 = 1.f;
                    __hip_atomic_store((gu32 *)(tick + blockIdx.y), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (dbw) {
                const unsigned t = __hip_atomic_fetch_add((gu32 *)(bg.tick + kTickDbias), 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (t == gridDim.x - 1) {
                    l2 = 1.f;
                    __hip_atomic_store((gu32 *)(bg.tick + kTickDbias), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            flag[0] = l1;
            flag[1] = l2;
        }
        __syncthreads();
        // the last arrival merges (sc1 loads: no acquire needed, Guideline 16)
        if (kStats && flag[0] != 0.f) {
            const int ch = 16 * NT, c0 = MTS == 3 ? 16 * NT * (int)blockIdx.y : 0;
            if constexpr ((MODE & kStatsOut) != 0) fin_bn_fwd(bo, c0, ch, cout);
            if constexpr ((MODE & kGradStats) != 0) fin_bn_grad(gs, c0, ch, cout, b0);
        }
        if (kDb && flag[1] != 0.f) {   // the conv bias gradient: 4 lanes per channel, a fixed order
            const int c = threadIdx.x >> 2, q = threadIdx.x & 3;
            float s = 0.f;
            if (c < cin)
                for (int bb = q; bb < b0; bb += 4) s += load_part1(bg.db_part + (size_t)c * b0 + bb);
            s = chan_sum(s, 4);
            if (q == 0 && c < cin) bg.dbias[c] = s;
        }
    }
}

// k_conv_mfma<CINP, 1> (plain: no BatchNorm work) for SPW samples per workgroup:
// workgroup (sample pair, 16-channel slice), the K split over the 4 waves as
// there.  A wave's weight registers (its K part of the slice) serve every sample,
// so a workgroup loads them once for SPW samples, and each k-step issues 3 SPW
// MFMAs on one weight operand.  Samples past nsamp (odd batch) compute on a copy
// of the last sample and store nothing.
template <int CINP, int SPW>
__global__ __launch_bounds__(kThreads) void k_conv_mfma_spw(const float *__restrict__ in, int cin,
                                                            const float *__restrict__ wk,
                                                            const float *__restrict__ bias, int cout, int coutp_all,
                                                            float *__restrict__ out, int accumulate, int nsamp) {
    constexpr int KS = 4, CSN = CINP / 4, KSTEPS = 9 * CSN, PER = KSTEPS / KS, MTS = 3;
    static_assert(KSTEPS % KS == 0, "4 whole K parts");
    extern __shared__ float sm[];
    float *red = sm + SPW * CINP * kPlane;   // K-split partials [3 parts][SPW][3 mt][64 lanes][4]
    const int lane = threadIdx.x & 63, part = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s0 = part * PER, row = lane & 15, kq = lane >> 4;
    const int co0 = 16 * (int)blockIdx.y;
    const float *wl = wk + (size_t)(4 * s0 + kq) * coutp_all + co0 + row;
    float bq[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) bq[i] = wl[(size_t)i * 4 * coutp_all];
    int bs[SPW];
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        const int b = (int)blockIdx.x * SPW + s;
        bs[s] = b < nsamp ? b : nsamp - 1;
        stage_planes_fast<CINP>(in + (size_t)bs[s] * cin * kCells, cin, sm + s * CINP * kPlane);
    }
    __syncthreads();
    const float *xb[SPW][MTS];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int mt = 0; mt < MTS; ++mt) {
            const int p = mt * 16 + row, pp = p < kCells ? p : 0;
            xb[s][mt] = sm + s * CINP * kPlane + kq * kPlane + (pp / kCols + 1) * 9 + pp % kCols + 1 - 10;
        }
    f32x4 acc[SPW][MTS];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int mt = 0; mt < MTS; ++mt) acc[s][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto kloop = [&](auto part_c) {
        constexpr int s0c = decltype(part_c)::value * PER;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int k = s0c + i, tap = k / CSN, cs = k % CSN;
            const int off = 4 * cs * kPlane + tap_off(tap) + 10;
#pragma unroll
            for (int s = 0; s < SPW; ++s)
#pragma unroll
                for (int mt = 0; mt < MTS; ++mt)
                    acc[s][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xb[s][mt][off], bq[i], acc[s][mt], 0, 0, 0);
        }
    };
    if (part == 0) kloop(std::integral_constant<int, 0>{});
    else if (part == 1) kloop(std::integral_constant<int, 1>{});
    else if (part == 2) kloop(std::integral_constant<int, 2>{});
    else kloop(std::integral_constant<int, 3>{});
    if (part > 0) {
        float *dst = red + ((size_t)(part - 1) * SPW * MTS * 64 + lane) * 4;
#pragma unroll
        for (int s = 0; s < SPW; ++s)
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) dst[(s * MTS + mt) * 64 * 4 + r] = acc[s][mt][r];
    }
    __syncthreads();
    if (part > 0) return;   // no barrier follows
#pragma unroll
    for (int q = 1; q < KS; ++q) {   // the fixed order of k_conv_mfma's sum
        const float *src = red + ((size_t)(q - 1) * SPW * MTS * 64 + lane) * 4;
#pragma unroll
        for (int s = 0; s < SPW; ++s)
#pragma unroll
            for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[s][mt][r] += src[(s * MTS + mt) * 64 * 4 + r];
    }
    const int n = co0 + row;
    if (n >= cout) return;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        if ((int)blockIdx.x * SPW + s >= nsamp) continue;
        float *ob = out + ((size_t)bs[s] * cout + n) * kCells;
#pragma unroll
        for (int mt = 0; mt < MTS; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int p = mt * 16 + 4 * kq + r;
                if (p < kCells) {
                    const float v = acc[s][mt][r] + bv;
                    ob[p] = accumulate ? ob[p] + v : v;
                }
            }
    }
}

// weight-gradient partials: workgroup (chunk, group) accumulates, over the
// kWgSamples samples of its chunk, the output tiles of its tile group:
//   part[chunk][n][k] = sum_{b in chunk} sum_p dz[b][n][p] * X[b][p][k]   (k tap-major over CINP)
// (the conv bias gradient, sum dz, comes out of the BN backward, k_bn_bwd)
// GEMM rows = output channels (coutp/16 tiles), columns = k (round16(9 CINP)/16
// tiles), reduction = each sample's 42 positions (11 k-steps of 4).
#ifndef SPAI_WG_SAMPLES
#define SPAI_WG_SAMPLES 4
#endif
constexpr int kWgSamples = SPAI_WG_SAMPLES;
#ifndef SPAI_WG_TILES
#define SPAI_WG_TILES 3
#endif
constexpr int kWgMaxTiles = SPAI_WG_TILES;   // tiles per wave (144 tiles / 12 groups / 4 waves at 64 x 64: 384 workgroups at B = 128)
// BIAS: one more GEMM column k = K over a plane of ones, part[..][n][K] = sum_p dz:
// the conv bias gradient (for the layers whose BN backward runs in the data
// gradient's staging, kBnGrad)
template <int CINP, bool BIAS>
__global__ __launch_bounds__(kThreads) void k_wgrad_mfma(const float *__restrict__ x, int cin,
                                                         const float *__restrict__ dz, int cout, int B, int groups,
                                                         float *__restrict__ part) {
    constexpr int K = 9 * CINP, K1 = K + (BIAS ? 1 : 0), Kp = (K1 + 15) & ~15, NK = Kp / 16;
    extern __shared__ float sm[];
    const int coutp = round16(cout), NTo = coutp / 16, ntiles = NTo * NK;
    float *xs = sm;                        // [CINP][kPlane]
    float *ds = sm + CINP * kPlane;        // [coutp][44], zero past 42 and past cout
    float *ones = ds + coutp * 44;         // BIAS: [kPlane] of 1.0
    const int chunk = blockIdx.x, group = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int row = lane & 15, kq = lane >> 4;
    // this wave's tiles: group's range [t0, t1), wave-strided
    const int t0 = ntiles * group / groups, t1 = ntiles * (group + 1) / groups;
    // positions past the 42 cells read cell 0's plane entry: their dz (A) is zero
    // in ds, so the products are exact zeros, and the k-loop needs no select
    int pb[11];
#pragma unroll
    for (int s = 0; s < 11; ++s) {
        const int p = 4 * s + kq;
        const int pp = p < kCells ? p : 0;
        pb[s] = (pp / kCols + 1) * 9 + pp % kCols + 1;
    }
    f32x4 acc[kWgMaxTiles];
#pragma unroll
    for (int j = 0; j < kWgMaxTiles; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int b0 = chunk * kWgSamples, b1 = min(B, b0 + kWgSamples);
    // Staging: the zero borders of the planes, the padding channels and the dz
    // padding (positions 42, 43, rows >= cout) are written once; each sample then
    // copies only its cin x 42 inputs and cout x 42 dz values, both contiguous in
    // memory (coalesced loads at immediate offsets), to LDS destinations computed
    // once per workgroup.  The next sample's values are loaded into registers
    // while the current sample's MFMAs run.
    constexpr int NX = (CINP * kCells + kThreads - 1) / kThreads;   // 11 at 64 channels
    constexpr int ND = (64 * kCells + kThreads - 1) / kThreads;     // cout <= 64
    const int nx = cin * kCells, nd = cout * kCells;
    for (int i = threadIdx.x; i < CINP * kPlane + coutp * 44; i += kThreads) sm[i] = 0.f;
    if (BIAS)
        for (int i = threadIdx.x; i < kPlane; i += kThreads) ones[i] = 1.f;
    int dx[NX], dd[ND];
#pragma unroll
    for (int j = 0; j < NX; ++j) {
        const int i = threadIdx.x + j * kThreads, c = i / kCells, cell = i - c * kCells;
        dx[j] = i < nx ? c * kPlane + (cell / kCols + 1) * 9 + cell % kCols + 1 : 0;   // 0: a border cell (gets 0)
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
        const int i = threadIdx.x + j * kThreads, n = i / kCells, p = i - n * kCells;
        dd[j] = i < nd ? CINP * kPlane + n * 44 + p : CINP * kPlane + kCells;   // a zero pad (gets 0)
    }
    float vx[NX], vd[ND];
    auto load = [&](int b) {
        const float *xb = x + (size_t)b * nx, *db = dz + (size_t)b * nd;
#pragma unroll
        for (int j = 0; j < NX; ++j) vx[j] = threadIdx.x + j * kThreads < nx ? xb[threadIdx.x + j * kThreads] : 0.f;
#pragma unroll
        for (int j = 0; j < ND; ++j) vd[j] = threadIdx.x + j * kThreads < nd ? db[threadIdx.x + j * kThreads] : 0.f;
    };
    load(b0);
    __syncthreads();   // the zero fill lands before any sample's values
    for (int b = b0; b < b1; ++b) {
#pragma unroll
        for (int j = 0; j < NX; ++j) sm[dx[j]] = vx[j];   // past the inputs: a 0 into a zero cell
#pragma unroll
        for (int j = 0; j < ND; ++j) sm[dd[j]] = vd[j];
        __syncthreads();
        if (b + 1 < b1) load(b + 1);
#pragma unroll
        for (int j = 0; j < kWgMaxTiles; ++j) {
            const int t = t0 + wave + 4 * j;
            if (t >= t1) break;
            const int mt = t / NK, kt = t - mt * NK;
            const float *arow = ds + (mt * 16 + row) * 44;    // A[m = channel][kk = position]
            const int k = kt * 16 + row;                      // B[kk = position][n = k]
            const bool kval = k < K;
            const int tap = k / CINP, c = k % CINP;           // CINP: compile-time
            // a padding column (k >= K1) reads position data too: its D column is never stored
            const float *xcol = BIAS && k == K ? ones : xs + (kval ? c * kPlane + tap_off(tap) : 0);
#pragma unroll
            for (int s = 0; s < 11; ++s) {
                const float av = arow[4 * s + kq];
                const float bv = xcol[pb[s]];
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
            }
        }
        __syncthreads();   // xs / ds are restaged for the next sample
    }
#pragma unroll
    for (int j = 0; j < kWgMaxTiles; ++j) {
        const int t = t0 + wave + 4 * j;
        if (t >= t1) break;
        const int mt = t / NK, kt = t - mt * NK;
        const int k = kt * 16 + row;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = mt * 16 + 4 * kq + r;
            if (n < cout && k < K1) part[((size_t)chunk * cout + n) * K1 + k] = acc[j][r];
        }
    }
}

// dW[n][c][tap] = sum_chunk part[chunk][n][tap * cinp + c]  (fixed order).  At
// batch 128 there are 32 chunks: all 32 loads in flight at once, and 64-thread
// workgroups (576 of them for 64 x 64, instead of 144 of 256 threads on 256 CUs)
#ifndef SPAI_WG_REDUCE_BATCH
#define SPAI_WG_REDUCE_BATCH 32
#endif
#ifndef SPAI_WG_REDUCE_THREADS
#define SPAI_WG_REDUCE_THREADS 64
#endif
constexpr int kWgReduceBatch = SPAI_WG_REDUCE_BATCH, kWgReduceThreads = SPAI_WG_REDUCE_THREADS;
__global__ void k_wgrad_reduce(const float *__restrict__ part, int B, int cin, int cout, float *__restrict__ dw,
                               float *__restrict__ dbias) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int cinp = round4(cin), K0 = 9 * cinp, K = K0 + (dbias ? 1 : 0);   // (the bias column k = K0)
    if (i < cout * K) {   // i = n * K + k: consecutive threads read consecutive partials (coalesced)
        const int n = i / K, k = i - n * K, tap = k / cinp, c = k - tap * cinp;
        if (c < cin || k == K0) {
            const float *src = part + i;
            const size_t stride = (size_t)cout * K;
            float s = 0.f;
            for (int b0 = 0; b0 < B; b0 += kWgReduceBatch) {   // kWgReduceBatch loads in flight, summed in batch order
                float v[kWgReduceBatch];
#pragma unroll
                for (int j = 0; j < kWgReduceBatch; ++j) v[j] = b0 + j < B ? src[(size_t)(b0 + j) * stride] : 0.f;
#pragma unroll
                for (int j = 0; j < kWgReduceBatch; ++j)
                    if (b0 + j < B) s += v[j];
            }
            if (k == K0) dbias[n] = s;
            else dw[((size_t)n * cin + c) * 9 + tap] = s;
        }
    }
}

// ------------------------------------------------------------------ batch norm
// One workgroup of kBn threads per channel.  A channel's B x 42 values are read
// once into registers (kBnPer per thread; batches past kBn * kBnPer = 6144
// values, B > 146, re-read the rest from memory), so the two-pass statistics
// and the output cost one memory pass.  Sums: fixed-order wave shuffles, then
// the 16 wave partials in order (deterministic).
constexpr int kBn = 1024, kBnPer = 6;
__device__ __forceinline__ float bn_block_sum(float v, float *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kBn / 64; ++w) t += red[w];
    return t;
}
__device__ __forceinline__ size_t bn_at(int i, int c, int c_n) {
    return ((size_t)(i / kCells) * c_n + c) * kCells + i % kCells;
}

// forward in train mode, per channel: batch mean and biased variance over
// (B, 42) (two passes over the registers), invstd = 1/sqrt(var + eps); running
// stats r = (1 - m) r + m * stat (unbiased var); a = relu(gamma * (z - mean) *
// invstd + beta [+ res])
__global__ __launch_bounds__(kBn) void k_bn_fwd(const float *__restrict__ z, int c_n, int B, float eps,
                                                float momentum, float *__restrict__ mean, float *__restrict__ invstd,
                                                float *__restrict__ run_mean, float *__restrict__ run_var,
                                                const float *__restrict__ gamma, const float *__restrict__ beta,
                                                const float *__restrict__ res, float *__restrict__ a) {
    __shared__ float red[2][kBn / 64];
    const int c = blockIdx.x, n = B * kCells;
    float v[kBnPer];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kBnPer; ++j) {
        const int i = threadIdx.x + j * kBn;
        v[j] = i < n ? z[bn_at(i, c, c_n)] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kBnPer; ++j) s += v[j];
    for (int i = threadIdx.x + kBnPer * kBn; i < n; i += kBn) s += z[bn_at(i, c, c_n)];
    const float mu = bn_block_sum(s, red[0]) / (float)n;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < kBnPer; ++j)
        if (threadIdx.x + j * kBn < n) q += (v[j] - mu) * (v[j] - mu);
    for (int i = threadIdx.x + kBnPer * kBn; i < n; i += kBn) {
        const float d = z[bn_at(i, c, c_n)] - mu;
        q += d * d;
    }
    const float var = bn_block_sum(q, red[1]) / (float)n;
    const float is = 1.0f / sqrtf(var + eps);
    if (threadIdx.x == 0) {
        mean[c] = mu;
        invstd[c] = is;
        run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * mu;
        run_var[c] = (1.0f - momentum) * run_var[c] + momentum * (n > 1 ? var * (float)n / (float)(n - 1) : var);
    }
    const float ga = gamma[c], be = beta[c];
    auto out = [&](int i, float zi) {
        const size_t k = bn_at(i, c, c_n);
        float y = ga * ((zi - mu) * is) + be;
        if (res) y += res[k];
        a[k] = fmaxf(y, 0.f);
    };
#pragma unroll
    for (int j = 0; j < kBnPer; ++j)
        if (threadIdx.x + j * kBn < n) out(threadIdx.x + j * kBn, v[j]);
    for (int i = threadIdx.x + kBnPer * kBn; i < n; i += kBn) out(i, z[bn_at(i, c, c_n)]);
}

// backward of a = relu(bn(z) [+ res]): dy = da * (a > 0); per channel
// dbeta = sum dy, dgamma = sum dy * xhat;  dz = gamma*invstd/N * (N dy - dbeta - xhat dgamma);
// the conv bias gradient dbias = sum dz (zero up to rounding: the conv feeds the BN);
// dy_out (optional) = dy, the residual block's skip-path gradient.  dz may be z
// itself (every element is read and written by the same thread)
__global__ __launch_bounds__(kBn) void k_bn_bwd(const float *__restrict__ da, const float *__restrict__ a,
                                                const float *z, int c_n, int B,
                                                const float *__restrict__ mean, const float *__restrict__ invstd,
                                                const float *__restrict__ gamma, float *__restrict__ dgamma,
                                                float *__restrict__ dbeta, float *__restrict__ dbias, float *dz,
                                                float *__restrict__ dy_out) {
    __shared__ float red[3][kBn / 64];
    const int c = blockIdx.x, n = B * kCells;
    const float mu = mean[c], is = invstd[c];
    float dy[kBnPer], xh[kBnPer];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < kBnPer; ++j) {
        const int i = threadIdx.x + j * kBn;
        const bool ok = i < n;
        const size_t k = ok ? bn_at(i, c, c_n) : 0;
        const float vd = ok ? da[k] : 0.f, va = ok ? a[k] : 0.f, vz = ok ? z[k] : mu;
        dy[j] = va > 0.f ? vd : 0.f;
        xh[j] = (vz - mu) * is;
    }
#pragma unroll
    for (int j = 0; j < kBnPer; ++j) {
        s1 += dy[j];
        s2 += dy[j] * xh[j];
    }
    for (int i = threadIdx.x + kBnPer * kBn; i < n; i += kBn) {
        const size_t k = bn_at(i, c, c_n);
        const float d = a[k] > 0.f ? da[k] : 0.f;
        s1 += d;
        s2 += d * ((z[k] - mu) * is);
    }
    const float sb = bn_block_sum(s1, red[0]), sg = bn_block_sum(s2, red[1]);
    const float g = gamma[c] * is / (float)n;
    float s3 = 0.f;
    auto out = [&](int i, float d, float x) {
        const size_t k = bn_at(i, c, c_n);
        const float v = g * ((float)n * d - sb - x * sg);
        dz[k] = v;
        if (dy_out) dy_out[k] = d;
        s3 += v;
    };
#pragma unroll
    for (int j = 0; j < kBnPer; ++j)
        if (threadIdx.x + j * kBn < n) out(threadIdx.x + j * kBn, dy[j], xh[j]);
    for (int i = threadIdx.x + kBnPer * kBn; i < n; i += kBn) {
        const size_t k = bn_at(i, c, c_n);
        out(i, a[k] > 0.f ? da[k] : 0.f, (z[k] - mu) * is);
    }
    const float sz = bn_block_sum(s3, red[2]);
    if (threadIdx.x == 0) {
        dbeta[c] = sb;
        dgamma[c] = sg;
        dbias[c] = sz;
    }
}

// ------------------------------------------------------------------ heads + loss

// one workgroup per sample: policy logits (1344 -> 7), value (126 -> 1, tanh),
// loss terms and the output gradients
//   dlogits = (softmax * sum(pi) - pi) / B,  dpre = 2 (v - z) / B * (1 - v^2)
// FUSED: rp / rv are the head convs' z, and their BatchNorm + ReLU (train mode,
// k_bn_fwd's arithmetic) is applied here from the convs' partials (BnIn), writing
// the activations a for the backward
template <bool FUSED>
__global__ __launch_bounds__(kThreads) void k_heads_loss(const float *__restrict__ rp, const float *__restrict__ rv,
                                                         const float *__restrict__ wp, const float *__restrict__ bp,
                                                         const float *__restrict__ wv, const float *__restrict__ bv,
                                                         const float *__restrict__ pi, const float *__restrict__ zv,
                                                         int B, float *__restrict__ dlogits, float *__restrict__ dpre,
                                                         float *__restrict__ loss_terms, BnIn bnp, BnIn bnv) {
    __shared__ float part[kThreads / 64][8];
    __shared__ float stp[FUSED ? kBnStatFloats : 1], stv[FUSED ? kBnStatFloats : 1];
    const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float *xp = rp + (size_t)b * 32 * kCells, *xv = rv + (size_t)b * 3 * kCells;
    if constexpr (FUSED) {
        bn_in_stats(bnp, 32, stp);
        bn_in_stats(bnv, 3, stv);
        __syncthreads();
    }
    auto act = [&](float z, const float *st, int c, float *a_out, int k) {
        if constexpr (!FUSED) return z;
        const float y = fmaxf(st[128 + c] * ((z - st[c]) * st[64 + c]) + st[192 + c], 0.f);
        a_out[k] = y;
        return y;
    };
    // one pass over the features: 7 policy logits and the value pre-activation at
    // once; wave sums by shuffles, then the 4 wave partials in order
    float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = threadIdx.x; k < 32 * kCells; k += kThreads) {
        const float xk = act(xp[k], stp, k / kCells, bnp.a_out + (size_t)b * 32 * kCells, k);
#pragma unroll
        for (int o = 0; o < 7; ++o) acc8[o] += xk * wp[o * 32 * kCells + k];
    }
    for (int k = threadIdx.x; k < 3 * kCells; k += kThreads)
        acc8[7] += act(xv[k], stv, k / kCells, bnv.a_out + (size_t)b * 3 * kCells, k) * wv[k];
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) acc8[o] += __shfl_xor(acc8[o], sh, 64);
    }
    if (lane == 0)
#pragma unroll
        for (int o = 0; o < 8; ++o) part[wave][o] = acc8[o];
    __syncthreads();
    float lg[7];
#pragma unroll
    for (int o = 0; o < 7; ++o) lg[o] = ((part[0][o] + part[1][o]) + part[2][o]) + part[3][o] + bp[o];
    const float pre = ((part[0][7] + part[1][7]) + part[2][7]) + part[3][7] + bv[0];
    if (threadIdx.x == 0) {
        float mx = lg[0];
        for (int o = 1; o < 7; ++o) mx = fmaxf(mx, lg[o]);
        float se = 0.f;
        for (int o = 0; o < 7; ++o) se += expf(lg[o] - mx);
        const float lse = mx + logf(se);
        float nll = 0.f, spi = 0.f;
        for (int o = 0; o < 7; ++o) {
            nll += (lg[o] - lse) * pi[b * 7 + o];
            spi += pi[b * 7 + o];
        }
        for (int o = 0; o < 7; ++o) dlogits[b * 7 + o] = (expf(lg[o] - lse) * spi - pi[b * 7 + o]) / (float)B;
        const float v = tanhf(pre), d = v - zv[b];
        dpre[b] = 2.0f * d / (float)B * (1.0f - v * v);
        loss_terms[2 * b] = -nll;      // policy term of sample b
        loss_terms[2 * b + 1] = d * d; // value term
    }
}

// linear backward, out features O, in features K:
//   dW[o][k] = sum_b dy[b][o] x[b][k];  db[o] = sum_b dy[b][o];  dx[b][k] = sum_o dy[b][o] W[o][k]
// dw[o][k] = sum_b dy[b][o] x[b][k], db[o] = sum_b dy[b][o].  A workgroup owns 64
// outputs; its 4 waves take a quarter of the batch each (16 loads in flight),
// and the quarters are added in order through LDS.
__global__ __launch_bounds__(kThreads) void k_linear_bwd_w(const float *__restrict__ x, const float *__restrict__ dy,
                                                           int B, int O, int K, float *__restrict__ dw,
                                                           float *__restrict__ db) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const int bq0 = B * q / 4, bq1 = B * (q + 1) / 4;
    float s = 0.f;
    if (i < O * K) {
        const int o = i / K, k = i - o * K;
        for (int b0 = bq0; b0 < bq1; b0 += 16) {
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = b0 + j < bq1 ? x[(size_t)(b0 + j) * K + k] : 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if (b0 + j < bq1) s += dy[(b0 + j) * O + o] * v[j];
        }
    }
    part[q][lane] = s;
    __syncthreads();
    if (q == 0 && i < O * K) dw[i] = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    if (blockIdx.x == 0 && q == 1 && lane < O) {   // db: 16 loads in flight, summed in batch order
        float t = 0.f;
        for (int b0 = 0; b0 < B; b0 += 16) {
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = b0 + j < B ? dy[(b0 + j) * O + lane] : 0.f;
#pragma unroll
            for (int j = 0; j < 16; ++j) t += v[j];
        }
        db[lane] = t;
    }
}
__global__ void k_linear_bwd_x(const float *__restrict__ dy, const float *__restrict__ w, int B, int O, int K,
                               float *__restrict__ dx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * K) return;
    const int b = (int)(i / K), k = (int)(i - (size_t)b * K);
    float s = 0.f;
    for (int o = 0; o < O; ++o) s += dy[b * O + o] * w[o * K + k];
    dx[i] = s;
}

// ------------------------------------------------------------------ Adam (torch semantics)
// m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;
// p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)      (g scaled by gscale)
// bc = {1 - b1^t, sqrt(1 - b2^t)} for this step (host-computed, staged with the batch)
__global__ void k_adam(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                       float *__restrict__ v, size_t n, float gscale, float lr, float b1, float b2, float eps,
                       const float *__restrict__ bc) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float bc1 = bc[0], bc2_sqrt = bc[1];
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= (lr / bc1) * (mi / (sqrtf(vi) / bc2_sqrt + eps));
}

// data-parallel weighting: this rank's mean gradient times B_rank / sum over ranks of B
__global__ void k_weight_grad(float *__restrict__ g, size_t n, float b_local, const float *__restrict__ b_sum) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    g[i] *= b_local / b_sum[0];
}

__global__ void k_set1(float *__restrict__ dst, float v) { *dst = v; }

// running stats gathered into / scattered from a packed buffer (cross-rank average)
__global__ void k_gather(const float *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t n,
                         float *__restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}
__global__ void k_scatter_scaled(const float *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t n,
                                 float scale, float *__restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[idx[i]] = src[i] * scale;
}

inline unsigned blocks_of(size_t n, int t = kThreads) { return (unsigned)((n + t - 1) / t); }

}  // namespace
}  // namespace spai

// ---------------------------------------------------------------------- host
namespace spai {
namespace {

int learner_alloc_batch(spai_learner *L, uint32_t B) {
    if (B <= L->max_batch) return SPAI_OK;
    const size_t act = (size_t)B * std::max(L->hidden, 32) * kCells;   // also the 32-channel policy head
    SPAI_TRY(L->batch_in.alloc((size_t)B * (3 * kCells + 8) + 2));
    for (float **h : {&L->stage, &L->stage_b}) {
        if (*h) (void)hipHostFree(*h);
        *h = nullptr;
        if (hipHostMalloc((void **)h, ((size_t)B * (3 * kCells + 10) + 2) * sizeof(float), hipHostMallocDefault) !=
            hipSuccess) {
            *h = nullptr;
            set_error("learner: pinned staging allocation failed");
            return SPAI_ERR_DEVICE;
        }
    }
    for (size_t l = 0; l < L->convs.size(); ++l) {
        SPAI_TRY(L->z[l].alloc((size_t)B * L->convs[l].co * kCells));
        SPAI_TRY(L->a[l].alloc((size_t)B * L->convs[l].co * kCells));
    }
    SPAI_TRY(L->d0.alloc(act));
    SPAI_TRY(L->d1.alloc(act));
    // trunk + the two heads' partials, the bias-gradient partials [64][B], the hand-off counters
    SPAI_TRY(L->bn_part.alloc((size_t)(2 * L->blocks + 3) * L->hidden * B * 2 + (size_t)L->hidden * B + kTicks));
    SPAI_TRY(L->d2.alloc(act));
    if (L->blocks > 0) SPAI_TRY(L->dzb.alloc((size_t)2 * L->blocks * B * L->hidden * kCells));
    SPAI_TRY(L->dlogits.alloc((size_t)B * 7));
    SPAI_TRY(L->dpre.alloc(B));
    SPAI_TRY(L->loss_terms.alloc((size_t)B * 2));
    const size_t cmax = (size_t)std::max(L->hidden, 32);
    for (auto &w : L->wpart_side)   // weight-gradient partials per chunk (one buffer per side stream)
        SPAI_TRY(w.alloc((size_t)((B + kWgSamples - 1) / kWgSamples) * cmax * (9 * round4(L->hidden) + 1)));
    L->max_batch = B;
    return SPAI_OK;
}

// out (+)= conv(in) on f32 MFMA with a packed weight matrix wk (forward or
// data-gradient orientation, k_pack_all).  The learner's shapes: input channels
// 3 (-> 4), 32 or 64; output 3 (1 tile), 32 (2) or 64 (4).  Where the k-steps
// split into 4 whole parts (32 and 64 input channels) every 16-channel tile is
// its own workgroup with the K split over its 4 waves (grid B x coutp/16: 4x
// the workgroups of one per sample); the stem's input (4 padded channels, 9
// k-steps) keeps one workgroup per sample with a wave per channel tile.
// samples per workgroup of the plain convs (1: k_conv_mfma; 2: k_conv_mfma_spw, a
// measured variant: 12.7 against 10.9 us per conv, 181k against 189k samples/s --
// its 272 registers leave one workgroup per CU, whose staging, k-loop and K-part
// sum then run back to back instead of overlapping another workgroup's;
// profiles/r05/learner/spw)
#ifndef SPAI_CONV_SPW
#define SPAI_CONV_SPW 1
#endif
constexpr int kConvSpw = SPAI_CONV_SPW;

template <int CINP, int MODE>
int launch_conv_t(int B, size_t lds, hipStream_t st, const float *in, int cin, const float *wk, const float *bias,
                  int cout, float *out, int acc, const BnIn &bn, const BnIn &bo, const BnGrad &bg, const GradStats &gs) {
    constexpr int ks = 9 * CINP / 4;
    const int nt = round16(cout) / 16;
#ifdef SPAI_SLICE_NT2   // variant: 32-channel slices, the K split over 2 wave pairs
    if constexpr (ks % 2 == 0) {
        if (nt % 2 == 0) {
            k_conv_mfma<CINP, 2, MODE><<<dim3(B, nt / 2), kThreads, lds, st>>>(in, cin, wk, bias, cout, 16 * nt, out,
                                                                              acc, bn, bo, bg, gs);
            return SPAI_OK;
        }
    }
#endif
    if constexpr (ks % 4 == 0) {
        if constexpr (MODE == 0 && kConvSpw > 1) {   // plain conv: kConvSpw samples per workgroup
            const size_t lds2 = ((size_t)kConvSpw * CINP * kPlane + (size_t)3 * kConvSpw * 3 * 64 * 4) * sizeof(float);
            k_conv_mfma_spw<CINP, kConvSpw><<<dim3((B + kConvSpw - 1) / kConvSpw, nt), kThreads, lds2, st>>>(
                in, cin, wk, bias, cout, 16 * nt, out, acc, B);
            return SPAI_OK;
        }
        k_conv_mfma<CINP, 1, MODE><<<dim3(B, nt), kThreads, lds, st>>>(in, cin, wk, bias, cout, 16 * nt, out, acc, bn,
                                                                      bo, bg, gs);
        return SPAI_OK;
    }
    if (nt == 4) {
        k_conv_mfma<CINP, 4, MODE><<<dim3(B), kThreads, lds, st>>>(in, cin, wk, bias, cout, 64, out, acc, bn, bo,
                                                                  bg, gs);
        return SPAI_OK;
    }
    set_error("learner conv: %d input / %d output channels not built", cin, cout);
    return SPAI_ERR_UNSUPPORTED;
}

// bn: the input's BatchNorm applied while staging (in = the producer's z), or
// null; bo: this conv's BatchNorm, whose per-(channel, sample) partials it leaves
// and merges (kStatsOut), or null; bg: the input (= da) turned into this layer's
// dz while staging (the BN backward), or null; gs: the BN-backward partials of the
// layer whose da this conv writes, merged here, or null
int launch_conv(const float *in, int cin, const float *wk, const float *bias, int cout, float *out, int B, bool acc,
                hipStream_t st, const BnIn *bn = nullptr, const BnIn *bo = nullptr, const BnGrad *bg = nullptr,
                const GradStats *gs = nullptr) {
    const int cinp = round4(cin);
    const size_t lds = ((size_t)cinp * kPlane + 2 * 2304 + (bn || bo || bg || gs ? kBnStatFloats + kLdsFlags : 0)) *
                       sizeof(float);
    const int a = acc ? 1 : 0;
    const BnIn bn0{};
    const BnGrad bg0{};
    const GradStats gs0{};
    const BnIn &b = bn ? *bn : bn0;
    const BnIn &o = bo ? *bo : bn0;
    const BnGrad &g = bg ? *bg : bg0;
    const GradStats &s = gs ? *gs : gs0;
    const int mode = (bn ? kBnIn : 0) | (bo ? kStatsOut : 0) | (bg ? kBnGrad : 0) | (gs ? kGradStats : 0);
    // the hand-off counters are per channel slice
    if ((bo || gs) && round16(cout) / 16 > kTickDbias) {
        set_error("learner conv: %d output channels exceed the BatchNorm hand-off's slices", cout);
        return SPAI_ERR_UNSUPPORTED;
    }
#define SPAI_CONV_CASE(C, M) \
    case (C) * 16 + (M): return launch_conv_t<C, M>(B, lds, st, in, cin, wk, bias, cout, out, a, b, o, g, s);
    switch (cinp * 16 + mode) {
    SPAI_CONV_CASE(4, 0)
    SPAI_CONV_CASE(4, kStatsOut)
    SPAI_CONV_CASE(4, kGradStats)
    SPAI_CONV_CASE(32, 0)
    SPAI_CONV_CASE(64, 0)
    SPAI_CONV_CASE(64, kStatsOut)
    SPAI_CONV_CASE(64, kBnIn)
    SPAI_CONV_CASE(64, kBnIn | kStatsOut)
    SPAI_CONV_CASE(64, kBnGrad)
    SPAI_CONV_CASE(64, kBnGrad | kGradStats)
    default: set_error("learner conv: %d input channels (mode %d) not built", cin, mode); return SPAI_ERR_UNSUPPORTED;
    }
#undef SPAI_CONV_CASE
}

// dW (and db, when given) of one conv: chunk partials on f32 MFMA, then a fixed-order sum over the chunks
int launch_wgrad(float *wpart, const float *x, int cin, const float *dz, int cout, int B, float *dw, hipStream_t st,
                 float *db = nullptr) {
    const int cinp = round4(cin), k1 = 9 * cinp + (db ? 1 : 0), nk = (k1 + 15) / 16, ntiles = (round16(cout) / 16) * nk;
    const int groups = std::max(1, (ntiles + 4 * kWgMaxTiles - 1) / (4 * kWgMaxTiles));
    const int chunks = (B + kWgSamples - 1) / kWgSamples;
    const size_t lds = ((size_t)cinp * kPlane + (size_t)round16(cout) * 44 + (db ? kPlane : 0)) * sizeof(float);
    const dim3 grid(chunks, groups);
    switch (cinp * 2 + (db ? 1 : 0)) {
    case 4 * 2: k_wgrad_mfma<4, false><<<grid, kThreads, lds, st>>>(x, cin, dz, cout, B, groups, wpart); break;
    case 64 * 2: k_wgrad_mfma<64, false><<<grid, kThreads, lds, st>>>(x, cin, dz, cout, B, groups, wpart); break;
    case 64 * 2 + 1: k_wgrad_mfma<64, true><<<grid, kThreads, lds, st>>>(x, cin, dz, cout, B, groups, wpart); break;
    default: set_error("learner wgrad: %d input channels not built", cin); return SPAI_ERR_UNSUPPORTED;
    }
    k_wgrad_reduce<<<blocks_of((size_t)cout * k1, kWgReduceThreads), kWgReduceThreads, 0, st>>>(wpart, chunks, cin, cout,
                                                                                               dw, db);
    return SPAI_OK;
}

}  // namespace

int learner_create(spai_engine *e, int blocks, int hidden, const float *params, size_t n, const spai_adam_config *cfg,
                   spai_learner **out) {
    SPAI_CHECK(e->game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "learner: only Connect4 is built");
    SPAI_CHECK(hidden == 64, SPAI_ERR_UNSUPPORTED, "learner: hidden must be 64 (got %d)", hidden);
    SPAI_CHECK(blocks >= 0 && blocks <= 40, SPAI_ERR_UNSUPPORTED, "learner: 0..40 blocks (got %d)", blocks);
    SPAI_CHECK(params && n == net_num_params(e->game, blocks, hidden), SPAI_ERR_INVALID, "expected %zu params, got %zu",
               net_num_params(e->game, blocks, hidden), n);
    spai_learner *L = new spai_learner();
    L->eng = e;
    L->blocks = blocks;
    L->hidden = hidden;
    if (cfg) L->cfg = *cfg;
    else spai_adam_config_default(&L->cfg);
    size_t off = 0;
    auto conv = [&](int ci, int co) {
        spai_learner::Conv c{ci, co, 0, 0, 0, 0, 0, 0, 0, 0};
        c.w = off;
        off += (size_t)co * ci * 9;
        c.b = off;
        off += co;
        c.g = off;
        c.be = off + co;
        c.mu = off + 2 * co;
        c.var = off + 3 * co;
        off += 4 * (size_t)co;
        L->convs.push_back(c);
    };
    conv(3, hidden);
    for (int i = 0; i < 2 * blocks; ++i) conv(hidden, hidden);
    conv(hidden, 32);
    L->pol_w = off;
    off += 7 * 32 * kCells;
    L->pol_b = off;
    off += 7;
    conv(hidden, 3);
    L->val_w = off;
    off += 3 * kCells;
    L->val_b = off;
    off += 1;
    L->n_params = off;
    int rc = SPAI_OK;
    auto chk = [&](int r) {
        if (rc == SPAI_OK) rc = r;
    };
    chk(L->p.alloc(n));
    chk(L->g.alloc(n));
    chk(L->bsum.alloc(1));
    chk(L->m.alloc(n));
    chk(L->v.alloc(n));
    {   // packed [k][n] matrices: every conv forward, every conv but the stem data gradient
        std::vector<uint32_t> desc;
        size_t woff = 0;
        auto entry = [&](size_t wparam, int cin, int cout, int dgrad) {
            const int cinp = round4(cin), coutp = round16(cout);
            desc.insert(desc.end(), {(uint32_t)wparam, (uint32_t)cin, (uint32_t)cout, (uint32_t)cinp, (uint32_t)coutp,
                                     (uint32_t)dgrad, (uint32_t)woff, 0u});
            woff += (size_t)9 * cinp * coutp;
            return woff - (size_t)9 * cinp * coutp;
        };
        for (size_t l = 0; l < L->convs.size(); ++l) {
            spai_learner::Conv &c = L->convs[l];
            c.wk = entry(c.w, c.ci, c.co, 0);
            c.wkd = l == 0 ? 0 : entry(c.w, c.co, c.ci, 1);
        }
        L->n_pack = (int)(desc.size() / kPackDesc);
        chk(L->wt.alloc(woff));
        chk(L->pack_desc.alloc(desc.size()));
        if (rc == SPAI_OK &&
            hipMemcpy(L->pack_desc.p, desc.data(), desc.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            set_error("learner: upload failed");
            rc = SPAI_ERR_DEVICE;
        }
    }
    L->z.resize(L->convs.size());
    L->a.resize(L->convs.size());
    L->mean.resize(L->convs.size());
    L->invstd.resize(L->convs.size());
    std::vector<uint32_t> ridx;
    for (size_t l = 0; l < L->convs.size(); ++l) {
        chk(L->mean[l].alloc(L->convs[l].co));
        chk(L->invstd[l].alloc(L->convs[l].co));
        for (int c = 0; c < L->convs[l].co; ++c) ridx.push_back((uint32_t)(L->convs[l].mu + c));
        for (int c = 0; c < L->convs[l].co; ++c) ridx.push_back((uint32_t)(L->convs[l].var + c));
    }
    chk(L->run_idx.alloc(ridx.size()));
    L->ev_dz.assign(L->convs.size(), nullptr);
    for (int k = 0; k < spai_learner::kWgStreams; ++k)
        if (rc == SPAI_OK && (hipStreamCreateWithFlags(&L->wg_stream[k], hipStreamNonBlocking) != hipSuccess ||
                              hipEventCreateWithFlags(&L->ev_wg_done[k], hipEventDisableTiming) != hipSuccess)) {
            set_error("learner: stream/event creation failed");
            rc = SPAI_ERR_DEVICE;
        }
    for (auto &ev : L->stage_ev)
        if (rc == SPAI_OK && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            set_error("learner: event creation failed");
            rc = SPAI_ERR_DEVICE;
        }
    for (auto &ev : L->ev_dz)
        if (rc == SPAI_OK && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            set_error("learner: event creation failed");
            rc = SPAI_ERR_DEVICE;
        }
    chk(L->run_buf.alloc(ridx.size()));
    if (rc == SPAI_OK) {
        hipStream_t st = e->stream;
        if (hipMemcpyAsync(L->p.p, params, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(L->run_idx.p, ridx.data(), ridx.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(L->m.p, 0, n * 4, st) != hipSuccess || hipMemsetAsync(L->v.p, 0, n * 4, st) != hipSuccess ||
            hipMemsetAsync(L->g.p, 0, n * 4, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            set_error("learner: upload failed");
            rc = SPAI_ERR_DEVICE;
        }
    }
    if (rc != SPAI_OK) {
        learner_destroy(L);
        return rc;
    }
    *out = L;
    return SPAI_OK;
}

void learner_destroy(spai_learner *L) {
    if (!L) return;
    if (L->eng) (void)hipStreamSynchronize(L->eng->stream);
    for (hipStream_t ws : L->wg_stream)
        if (ws) (void)hipStreamSynchronize(ws);
    if (L->graph) (void)hipGraphExecDestroy(L->graph);
    if (L->comm) (void)ncclCommDestroy((ncclComm_t)L->comm);
    for (hipEvent_t ev : L->ev_dz)
        if (ev) (void)hipEventDestroy(ev);
    for (int k = 0; k < spai_learner::kWgStreams; ++k) {
        if (L->ev_wg_done[k]) (void)hipEventDestroy(L->ev_wg_done[k]);
        if (L->wg_stream[k]) (void)hipStreamDestroy(L->wg_stream[k]);
        L->wpart_side[k].release();
    }
    L->pack_desc.release();
    if (L->stage) (void)hipHostFree(L->stage);
    if (L->stage_b) (void)hipHostFree(L->stage_b);
    if (L->terms_host) (void)hipHostFree(L->terms_host);
    for (hipEvent_t ev : L->stage_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (L->host_buf) (void)hipHostFree(L->host_buf);
    for (auto *b : {&L->p, &L->g, &L->bsum, &L->m, &L->v, &L->wt, &L->batch_in, &L->d0, &L->d1, &L->d2, &L->dzb, &L->bn_part, &L->dlogits,
                    &L->dpre, &L->loss_terms, &L->run_buf})
        b->release();
    L->run_idx.release();
    for (auto *vec : {&L->z, &L->a, &L->mean, &L->invstd})
        for (auto &b : *vec) b.release();
    delete L;
}

// One cross-rank sum of n device floats, in place, in stream order: RCCL over
// xGMI, or the caller's host collective (spai_learner_set_host_comm) through the
// pinned staging buffer, which blocks the calling thread until every rank arrived.
static int learner_allreduce(spai_learner *L, float *buf, size_t n, hipStream_t st, const char *what) {
    if (L->comm) {
        if (ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, (ncclComm_t)L->comm, st) != ncclSuccess) {
            set_error("ncclAllReduce of %s failed", what);
            return SPAI_ERR_DEVICE;
        }
        return SPAI_OK;
    }
    SPAI_CHECK(L->host_ar && n <= L->host_buf_n, SPAI_ERR_INVALID, "host all-reduce of %s: no collective", what);
    SPAI_HIP(hipMemcpyAsync(L->host_buf, buf, n * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    const int r = L->host_ar(L->host_ar_user, L->host_buf, n);
    SPAI_CHECK(r == 0, SPAI_ERR_DEVICE, "host all-reduce of %s failed (%d)", what, r);
    SPAI_HIP(hipMemcpyAsync(buf, L->host_buf, n * 4, hipMemcpyHostToDevice, st));
    return SPAI_OK;
}

// carved from the end of bn_part: the bias-gradient partials, then the counters
static float *learner_db_part(spai_learner *L, uint32_t B) {
    return L->bn_part.p + (size_t)(2 * L->blocks + 3) * L->hidden * B * 2;
}
static unsigned *learner_ticks(spai_learner *L, uint32_t B) {
    return (unsigned *)(learner_db_part(L, B) + (size_t)L->hidden * B);
}

// Everything of one train step after the batch upload: gradients zeroed, weights
// packed, forward, loss, backward (weight gradients on the side streams), the cross-rank
// reduction when there is a communicator, Adam.  Launch-only (no host sync).
int enqueue_step(spai_learner *L, uint32_t B, hipStream_t st, const float *x_in, const float *pi_in,
                 const float *z_in, const float *bc) {
    float *P = L->p.p, *G = L->g.p;
    // G needs no clearing: every trainable entry is written (not accumulated) by
    // this step's kernels, and the BN running-statistic entries stay at the zero
    // they got at learner_create
    const float eps = L->cfg.bn_eps, mom = L->cfg.bn_momentum;
    const size_t nl = L->convs.size();
    k_pack_all<<<dim3(blocks_of((size_t)9 * 64 * 64), L->n_pack), kThreads, 0, st>>>(P, L->pack_desc.p, L->wt.p,
                                                                                        learner_ticks(L, B));
    const float *W = L->wt.p;
    const int pol = (int)nl - 2, val = (int)nl - 1;

    // ---------------- forward (train mode)
    int crc = SPAI_OK;   // conv launch status (shape dispatch)
    auto conv_bn_act = [&](int l, const float *in, const float *res) {
        const spai_learner::Conv &c = L->convs[l];
        if (crc == SPAI_OK) crc = launch_conv(in, c.ci, W + c.wk, P + c.b, c.co, L->z[l].p, (int)B, false, st);
        k_bn_fwd<<<c.co, kBn, 0, st>>>(L->z[l].p, c.co, (int)B, eps, mom, L->mean[l].p, L->invstd[l].p, P + c.mu,
                                       P + c.var, P + c.g, P + c.be, res, L->a[l].p);
    };
    // default: a k_bn_fwd kernel after every conv.  SPAI_LEARNER_BN_FUSE=1 (measured
    // variant, not the default): the trunk's BN + ReLU (+ residual) run inside the
    // next conv's staging (BnIn), the statistics merged inside the producer conv --
    // 150-172k samples/s against 190-196k (profiles/r05/learner): at B = 128 a conv
    // is a ~11 us, latency-bound launch, and the in-launch hand-off's drain, ticket
    // and merge (or, merged in the consumer's prologue, every workgroup's read of
    // the B partials) cost more than the k_bn_fwd / k_bn_bwd launches they remove
    static const bool fuse = [] {
        const char *v = std::getenv("SPAI_LEARNER_BN_FUSE");
        return v && std::atoi(v) != 0;
    }();
    const float *h = nullptr;
    if (fuse) {
        const int last = 2 * L->blocks;   // the trunk's last conv
        auto part_of = [&](int l) { return (float2 *)L->bn_part.p + (size_t)l * L->hidden * B; };
        // layer l's BN input to its consumer: the residual is the block input a[l - 2] for a block's second conv
        unsigned *tick = learner_ticks(L, B);
        auto bn_of = [&](int l) {
            const spai_learner::Conv &c = L->convs[l];
            const bool res = l >= 2 && l <= last && l % 2 == 0;
            return BnIn{part_of(l), P + c.g, P + c.be, res ? L->a[l - 2].p : nullptr, L->a[l].p, L->mean[l].p,
                        L->invstd[l].p, P + c.mu, P + c.var, (int)B, eps, mom, tick};
        };
        {
            const spai_learner::Conv &c = L->convs[0];
            const BnIn o = bn_of(0);
            crc = launch_conv(x_in, c.ci, W + c.wk, P + c.b, c.co, L->z[0].p, (int)B, false, st, nullptr, &o);
        }
        for (int l = 1; l <= last && crc == SPAI_OK; ++l) {   // relu(h + BN(conv(relu(BN(conv(h)))))), model/mod.rs:152-165
            const spai_learner::Conv &c = L->convs[l];
            const BnIn b = bn_of(l - 1), o = bn_of(l);
            crc = launch_conv(L->z[l - 1].p, c.ci, W + c.wk, P + c.b, c.co, L->z[l].p, (int)B, false, st, &b, &o);
        }
        if (crc == SPAI_OK) {   // the policy head conv applies the trunk's last BN and writes the trunk output
            const spai_learner::Conv &c = L->convs[pol];
            const BnIn b = bn_of(last), o = bn_of(pol);
            crc = launch_conv(L->z[last].p, c.ci, W + c.wk, P + c.b, c.co, L->z[pol].p, (int)B, false, st, &b, &o);
        }
        h = L->a[last].p;
        if (crc == SPAI_OK) {
            const spai_learner::Conv &c = L->convs[val];
            const BnIn o = bn_of(val);
            crc = launch_conv(h, c.ci, W + c.wk, P + c.b, c.co, L->z[val].p, (int)B, false, st, nullptr, &o);
        }
        // the heads' BN + ReLU inside the loss kernel
        k_heads_loss<true><<<B, kThreads, 0, st>>>(L->z[pol].p, L->z[val].p, P + L->pol_w, P + L->pol_b, P + L->val_w,
                                                   P + L->val_b, pi_in, z_in, (int)B, L->dlogits.p, L->dpre.p,
                                                   L->loss_terms.p, bn_of(pol), bn_of(val));
    } else {
        conv_bn_act(0, x_in, nullptr);
        h = L->a[0].p;
        for (int k = 0; k < L->blocks; ++k) {   // relu(h + BN(conv(relu(BN(conv(h)))))) (model/mod.rs:152-165)
            conv_bn_act(1 + 2 * k, h, nullptr);
            conv_bn_act(2 + 2 * k, L->a[1 + 2 * k].p, h);
            h = L->a[2 + 2 * k].p;
        }
        conv_bn_act(pol, h, nullptr);
        conv_bn_act(val, h, nullptr);
    }
    if (!fuse)
        k_heads_loss<false><<<B, kThreads, 0, st>>>(L->a[pol].p, L->a[val].p, P + L->pol_w, P + L->pol_b, P + L->val_w,
                                                    P + L->val_b, pi_in, z_in, (int)B, L->dlogits.p, L->dpre.p,
                                                    L->loss_terms.p, BnIn{}, BnIn{});

    // ---------------- backward
    // heads: linears -> relu/BN -> conv; dh (d0) = dgrad(policy) + dgrad(value)
    k_linear_bwd_w<<<(7 * 32 * kCells + 63) / 64, kThreads, 0, st>>>(L->a[pol].p, L->dlogits.p, (int)B, 7, 32 * kCells,
                                                                     G + L->pol_w, G + L->pol_b);
    k_linear_bwd_x<<<blocks_of((size_t)B * 32 * kCells), kThreads, 0, st>>>(L->dlogits.p, P + L->pol_w, (int)B, 7,
                                                                             32 * kCells, L->d1.p);
    // conv l's dz (written over z[l] by k_bn_bwd) feeds its data gradient here and
    // its weight gradient on a side stream; nothing rewrites z[l] before the next step
#ifndef SPAI_WG_SIDE
#define SPAI_WG_SIDE spai_learner::kWgStreams
#endif
    int side = 0;
    // dz: the layer's BN-backward output (z[l] overwritten by k_bn_bwd, or the fused
    // path's dz buffer); db: the bias gradient from the weight gradient (fused path)
    auto wgrad_async = [&](int l, const float *in, const float *dz = nullptr, float *db = nullptr) {
        const spai_learner::Conv &c = L->convs[l];
        if (crc != SPAI_OK) return;
        const int k = side++ % SPAI_WG_SIDE;
        if (hipEventRecord(L->ev_dz[l], st) != hipSuccess ||
            hipStreamWaitEvent(L->wg_stream[k], L->ev_dz[l], 0) != hipSuccess) {
            set_error("learner: event record/wait failed");
            crc = SPAI_ERR_DEVICE;
            return;
        }
        crc = launch_wgrad(L->wpart_side[k].p, in, c.ci, dz ? dz : L->z[l].p, c.co, (int)B, G + c.w, L->wg_stream[k],
                           db);
    };
    auto bn_conv_bwd = [&](int l, const float *da, const float *in, float *dx, bool acc, float *dy_out) {
        const spai_learner::Conv &c = L->convs[l];
        k_bn_bwd<<<c.co, kBn, 0, st>>>(da, L->a[l].p, L->z[l].p, c.co, (int)B, L->mean[l].p, L->invstd[l].p,
                                       P + c.g, G + c.g, G + c.be, G + c.b, L->z[l].p, dy_out);
        wgrad_async(l, in);
        if (dx && crc == SPAI_OK) crc = launch_conv(L->z[l].p, c.co, W + c.wkd, nullptr, c.ci, dx, (int)B, acc, st);
    };
    bn_conv_bwd(pol, L->d1.p, h, L->d0.p, false, nullptr);
    k_linear_bwd_w<<<(3 * kCells + 63) / 64, kThreads, 0, st>>>(L->a[val].p, L->dpre.p, (int)B, 1, 3 * kCells,
                                                                G + L->val_w, G + L->val_b);
    k_linear_bwd_x<<<blocks_of((size_t)B * 3 * kCells), kThreads, 0, st>>>(L->dpre.p, P + L->val_w, (int)B, 1,
                                                                            3 * kCells, L->d1.p);
    // with the forward fusion on (SPAI_LEARNER_BN_FUSE=1), the trunk's BN backward runs in
    // the data gradient's staging (BnGrad), its partials from the producer of da
    // (GradStats), unless SPAI_LEARNER_BNB_FUSE=0 (a k_bn_bwd kernel before every data gradient)
    static const bool bfuse = [] {
        const char *v = std::getenv("SPAI_LEARNER_BNB_FUSE");
        return !v || std::atoi(v) != 0;
    }();
    if (fuse && bfuse) {
        const int last = 2 * L->blocks;
        auto gpart_of = [&](int l) { return (float2 *)L->bn_part.p + (size_t)l * L->hidden * B; };
        auto dzb_of = [&](int l) { return L->dzb.p + (size_t)(l - 1) * B * L->hidden * kCells; };   // l >= 1
        unsigned *tick = learner_ticks(L, B);
        float *db_part = learner_db_part(L, B);
        auto gs_of = [&](int l) {
            const spai_learner::Conv &c = L->convs[l];
            return GradStats{L->a[l].p, L->z[l].p, L->mean[l].p, L->invstd[l].p, gpart_of(l), G + c.g, G + c.be, tick};
        };
        auto bg_of = [&](int l, float *dy_out) {
            const spai_learner::Conv &c = L->convs[l];
            return BnGrad{L->a[l].p, L->z[l].p, L->mean[l].p, L->invstd[l].p, P + c.g, G + c.g, G + c.be, dzb_of(l),
                          dy_out, db_part, G + c.b, tick, (int)B};
        };
        {   // value head: its BN backward as before; its data gradient completes dL/d(trunk output)
            const spai_learner::Conv &c = L->convs[val];
            k_bn_bwd<<<c.co, kBn, 0, st>>>(L->d1.p, L->a[val].p, L->z[val].p, c.co, (int)B, L->mean[val].p,
                                           L->invstd[val].p, P + c.g, G + c.g, G + c.be, G + c.b, L->z[val].p, nullptr);
            wgrad_async(val, h);
            const GradStats g = gs_of(last);
            if (crc == SPAI_OK)
                crc = launch_conv(L->z[val].p, c.co, W + c.wkd, nullptr, c.ci, L->d0.p, (int)B, true, st, nullptr,
                                  nullptr, nullptr, last > 0 ? &g : nullptr);
        }
        float *X = L->d0.p, *Y = L->d1.p, *T = L->d2.p;   // dL/d(block output), dL/d(relu1 output), skip + block input
        for (int k = L->blocks - 1; k >= 0 && crc == SPAI_OK; --k) {
            const int l1 = 1 + 2 * k, l2 = 2 + 2 * k;
            const float *hin = L->a[l1 - 1].p;
            {   // conv 2: dz from X (dy = the skip gradient -> T), dx -> Y, the partials of conv 1's BN
                const spai_learner::Conv &c = L->convs[l2];
                const BnGrad bgv = bg_of(l2, T);
                const GradStats g = gs_of(l1);
                crc = launch_conv(X, c.co, W + c.wkd, nullptr, c.ci, Y, (int)B, false, st, nullptr, nullptr, &bgv, &g);
                wgrad_async(l2, L->a[l1].p, dzb_of(l2));
            }
            if (crc == SPAI_OK) {   // conv 1: dz from Y, dx accumulated into T = dL/d(block input)
                const spai_learner::Conv &c = L->convs[l1];
                const BnGrad bgv = bg_of(l1, nullptr);
                const GradStats g = gs_of(l1 - 1);
                crc = launch_conv(Y, c.co, W + c.wkd, nullptr, c.ci, T, (int)B, true, st, nullptr, nullptr, &bgv,
                                  l1 - 1 > 0 ? &g : nullptr);
                wgrad_async(l1, hin, dzb_of(l1));
            }
            float *nx = T;
            T = Y;
            Y = X;
            X = nx;
        }
        bn_conv_bwd(0, X, x_in, nullptr, false, nullptr);   // stem: no data gradient
    } else {
    bn_conv_bwd(val, L->d1.p, h, L->d0.p, true, nullptr);
    // residual blocks in reverse; d0 holds dL/d(block output)
    for (int k = L->blocks - 1; k >= 0; --k) {
        const int l1 = 1 + 2 * k, l2 = 2 + 2 * k;
        const float *hin = k == 0 ? L->a[0].p : L->a[l2 - 2].p;
        // BN2/conv2 backward: dt = d(out) * (out > 0) is the gradient of the pre-ReLU sum, shared
        // by BN2 and the skip path (k_bn_bwd also writes it to d1); conv2's input is a[l1]; its
        // data gradient overwrites d0 with dL/d(relu1 output)
        bn_conv_bwd(l2, L->d0.p, L->a[l1].p, L->d0.p, false, L->d1.p);
        // BN1/conv1 backward: da = d0 (gradient wrt relu1 output), mask a[l1]; its input is hin;
        // dgrad accumulates into d1 (= dt, the skip gradient) -> d(block input)
        bn_conv_bwd(l1, L->d0.p, hin, L->d1.p, true, nullptr);
        std::swap(L->d0, L->d1);   // d0 = dL/d(block input)
    }
    // stem: no data gradient
    bn_conv_bwd(0, L->d0.p, x_in, nullptr, false, nullptr);
    }
    // join: every weight gradient is in G before the reduction and Adam
    for (int k = 0; k < SPAI_WG_SIDE && crc == SPAI_OK; ++k)
        if (hipEventRecord(L->ev_wg_done[k], L->wg_stream[k]) != hipSuccess ||
            hipStreamWaitEvent(st, L->ev_wg_done[k], 0) != hipSuccess) {
            set_error("learner: event record/wait failed");
            crc = SPAI_ERR_DEVICE;
        }
    SPAI_TRY(crc);
    // ---------------- cross-rank reduction + Adam
    // The global step's gradient is the mean over every rank's samples: each rank
    // weights its own mean gradient by B / sum(B) (one 4-byte all-reduce first),
    // then the gradients are summed.  Exact for unequal per-rank batches; a 1-rank
    // communicator multiplies by 1 and reduces to a copy (bit-identical step).
    const float gscale = 1.0f;
    const bool dp = L->comm || L->host_ar;
    if (dp) {
        k_set1<<<1, 1, 0, st>>>(L->bsum.p, (float)B);
        SPAI_TRY(learner_allreduce(L, L->bsum.p, 1, st, "the batch sizes"));
        k_weight_grad<<<blocks_of(L->n_params), kThreads, 0, st>>>(G, L->n_params, (float)B, L->bsum.p);
        SPAI_TRY(learner_allreduce(L, G, L->n_params, st, "the gradients"));
    }
    k_adam<<<blocks_of(L->n_params), kThreads, 0, st>>>(P, G, L->m.p, L->v.p, L->n_params, gscale, L->cfg.lr,
                                                        L->cfg.beta1, L->cfg.beta2, L->cfg.eps, bc);
    if (dp) {   // average the BN running statistics so replicas stay identical
        const uint32_t nr = (uint32_t)L->run_idx.n;
        k_gather<<<blocks_of(nr), kThreads, 0, st>>>(P, L->run_idx.p, nr, L->run_buf.p);
        SPAI_TRY(learner_allreduce(L, L->run_buf.p, nr, st, "the BN running statistics"));
        k_scatter_scaled<<<blocks_of(nr), kThreads, 0, st>>>(L->run_buf.p, L->run_idx.p, nr, 1.0f / (float)L->world, P);
    }
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

// one step's batch and Adam bias corrections into the pinned staging half `stage`,
// one DMA of it, the step (eager, or the captured graph); launch-only
static int stage_and_enqueue(spai_learner *L, uint32_t B, const float *states, const float *policies,
                             const float *values, float *stage) {
    hipStream_t st = L->eng->stream;
    const size_t nin = (size_t)B * (3 * kCells + 8);
    L->step += 1;
    const double t = (double)L->step;
    stage[nin] = (float)(1.0 - std::pow((double)L->cfg.beta1, t));
    stage[nin + 1] = (float)std::sqrt(1.0 - std::pow((double)L->cfg.beta2, t));
    std::memcpy(stage, states, (size_t)B * 3 * kCells * 4);
    std::memcpy(stage + (size_t)B * 3 * kCells, policies, (size_t)B * 7 * 4);
    std::memcpy(stage + (size_t)B * (3 * kCells + 7), values, (size_t)B * 4);
    SPAI_HIP(hipMemcpyAsync(L->batch_in.p, stage, (nin + 2) * 4, hipMemcpyHostToDevice, st));
    const float *x_in = L->batch_in.p, *pi_in = x_in + (size_t)B * 3 * kCells, *z_in = pi_in + (size_t)B * 7;
    const float *bc = L->batch_in.p + nin;
    // SPAI_LEARNER_GRAPH=1 (measured variant): the step's launches captured once per
    // batch size into a hipGraph and replayed (single-rank learners only: the host
    // collective syncs inside the step).  Slower: the replay runs every kernel on one
    // queue, so the weight gradients lose their overlap with the data-gradient chain
    // (profiles/r05/learner/graph; round 2 likewise, profiles/r02/learner/graph_ab.txt)
    static const bool use_graph = [] {
        const char *v = std::getenv("SPAI_LEARNER_GRAPH");
        return v && std::atoi(v) != 0;
    }();
    if (use_graph && !L->comm && !L->host_ar) {
        if (!L->graph || L->graph_batch != B) {
            if (L->graph) (void)hipGraphExecDestroy(L->graph);
            L->graph = nullptr;
            hipGraph_t g = nullptr;
            SPAI_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            const int rc = enqueue_step(L, B, st, x_in, pi_in, z_in, bc);
            const hipError_t ec = hipStreamEndCapture(st, &g);
            if (rc != SPAI_OK || ec != hipSuccess) {   // a failed capture: free the partial graph before returning
                if (g) (void)hipGraphDestroy(g);
                SPAI_TRY(rc);
            }
            SPAI_CHECK(ec == hipSuccess && g, SPAI_ERR_DEVICE, "learner: step capture failed (%s)", hipGetErrorString(ec));
            const hipError_t ei = hipGraphInstantiate(&L->graph, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            SPAI_CHECK(ei == hipSuccess, SPAI_ERR_DEVICE, "learner: graph instantiation failed (%s)", hipGetErrorString(ei));
            L->graph_batch = B;
        }
        SPAI_HIP(hipGraphLaunch(L->graph, st));
    } else {
        SPAI_TRY(enqueue_step(L, B, st, x_in, pi_in, z_in, bc));
    }
    L->last_batch = B;
    return SPAI_OK;
}

// the fixed-order host sums of one step's loss terms
static void sum_loss(const float *terms, uint32_t B, float *loss3) {
    double lp = 0, lv = 0;
    for (uint32_t b = 0; b < B; ++b) {
        lp += terms[2 * b];
        lv += terms[2 * b + 1];
    }
    loss3[1] = (float)(lp / B);
    loss3[2] = (float)(lv / B);
    loss3[0] = loss3[1] + loss3[2];
}

int learner_train_batch(spai_learner *L, uint32_t B, const float *states, const float *policies, const float *values,
                        float *loss3) {
    SPAI_CHECK(B >= 1, SPAI_ERR_INVALID, "train_batch: empty batch");
    SPAI_TRY(learner_alloc_batch(L, B));
    hipStream_t st = L->eng->stream;
    SPAI_TRY(stage_and_enqueue(L, B, states, policies, values, L->stage));
    const size_t nin = (size_t)B * (3 * kCells + 8);
    float *terms = L->stage + nin + 2;   // the staged inputs were consumed by the DMA above (stream order)
    SPAI_HIP(hipMemcpyAsync(terms, L->loss_terms.p, (size_t)B * 2 * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    if (loss3) sum_loss(terms, B, loss3);
    return SPAI_OK;
}

// k consecutive train steps of B samples each (batch j = rows [j B, (j + 1) B) of
// the arrays), exactly k learner_train_batch calls, with one host synchronisation
// at the end instead of one per step: step j + 1's batch is staged into the other
// pinned half while step j runs (the half is refilled once its previous upload is
// done), and every step's loss terms come back by a stream-ordered copy.
// losses[3 j ..] = step j's {total, policy, value}.
int learner_train_batches(spai_learner *L, uint32_t k, uint32_t B, const float *states, const float *policies,
                          const float *values, float *losses) {
    SPAI_CHECK(B >= 1 && k >= 1, SPAI_ERR_INVALID, "train_batches: need k >= 1 batches of B >= 1 samples");
    SPAI_TRY(learner_alloc_batch(L, B));
    hipStream_t st = L->eng->stream;
    const size_t need = (size_t)k * B * 2;
    if (L->terms_host_n < need) {
        if (L->terms_host) (void)hipHostFree(L->terms_host);
        L->terms_host = nullptr;
        L->terms_host_n = 0;
        SPAI_HIP(hipHostMalloc((void **)&L->terms_host, need * sizeof(float), hipHostMallocDefault));
        L->terms_host_n = need;
    }
    for (uint32_t j = 0; j < k; ++j) {
        float *half = (j & 1) ? L->stage_b : L->stage;
        if (j >= 2) SPAI_HIP(hipEventSynchronize(L->stage_ev[j & 1]));   // its previous upload is done
        SPAI_TRY(stage_and_enqueue(L, B, states + (size_t)j * B * 3 * kCells, policies + (size_t)j * B * 7,
                                   values + (size_t)j * B, half));
        SPAI_HIP(hipEventRecord(L->stage_ev[j & 1], st));   // after the upload (and the step) in stream order
        SPAI_HIP(hipMemcpyAsync(L->terms_host + (size_t)j * B * 2, L->loss_terms.p, (size_t)B * 2 * 4,
                                hipMemcpyDeviceToHost, st));
    }
    SPAI_HIP(hipStreamSynchronize(st));
    if (losses)
        for (uint32_t j = 0; j < k; ++j) sum_loss(L->terms_host + (size_t)j * B * 2, B, losses + 3 * j);
    return SPAI_OK;
}

// Model::train (model/mod.rs:100-149): a fresh Adam (the reference builds the
// optimizer inside train), one permutation of the n samples (Tensor::randperm,
// here a Philox-keyed Fisher-Yates), then `epochs` passes of ceil(n / batch)
// train steps over the permuted samples (the last batch may be short).
int learner_train_epochs(spai_learner *L, uint32_t n, const float *states, const float *policies,
                         const float *values, uint32_t epochs, uint32_t batch, uint64_t seed, float *loss3) {
    SPAI_CHECK(n >= 1 && batch >= 1, SPAI_ERR_INVALID, "train: need samples and a batch size");
    hipStream_t st = L->eng->stream;
    SPAI_HIP(hipMemsetAsync(L->m.p, 0, L->n_params * 4, st));   // Adam::default().build(..) per call
    SPAI_HIP(hipMemsetAsync(L->v.p, 0, L->n_params * 4, st));
    L->step = 0;
    std::vector<uint32_t> perm;
    choose_multiple(n, n, seed, 0x7EA1Bull, perm);   // a full random permutation
    std::vector<float> s((size_t)batch * 126), p((size_t)batch * 7), v(batch);
    const uint32_t nb = (n + batch - 1) / batch;
    for (uint32_t ep = 0; ep < epochs; ++ep)
        for (uint32_t b = 0; b < nb; ++b) {
            const uint32_t lo = b * batch, m = std::min(batch, n - lo);
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t j = perm[lo + i];
                memcpy(&s[(size_t)i * 126], states + (size_t)j * 126, 126 * 4);
                memcpy(&p[(size_t)i * 7], policies + (size_t)j * 7, 7 * 4);
                v[i] = values[j];
            }
            SPAI_TRY(learner_train_batch(L, m, s.data(), p.data(), v.data(), loss3));
        }
    return SPAI_OK;
}

int learner_params(spai_learner *L, float *params, size_t n, bool grads) {
    SPAI_CHECK(n == L->n_params, SPAI_ERR_INVALID, "expected %zu params, got %zu", L->n_params, n);
    hipStream_t st = L->eng->stream;
    SPAI_HIP(hipMemcpyAsync(params, grads ? L->g.p : L->p.p, n * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

// the latest step's post-ReLU activations of conv layer `layer` (construction
// order: stem, 2*blocks residual convs, policy head, value head), [B][co][6][7]
int learner_activation(spai_learner *L, int layer, float *out, size_t n) {
    SPAI_CHECK(layer >= 0 && (size_t)layer < L->convs.size(), SPAI_ERR_INVALID, "layer %d of %zu", layer,
               L->convs.size());
    SPAI_CHECK(L->last_batch > 0, SPAI_ERR_INVALID, "no train step yet");
    const size_t want = (size_t)L->last_batch * L->convs[layer].co * kCells;
    SPAI_CHECK(n == want, SPAI_ERR_INVALID, "expected %zu activations, got %zu", want, n);
    hipStream_t st = L->eng->stream;
    SPAI_HIP(hipMemcpyAsync(out, L->a[layer].p, n * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

int learner_set_comm(spai_learner *L, int rank, int world, const uint8_t *id) {
    SPAI_CHECK(world >= 1 && rank >= 0 && rank < world, SPAI_ERR_INVALID, "bad rank %d / world %d", rank, world);
    if (L->comm) {
        (void)ncclCommDestroy((ncclComm_t)L->comm);
        L->comm = nullptr;
    }
    L->host_ar = nullptr;   // an RCCL communicator (or none) replaces a host collective
    L->host_ar_user = nullptr;
    L->rank = rank;
    L->world = world;
    if (!id) return SPAI_OK;   // world == 1 without an id: no communicator
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == SPAI_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(uid.internal, id, SPAI_COMM_ID_BYTES);
    SPAI_HIP(hipSetDevice(L->eng->device));
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, world, uid, rank);
    SPAI_CHECK(r == ncclSuccess, SPAI_ERR_DEVICE, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
    L->comm = c;
    return SPAI_OK;
}

// weight refresh of data-parallel replicas: every rank's parameters (BN running
// statistics included) become rank `root`'s, by one RCCL broadcast over xGMI
int learner_broadcast(spai_learner *L, int root) {
    SPAI_CHECK(root >= 0 && root < L->world, SPAI_ERR_INVALID, "broadcast root %d outside world %d", root, L->world);
    hipStream_t st = L->eng->stream;
    if (L->host_ar) {   // rank root's values plus -0.0 from every other rank: x + -0.0 == x exactly
        SPAI_HIP(hipStreamSynchronize(st));
        if (L->rank == root) {
            SPAI_HIP(hipMemcpy(L->host_buf, L->p.p, L->n_params * 4, hipMemcpyDeviceToHost));
        } else {
            for (size_t i = 0; i < L->n_params; ++i) L->host_buf[i] = -0.0f;
        }
        const int r = L->host_ar(L->host_ar_user, L->host_buf, L->n_params);
        SPAI_CHECK(r == 0, SPAI_ERR_DEVICE, "host all-reduce of the parameters failed (%d)", r);
        SPAI_HIP(hipMemcpy(L->p.p, L->host_buf, L->n_params * 4, hipMemcpyHostToDevice));
        return SPAI_OK;
    }
    if (!L->comm) return SPAI_OK;   // no communicator: a single replica
    if (ncclBroadcast(L->p.p, L->p.p, L->n_params, ncclFloat32, root, (ncclComm_t)L->comm, st) != ncclSuccess) {
        set_error("ncclBroadcast of the parameters failed");
        return SPAI_ERR_DEVICE;
    }
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

// host collective in place of RCCL (the same step, each all-reduce staged through pinned memory)
int learner_set_host_comm(spai_learner *L, int rank, int world, spai_host_allreduce fn, void *user) {
    SPAI_CHECK(world >= 1 && rank >= 0 && rank < world, SPAI_ERR_INVALID, "bad rank %d / world %d", rank, world);
    if (L->comm) {
        (void)ncclCommDestroy((ncclComm_t)L->comm);
        L->comm = nullptr;
    }
    // NULL or world 1 drops the collective (spai.h): a 1-rank reduction is the
    // identity, and staging it through host memory would cost the step its
    // launch-only property (three syncs and callbacks per step)
    const bool on = fn && world > 1;
    L->rank = on ? rank : 0;
    L->world = on ? world : 1;
    L->host_ar = on ? fn : nullptr;
    L->host_ar_user = on ? user : nullptr;
    if (!on) return SPAI_OK;
    const size_t need = std::max(L->n_params, L->run_idx.n);
    if (L->host_buf_n < need) {
        if (L->host_buf) (void)hipHostFree(L->host_buf);
        L->host_buf = nullptr;
        L->host_buf_n = 0;
        if (hipHostMalloc((void **)&L->host_buf, need * sizeof(float), hipHostMallocDefault) != hipSuccess) {
            L->host_buf = nullptr;
            L->host_ar = nullptr;
            L->world = 1;
            set_error("learner: pinned host-collective buffer allocation failed");
            return SPAI_ERR_DEVICE;
        }
        L->host_buf_n = need;
    }
    return SPAI_OK;
}

int comm_unique_id(uint8_t *id) {
    ncclUniqueId uid;
    const ncclResult_t r = ncclGetUniqueId(&uid);
    SPAI_CHECK(r == ncclSuccess, SPAI_ERR_DEVICE, "ncclGetUniqueId failed: %s", ncclGetErrorString(r));
    memcpy(id, uid.internal, SPAI_COMM_ID_BYTES);
    return SPAI_OK;
}

}  // namespace spai

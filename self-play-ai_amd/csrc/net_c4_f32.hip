// net_c4_f32.hip — the Connect4 ResNet forward in fp32 (spai_net_create with
// SPAI_DTYPE_F32): the reference's own arithmetic, for parity work.
//
// Reference: model/mod.rs:152-184 (stem conv3x3 + BN + ReLU, residual blocks
// relu(x + BN(conv(relu(BN(conv(x)))))) ), model/connect_four.rs:50-81 (policy
// head conv 64->32 + BN + ReLU + flatten + linear 1344->7; value head conv
// 64->3 + BN + ReLU + flatten + linear 126->1 + tanh), model/mod.rs:62-93
// (softmax(-1), then mask_invalid_actions).  The reference computes all of this
// in fp32 through libtorch (model/mod.rs:36-98).
//
// Every output element is summed in ONE fixed order — bias first, then input
// channel, kernel row, kernel column (the loop nest of oracle/spai_oracle.c
// conv3x3) — with separate multiply and add (-ffp-contract=off), BatchNorm
// unfolded as ((x - mean) * inv) * gamma + beta with inv = 1 / sqrt(var + eps)
// computed on the host, and the linears summed sequentially over the NCHW
// flatten.  Conv and linear outputs are therefore bit-identical to the CPU
// oracle's; only expf / tanhf (device libm vs glibc) may differ in the last ulp.
//
// Layout: one workgroup (4 waves) per position.  Activations live in LDS as
// fp32 [72 padded cells][64 channels] on an 8 x 9 grid with a zero border, so
// a 3x3 tap is a constant offset and an out-of-board tap adds an exact +-0
// (the oracle skips it; x + 0 == x).  Thread t owns output channel t & 63 at
// cells (t >> 6) + 4k: a wave's 64 lanes read the same activation (LDS
// broadcast) and 64 consecutive weights (one coalesced load, weights stored
// [ci][tap][co]).  Throughput is not the point of this kernel; the bf16 MFMA
// kernel (net_c4.hip) is the production path.
#include <cmath>
#include <vector>

#include "spai_internal.h"

namespace spai {
namespace {

constexpr int kHid = 64;
constexpr int kThreads = 256;
constexpr int kGridW = 9, kGridCells = 72;      // padded 8 x 9 grid
constexpr int kCellsPerThread = 11;             // ceil(42 / 4)
constexpr int kHeadCo = 35;                     // 32 policy + 3 value channels
constexpr int kPolIn = 32 * c4::kCells, kValIn = 3 * c4::kCells;

// LDS carve (floats)
constexpr int kA = 0;                           // [72][64]
constexpr int kB = kA + kGridCells * kHid;      // [72][64]
constexpr int kX = kB + kGridCells * kHid;      // input planes [72][4]
constexpr int kH = kX + kGridCells * 4;         // head features, NCHW [35][42]
constexpr int kOut = kH + kHeadCo * c4::kCells; // logits [7] + value pre-activation [1]
constexpr int kLdsFloats = kOut + 8;

// per-layer device views: weights [ci][9][co], BN [5][co] = conv bias, mean, inv, gamma, beta
struct F32Params {
    const float *stem_w, *stem_bn;
    const float *res_w, *res_bn;   // layer l at + l * (64*9*64) / + l * (5*64)
    const float *head_w, *head_bn; // co 0..31 policy, 32..34 value
    const float *pol_w, *pol_b;    // [7][1344], [7]
    const float *val_w, *val_b;    // [126], [1]
    int blocks;
};

__device__ __forceinline__ int padded(int cell) {
    const int h = cell / c4::kCols, w = cell - h * c4::kCols;
    return (h + 1) * kGridW + (w + 1);
}

// out-of-line on purpose: one copy per (CI, CO, MODE), not one per call site
// MODE 0: relu(BN(conv)) -> out[cell][co]
// MODE 1: relu(out + BN(conv)) -> out (residual; `out` holds the block input)
// MODE 2: relu(BN(conv)) -> head features out[co*42 + cell]
template <int CI, int PITCH, int CO, int MODE>
__device__ __noinline__ void conv_f32(const float *in, float *out, const float *__restrict__ W,
                                      const float *__restrict__ bn, int tid) {
    const int co = tid & 63, g = tid >> 6;
    if (co >= CO) return;
    float acc[kCellsPerThread];
    int pc[kCellsPerThread];
    const float bias = bn[co];
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
        const int cell = g + 4 * k;
        pc[k] = cell < c4::kCells ? padded(cell) : padded(0);
        acc[k] = bias;
    }
    for (int i = 0; i < CI; ++i) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const float wv = W[(i * 9 + tap) * CO + co];
            const int off = (tap / 3 - 1) * kGridW + (tap % 3 - 1);
#pragma unroll
            for (int k = 0; k < kCellsPerThread; ++k) acc[k] = acc[k] + wv * in[(pc[k] + off) * PITCH + i];
        }
    }
    const float mu = bn[CO + co], inv = bn[2 * CO + co], gm = bn[3 * CO + co], be = bn[4 * CO + co];
#pragma unroll
    for (int k = 0; k < kCellsPerThread; ++k) {
        const int cell = g + 4 * k;
        if (cell >= c4::kCells) continue;
        float v = (acc[k] - mu) * inv * gm + be;
        if (MODE == 1) v = out[pc[k] * kHid + co] + v;
        if (v < 0.0f) v = 0.0f;
        if (MODE == 2) out[co * c4::kCells + cell] = v;
        else out[pc[k] * kHid + co] = v;
    }
}

// One position per workgroup.  FROM_X: Net::forward on x [n][3][6][7];
// otherwise the leaf bitboards (encoding fused, connect_four.rs:242-259).
template <bool FROM_X>
__global__ __launch_bounds__(kThreads) void k_forward_f32(const uint32_t *__restrict__ count_ptr, uint32_t count_imm,
                                                          const uint64_t *__restrict__ mine,
                                                          const uint64_t *__restrict__ theirs,
                                                          const float *__restrict__ x, F32Params P,
                                                          float *__restrict__ priors, float *__restrict__ value,
                                                          float *__restrict__ logits) {
    __shared__ float s[kLdsFloats];
    const uint32_t count = count_ptr ? *count_ptr : count_imm;
    const uint32_t slot = blockIdx.x;
    if (slot >= count) return;
    const int tid = threadIdx.x;
    for (int i = tid; i < kX + kGridCells * 4; i += kThreads) s[i] = 0.0f;   // A, B, X incl. the zero border
    __syncthreads();
    uint64_t m = 0, t = 0;
    if (!FROM_X) {
        m = mine[slot];
        t = theirs[slot];
    }
    if (tid < 3 * c4::kCells) {
        const int ch = tid / c4::kCells, cell = tid - ch * c4::kCells;
        float v;
        if (FROM_X) {
            v = x[(size_t)slot * 3 * c4::kCells + tid];
        } else {
            const int r = cell / c4::kCols, c = cell - r * c4::kCols, b = c * 7 + r;
            const bool mi = (m >> b) & 1ull, th = (t >> b) & 1ull;
            v = (ch == 0 ? mi : ch == 1 ? th : !(mi || th)) ? 1.0f : 0.0f;
        }
        s[kX + padded(cell) * 4 + ch] = v;
    }
    __syncthreads();
    conv_f32<3, 4, kHid, 0>(s + kX, s + kA, P.stem_w, P.stem_bn, tid);
    __syncthreads();
    constexpr size_t kLw = (size_t)kHid * 9 * kHid, kLb = 5 * kHid;
    for (int b = 0; b < P.blocks; ++b) {
        conv_f32<kHid, kHid, kHid, 0>(s + kA, s + kB, P.res_w + (2 * b) * kLw, P.res_bn + (2 * b) * kLb, tid);
        __syncthreads();
        conv_f32<kHid, kHid, kHid, 1>(s + kB, s + kA, P.res_w + (2 * b + 1) * kLw, P.res_bn + (2 * b + 1) * kLb, tid);
        __syncthreads();
    }
    conv_f32<kHid, kHid, kHeadCo, 2>(s + kA, s + kH, P.head_w, P.head_bn, tid);
    __syncthreads();
    // linears, summed sequentially over the NCHW flatten (oracle forward_one)
    if (tid < c4::kActions) {
        float acc = 0.0f;
        const float *w = P.pol_w + (size_t)tid * kPolIn;
        for (int i = 0; i < kPolIn; ++i) acc = acc + s[kH + i] * w[i];
        s[kOut + tid] = acc + P.pol_b[tid];
    } else if (tid == 64) {   // another wave
        float acc = 0.0f;
        for (int i = 0; i < kValIn; ++i) acc = acc + s[kH + kPolIn + i] * P.val_w[i];
        s[kOut + 7] = acc + P.val_b[0];
    }
    __syncthreads();
    if (tid == 0) {
        float lg[c4::kActions];
        for (int a = 0; a < c4::kActions; ++a) lg[a] = s[kOut + a];
        value[slot] = tanhf(s[kOut + 7]);
        if (logits)
            for (int a = 0; a < c4::kActions; ++a) logits[(size_t)slot * c4::kActions + a] = lg[a];
        if (priors) {   // softmax(-1) as the oracle's or_predict, then mask_invalid_actions
            float mx = lg[0];
            for (int a = 1; a < c4::kActions; ++a) mx = lg[a] > mx ? lg[a] : mx;
            float e[c4::kActions], sum = 0.0f;
            for (int a = 0; a < c4::kActions; ++a) {
                e[a] = expf(lg[a] - mx);
                sum = sum + e[a];
            }
            for (int a = 0; a < c4::kActions; ++a) e[a] = e[a] / sum;
            float out[c4::kActions];
            c4::mask_renorm(e, c4::open_columns(m | t), out);
            for (int a = 0; a < c4::kActions; ++a) priors[(size_t)slot * kPriorStride + a] = out[a];
            priors[(size_t)slot * kPriorStride + 7] = 0.0f;
        }
    }
}

F32Params params_f32(const spai_net *n) {
    const float *b = n->f32.p;
    const size_t nres = (size_t)2 * n->blocks;
    F32Params P;
    size_t o = 0;
    P.stem_w = b + o; o += (size_t)3 * 9 * kHid;
    P.stem_bn = b + o; o += 5 * kHid;
    P.res_w = b + o; o += nres * kHid * 9 * kHid;
    P.res_bn = b + o; o += nres * 5 * kHid;
    P.head_w = b + o; o += (size_t)kHid * 9 * kHeadCo;
    P.head_bn = b + o; o += 5 * kHeadCo;
    P.pol_w = b + o; o += (size_t)7 * kPolIn;
    P.pol_b = b + o; o += 7;
    P.val_w = b + o; o += kValIn;
    P.val_b = b + o;
    P.blocks = n->blocks;
    return P;
}

}  // namespace

// params in construction order (net_c4.hip net_create) -> the flat fp32 device
// buffer params_f32 reads: per conv W^T [ci][9][co] and BN [5][co]
int net_create_f32(spai_net *n, const float *params) {
    std::vector<float> buf;
    const float *p = params;
    // take conv (w [co][ci][3][3], b [co], BN [4][co]) into W^T and BN rows; co_off places
    // the head's value channels after the policy channels of one combined layer
    auto take = [&](int ci, int co, std::vector<float> &w, std::vector<float> &bn, int co_total, int co_off) {
        const float *cw = p, *cb = p + (size_t)co * ci * 9, *g = cb + co, *be = g + co, *mu = be + co, *var = mu + co;
        for (int o = 0; o < co; ++o) {
            for (int i = 0; i < ci; ++i)
                for (int tap = 0; tap < 9; ++tap)
                    w[((size_t)i * 9 + tap) * co_total + co_off + o] = cw[((size_t)o * ci + i) * 9 + tap];
            bn[0 * co_total + co_off + o] = cb[o];
            bn[1 * co_total + co_off + o] = mu[o];
            bn[2 * co_total + co_off + o] = 1.0f / sqrtf(var[o] + 1e-5f);   // oracle bn_relu
            bn[3 * co_total + co_off + o] = g[o];
            bn[4 * co_total + co_off + o] = be[o];
        }
        p += (size_t)co * ci * 9 + co + 4 * co;
    };
    auto append = [&](const std::vector<float> &v) { buf.insert(buf.end(), v.begin(), v.end()); };
    std::vector<float> w((size_t)3 * 9 * kHid), bn(5 * kHid);
    take(3, kHid, w, bn, kHid, 0);
    append(w);
    append(bn);
    const int nres = 2 * n->blocks;
    std::vector<float> rw((size_t)nres * kHid * 9 * kHid), rbn((size_t)nres * 5 * kHid);
    for (int l = 0; l < nres; ++l) {
        std::vector<float> lw((size_t)kHid * 9 * kHid), lbn(5 * kHid);
        take(kHid, kHid, lw, lbn, kHid, 0);
        std::copy(lw.begin(), lw.end(), rw.begin() + (size_t)l * lw.size());
        std::copy(lbn.begin(), lbn.end(), rbn.begin() + (size_t)l * lbn.size());
    }
    append(rw);
    append(rbn);
    std::vector<float> hw((size_t)kHid * 9 * kHeadCo), hbn(5 * kHeadCo);
    take(kHid, 32, hw, hbn, kHeadCo, 0);                  // policy head conv
    const float *pol = p;
    p += (size_t)7 * kPolIn + 7;
    take(kHid, 3, hw, hbn, kHeadCo, 32);                  // value head conv
    const float *val = p;
    append(hw);
    append(hbn);
    buf.insert(buf.end(), pol, pol + (size_t)7 * kPolIn + 7);
    buf.insert(buf.end(), val, val + kValIn + 1);
    SPAI_TRY(n->f32.alloc(buf.size()));
    SPAI_HIP(hipMemcpy(n->f32.p, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
    return SPAI_OK;
}

// `count` (device scalar, or count_imm when null) positions; the grid covers max_n
int net_f32_launch(spai_net *n, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint64_t *mine,
                   const uint64_t *theirs, const float *x, float *priors, float *value, float *logits) {
    if (!max_n) return SPAI_OK;
    if (x)
        k_forward_f32<true><<<max_n, kThreads, 0, st>>>(d_count, max_n, nullptr, nullptr, x, params_f32(n), priors,
                                                        value, logits);
    else
        k_forward_f32<false><<<max_n, kThreads, 0, st>>>(d_count, max_n, mine, theirs, nullptr, params_f32(n),
                                                         priors, value, logits);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

}  // namespace spai

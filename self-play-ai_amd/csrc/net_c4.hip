// net_c4.hip — Connect4 policy/value ResNet forward as ONE fused HIP kernel.
//
// Reference: model/mod.rs:152-184 (stem conv3x3+BN+ReLU, residual blocks
// relu(x + BN(conv(relu(BN(conv(x)))))) ), model/connect_four.rs:50-81 (policy
// head conv3x3 64->32 + BN + ReLU + flatten + linear 1344->7; value head conv3x3
// 64->3 + BN + ReLU + flatten + linear 126->1 + tanh), model/mod.rs:62-93
// (softmax(-1), then mask_invalid_actions).
//
// MI355X design:
//  * one workgroup = 4 waves = S = 8 positions' whole forward.  The 8 x 42
//    activations stay in LDS for all layers (bf16, [position][64 channels],
//    128-B rows with the 16-B chunk index XOR-swizzled by row&7 so the
//    ds_read_b128 B-fragment reads are bank-conflict free); only weights are
//    read from global memory (L2-resident, 0.9 MB for 6x64).
//  * every 3x3 conv is an implicit GEMM on v_mfma_f32_16x16x32_bf16:
//    D[co][pos] = sum_k W[co][k] * X[k][pos], k = tap*64 + ci.  A = weights,
//    pre-packed on the host in exact fragment order (one 1 KiB coalesced
//    global_load_dwordx4 per wave per 16x32 fragment), BN folded in;
//    B = activations from LDS; out-of-board taps read a zero row.
//  * the stem builds its input planes [mine, theirs, empty] straight from the
//    leaf bitboards (encoding fused, connect_four.rs:242-259).
//  * epilogues fuse bias, residual add and ReLU; the head conv writes fp32,
//    the two linears, tanh, softmax and the legal-move mask run in-kernel.
//  * wave w owns position tiles [6,5,5,5] of the 21 16-position tiles and all
//    4 co tiles (24/20 accumulators).
// Algorithmic FLOPs per position (6 blocks x 64): 39,016,572.
#include <cmath>
#include <cstring>

#include "spai_internal.h"

namespace spai {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kHid = 64;
constexpr int kS = 8;                      // positions per workgroup
constexpr int kP = kS * c4::kCells;        // 336 board cells per workgroup
constexpr int kPT = kP / 16;               // 21 position tiles
constexpr int kWaves = 4;
constexpr int kThreads = kWaves * 64;
constexpr int kKStepsRes = 18;             // 576 / 32
constexpr int kHeadC = 35;                 // 32 policy + 3 value channels
constexpr int kHeadCT = 3;                 // 48 padded co
constexpr int kPolIn = 32 * c4::kCells;    // 1344
constexpr int kValIn = 3 * c4::kCells;     // 126

// LDS carve (bytes)
constexpr int kZ = 0;                      // 128 B of zeros (out-of-board taps)
constexpr int kX = 128;                    // [336][128 B] bf16 activations
constexpr int kY = kX + kP * 128;          // second activation buffer
constexpr int kH = kY;                     // fp32 head conv output [8][35][42] overlays Y
constexpr int kHBytes = kS * kHeadC * c4::kCells * 4;
constexpr int kB = kH + kHBytes;           // 8 x (mine, theirs)
constexpr int kL = kB + kS * 16;           // logits scratch [8][8] f32
constexpr int kLdsBytes = kL + kS * 8 * 4;
static_assert(kY + kP * 128 <= kB, "heads overlay");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct NetParams {
    const uint4 *w_stem;   // [4 ct][64 lanes] 16 B fragments
    const uint4 *w_res;    // [2*blocks][18 ks][4 ct][64]
    const uint4 *w_head;   // [18][3][64]
    const float *b_stem;   // [64]
    const float *b_res;    // [2*blocks][64]
    const float *b_head;   // [48]
    const float *w_pol;    // [7][1344]
    const float *b_pol;    // [7]
    const float *w_val;    // [126]
    const float *b_val;    // [1]
    int blocks;
};

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    __bf16 ha = (__bf16)a, hb = (__bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

// byte offset of the 16-B channel chunk `c` (0..7) of activation row `r` in a buffer at `base`
__device__ __forceinline__ int act_off(int base, int r, int c) { return base + r * 128 + ((c ^ (r & 7)) << 4); }

// implicit-GEMM 3x3 conv over LDS activations at `in_base`: acc[t][ct] += W[ct] * X[tile t]
template <int NT, int CT>
__device__ __forceinline__ void conv_mfma(const uint8_t *smem, int in_base, const uint4 *__restrict__ w, int t0,
                                          int lane, f32x4 (&acc)[NT][CT]) {
    const int col = lane & 15, q = lane >> 4;
    int pos[NT], ph[NT], pw[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        int p = (t0 + t) * 16 + col;
        int cell = p % c4::kCells;
        pos[t] = p;
        ph[t] = cell / c4::kCols;
        pw[t] = cell - ph[t] * c4::kCols;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 a_cur[2][CT];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int c = 0; c < CT; ++c) a_cur[hf][c] = w[(hf * CT + c) * 64 + lane];

#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        const int dh = tap / 3 - 1, dw = tap % 3 - 1;
        uint4 a_nxt[2][CT];
        if (tap < 8) {
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int c = 0; c < CT; ++c) a_nxt[hf][c] = w[(((tap + 1) * 2 + hf) * CT + c) * 64 + lane];
        }
        int rows[NT];
        bool ok[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            ok[t] = (unsigned)(ph[t] + dh) < (unsigned)c4::kRows && (unsigned)(pw[t] + dw) < (unsigned)c4::kCols;
            rows[t] = pos[t] + dh * c4::kCols + dw;
        }
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            uint4 b[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                int off = ok[t] ? act_off(in_base, rows[t], hf * 4 + q) : kZ + (q << 4);
                b[t] = *(const uint4 *)(smem + off);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int c = 0; c < CT; ++c)
                    acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a_cur[hf][c]), as_bf16x8(b[t]),
                                                                       acc[t][c], 0, 0, 0);
        }
        if (tap < 8) {
#pragma unroll
            for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                for (int c = 0; c < CT; ++c) a_cur[hf][c] = a_nxt[hf][c];
        }
    }
}

// epilogue for a 64-channel bf16 output: relu(acc + bias [+ residual]) -> LDS
template <int NT>
__device__ __forceinline__ void epilogue_act(uint8_t *smem, int out_base, const float *__restrict__ bias, int t0,
                                             int lane, bool residual, f32x4 (&acc)[NT][4]) {
    const int col = lane & 15, q = lane >> 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int co0 = c * 16 + 4 * q;
        const float4 b = *(const float4 *)(bias + co0);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int p = (t0 + t) * 16 + col;
            const int off = act_off(out_base, p, co0 >> 3) + ((co0 & 4) << 1);
            float v0 = acc[t][c][0] + b.x, v1 = acc[t][c][1] + b.y, v2 = acc[t][c][2] + b.z, v3 = acc[t][c][3] + b.w;
            if (residual) {
                uint2 r = *(const uint2 *)(smem + off);
                v0 += __builtin_bit_cast(float, r.x << 16);
                v1 += __builtin_bit_cast(float, r.x & 0xFFFF0000u);
                v2 += __builtin_bit_cast(float, r.y << 16);
                v3 += __builtin_bit_cast(float, r.y & 0xFFFF0000u);
            }
            v0 = fmaxf(v0, 0.f);
            v1 = fmaxf(v1, 0.f);
            v2 = fmaxf(v2, 0.f);
            v3 = fmaxf(v3, 0.f);
            *(uint2 *)(smem + off) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        }
    }
}

// stem: B operand = the 27 input planes x taps built in registers, one k-step
template <int NT, bool FROM_X>
__device__ __forceinline__ void stem(uint8_t *smem, const NetParams &P, const float *__restrict__ x, int base_slot,
                                     int valid, int t0, int lane) {
    const int col = lane & 15, q = lane >> 4;
    const uint64_t *bb = (const uint64_t *)(smem + kB);
    uint4 a[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = P.w_stem[c * 64 + lane];
    f32x4 acc[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int p = (t0 + t) * 16 + col;
        const int s = p / c4::kCells, cell = p - s * c4::kCells;
        const int h = cell / c4::kCols, wc = cell - h * c4::kCols;
        const uint64_t mine = bb[2 * s], theirs = bb[2 * s + 1], occ = mine | theirs;
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int kk = 8 * q + j;
            float v = 0.f;
            if (kk < 27) {
                const int tap = kk / 3, ch = kk - tap * 3;
                const int hh = h + tap / 3 - 1, ww = wc + tap % 3 - 1;
                if ((unsigned)hh < (unsigned)c4::kRows && (unsigned)ww < (unsigned)c4::kCols) {
                    if (FROM_X) {
                        v = (s < valid) ? x[((size_t)(base_slot + s) * 3 + ch) * c4::kCells + hh * c4::kCols + ww] : 0.f;
                    } else {
                        const int bit = ww * 7 + hh;
                        const uint64_t src = ch == 0 ? mine : ch == 1 ? theirs : ~occ;
                        v = (float)((src >> bit) & 1ull);
                    }
                }
            }
            e[j] = __builtin_bit_cast(uint16_t, (__bf16)v);
        }
        uint4 bv = make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16, e[4] | (uint32_t)e[5] << 16,
                              e[6] | (uint32_t)e[7] << 16);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
            acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[c]), as_bf16x8(bv), acc[t][c], 0, 0, 0);
        }
    }
    epilogue_act<NT>(smem, kX, P.b_stem, t0, lane, false, acc);
}

template <int NT>
__device__ __forceinline__ void res_layer(uint8_t *smem, const NetParams &P, int layer, int t0, int lane) {
    f32x4 acc[NT][4];
    const bool second = layer & 1;   // conv1: X -> Y ; conv2: Y -> X with residual X
    conv_mfma<NT, 4>(smem, second ? kY : kX, P.w_res + (size_t)layer * kKStepsRes * 4 * 64, t0, lane, acc);
    epilogue_act<NT>(smem, second ? kX : kY, P.b_res + layer * kHid, t0, lane, second, acc);
}

template <int NT>
__device__ __forceinline__ void head_layer(uint8_t *smem, const NetParams &P, int t0, int lane) {
    f32x4 acc[NT][kHeadCT];
    conv_mfma<NT, kHeadCT>(smem, kX, P.w_head, t0, lane, acc);
    const int col = lane & 15, q = lane >> 4;
    float *H = (float *)(smem + kH);
#pragma unroll
    for (int c = 0; c < kHeadCT; ++c) {
        const int co0 = c * 16 + 4 * q;
        const float4 b = *(const float4 *)(P.b_head + co0);
        const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int p = (t0 + t) * 16 + col;
            const int s = p / c4::kCells, cell = p - s * c4::kCells;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + r;
                if (co < kHeadC) H[(s * kHeadC + co) * c4::kCells + cell] = fmaxf(acc[t][c][r] + bv[r], 0.f);
            }
        }
    }
}

template <bool FROM_X>
__global__ __launch_bounds__(kThreads) void k_forward(const uint32_t *__restrict__ count_ptr, uint32_t count_imm,
                                                      const uint64_t *__restrict__ mine, const uint64_t *__restrict__ theirs,
                                                      const float *__restrict__ x, NetParams P, float *__restrict__ priors,
                                                      float *__restrict__ value, float *__restrict__ logits) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kLdsBytes];
    const uint32_t count = count_ptr ? *count_ptr : count_imm;
    const int base = blockIdx.x * kS;
    if (base >= (int)count) return;
    const int valid = min(kS, (int)count - base);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    if (tid < 32) ((uint32_t *)(smem + kZ))[tid] = 0u;
    if (tid < kS) {
        uint64_t m = 0, t = 0;
        if (!FROM_X && tid < valid) {
            m = mine[base + tid];
            t = theirs[base + tid];
        }
        ((uint64_t *)(smem + kB))[2 * tid] = m;
        ((uint64_t *)(smem + kB))[2 * tid + 1] = t;
    }
    __syncthreads();

    // position tiles per wave: [0,6) [6,11) [11,16) [16,21)
    const int t0 = wave == 0 ? 0 : 1 + 5 * wave;
    if (wave == 0) stem<6, FROM_X>(smem, P, x, base, valid, t0, lane);
    else stem<5, FROM_X>(smem, P, x, base, valid, t0, lane);
    __syncthreads();
    for (int layer = 0; layer < 2 * P.blocks; ++layer) {
        if (wave == 0) res_layer<6>(smem, P, layer, t0, lane);
        else res_layer<5>(smem, P, layer, t0, lane);
        __syncthreads();
    }
    if (wave == 0) head_layer<6>(smem, P, t0, lane);
    else head_layer<5>(smem, P, t0, lane);
    __syncthreads();

    // linears: 64 (position, output) pairs x 4 partial sums; output 7 = value
    {
        const float *H = (const float *)(smem + kH);
        const int pair = tid >> 2, part = tid & 3;
        const int s = pair >> 3, o = pair & 7;
        float acc = 0.f;
        if (o < c4::kActions) {
            const float *h = H + s * kHeadC * c4::kCells;
            const float *wr = P.w_pol + o * kPolIn;
            for (int i = part * (kPolIn / 4); i < (part + 1) * (kPolIn / 4); ++i) acc += h[i] * wr[i];
        } else {
            const float *h = H + (s * kHeadC + 32) * c4::kCells;
            for (int i = part; i < kValIn; i += 4) acc += h[i] * P.w_val[i];
        }
        acc += __shfl_xor(acc, 1, 4);
        acc += __shfl_xor(acc, 2, 4);
        if (part == 0) ((float *)(smem + kL))[s * 8 + o] = acc;
    }
    __syncthreads();
    if (tid < valid) {
        const float *L = (const float *)(smem + kL) + tid * 8;
        const int slot = base + tid;
        float lg[c4::kActions];
        float mx = -INFINITY;
#pragma unroll
        for (int a = 0; a < c4::kActions; ++a) {
            lg[a] = L[a] + P.b_pol[a];
            mx = fmaxf(mx, lg[a]);
        }
        const float v = tanhf(L[7] + P.b_val[0]);
        value[slot] = v;
        if (logits) {
#pragma unroll
            for (int a = 0; a < c4::kActions; ++a) logits[(size_t)slot * c4::kActions + a] = lg[a];
        }
        if (priors) {
            float e[c4::kActions], sum = 0.f;
#pragma unroll
            for (int a = 0; a < c4::kActions; ++a) {
                e[a] = __expf(lg[a] - mx);
                sum += e[a];
            }
            const float inv = 1.0f / sum;
#pragma unroll
            for (int a = 0; a < c4::kActions; ++a) e[a] *= inv;
            const uint64_t *bb = (const uint64_t *)(smem + kB);
            float out[c4::kActions];
            c4::mask_renorm(e, c4::open_columns(bb[2 * tid] | bb[2 * tid + 1]), out);
            float4 *pr = (float4 *)(priors + (size_t)slot * kPriorStride);
            pr[0] = make_float4(out[0], out[1], out[2], out[3]);
            pr[1] = make_float4(out[4], out[5], out[6], 0.f);
        }
    }
}

// ---------------------------------------------------------------- host packing
uint16_t f2bf(float f) {   // round to nearest even
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)((u >> 16) | ((u & 0xFFFF) ? 0x40 : 0));
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

struct ConvRef {
    const float *w, *b, *bn;   // w [co][ci][3][3], b [co], bn [4][co]
    int ci, co;
};

// BN-folded weight w'[co][ci][tap] and bias b'[co]
void fold(const ConvRef &c, std::vector<float> &w, std::vector<float> &b) {
    w.assign((size_t)c.co * c.ci * 9, 0.f);
    b.assign(c.co, 0.f);
    for (int o = 0; o < c.co; ++o) {
        const float g = c.bn[o], be = c.bn[c.co + o], mu = c.bn[2 * c.co + o], var = c.bn[3 * c.co + o];
        const float scale = g / std::sqrt(var + 1e-5f);
        for (int i = 0; i < c.ci * 9; ++i) w[(size_t)o * c.ci * 9 + i] = c.w[(size_t)o * c.ci * 9 + i] * scale;
        b[o] = (c.b[o] - mu) * scale + be;
    }
}

}  // namespace

size_t net_num_params(int game, int blocks, int hidden) {
    if (game != SPAI_GAME_CONNECT4) return 0;
    auto conv = [](size_t ci, size_t co) { return co * ci * 9 + co + 4 * co; };
    size_t n = conv(3, hidden) + (size_t)blocks * 2 * conv(hidden, hidden);
    n += conv(hidden, 32) + 7 * kPolIn + 7;
    n += conv(hidden, 3) + kValIn + 1;
    return n;
}

int net_create(spai_engine *e, int blocks, int hidden, const float *params, size_t nparams, spai_net **out) {
    SPAI_CHECK(e->game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "device net: only Connect4 is built");
    SPAI_CHECK(hidden == kHid, SPAI_ERR_UNSUPPORTED, "device net: hidden must be 64 (got %d)", hidden);
    SPAI_CHECK(blocks >= 0 && blocks <= 64, SPAI_ERR_INVALID, "bad block count %d", blocks);
    SPAI_CHECK(params && nparams == net_num_params(e->game, blocks, hidden), SPAI_ERR_INVALID,
               "expected %zu params, got %zu", net_num_params(e->game, blocks, hidden), nparams);
    // walk the parameter list in construction order
    const float *p = params;
    auto take_conv = [&](int ci, int co) {
        ConvRef c{p, p + (size_t)co * ci * 9, p + (size_t)co * ci * 9 + co, ci, co};
        p += (size_t)co * ci * 9 + co + 4 * co;
        return c;
    };
    ConvRef stem_c = take_conv(3, kHid);
    std::vector<ConvRef> res;
    for (int i = 0; i < 2 * blocks; ++i) res.push_back(take_conv(kHid, kHid));
    ConvRef pol_c = take_conv(kHid, 32);
    const float *pol_w = p, *pol_b = p + 7 * kPolIn;
    p += 7 * kPolIn + 7;
    ConvRef val_c = take_conv(kHid, 3);
    const float *val_w = p, *val_b = p + kValIn;
    p += kValIn + 1;

    std::vector<float> fw, fb;
    // stem fragments: [ct 4][lane 64][8]; k = tap*3 + ci for k < 27
    std::vector<uint16_t> ws(4 * 64 * 8, 0);
    std::vector<float> bs(kHid);
    fold(stem_c, fw, fb);
    for (int ct = 0; ct < 4; ++ct)
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
                int co = ct * 16 + (l & 15), k = 8 * (l >> 4) + j;
                float v = 0.f;
                if (k < 27) v = fw[(size_t)co * 27 + (k % 3) * 9 + k / 3];
                ws[(ct * 64 + l) * 8 + j] = f2bf(v);
            }
    for (int o = 0; o < kHid; ++o) bs[o] = fb[o];
    // residual convs: [layer][ks 18][ct 4][lane 64][8]; k = tap*64 + ci
    std::vector<uint16_t> wr((size_t)2 * blocks * kKStepsRes * 4 * 64 * 8);
    std::vector<float> br((size_t)2 * blocks * kHid);
    for (int L = 0; L < 2 * blocks; ++L) {
        fold(res[L], fw, fb);
        for (int ks = 0; ks < kKStepsRes; ++ks)
            for (int ct = 0; ct < 4; ++ct)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 8; ++j) {
                        int co = ct * 16 + (l & 15), k = ks * 32 + 8 * (l >> 4) + j;
                        int tap = k / kHid, ci = k % kHid;
                        wr[((((size_t)L * kKStepsRes + ks) * 4 + ct) * 64 + l) * 8 + j] =
                            f2bf(fw[((size_t)co * kHid + ci) * 9 + tap]);
                    }
        for (int o = 0; o < kHid; ++o) br[(size_t)L * kHid + o] = fb[o];
    }
    // head conv: co 0..31 policy, 32..34 value, rest zero
    std::vector<float> pw, pb, vw, vb;
    fold(pol_c, pw, pb);
    fold(val_c, vw, vb);
    std::vector<uint16_t> wh((size_t)kKStepsRes * kHeadCT * 64 * 8, 0);
    std::vector<float> bh(48, 0.f);
    for (int ks = 0; ks < kKStepsRes; ++ks)
        for (int ct = 0; ct < kHeadCT; ++ct)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    int co = ct * 16 + (l & 15), k = ks * 32 + 8 * (l >> 4) + j;
                    int tap = k / kHid, ci = k % kHid;
                    float v = 0.f;
                    if (co < 32) v = pw[((size_t)co * kHid + ci) * 9 + tap];
                    else if (co < kHeadC) v = vw[((size_t)(co - 32) * kHid + ci) * 9 + tap];
                    wh[(((size_t)ks * kHeadCT + ct) * 64 + l) * 8 + j] = f2bf(v);
                }
    for (int o = 0; o < 32; ++o) bh[o] = pb[o];
    for (int o = 0; o < 3; ++o) bh[32 + o] = vb[o];

    spai_net *n = new spai_net();
    n->eng = e;
    n->blocks = blocks;
    n->hidden = hidden;
    int rc = SPAI_OK;
    auto up = [&](auto &buf, const auto &vec) {
        if (rc != SPAI_OK) return;
        rc = buf.alloc(vec.size());
        if (rc == SPAI_OK && !vec.empty() &&
            hipMemcpy(buf.p, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice) != hipSuccess) {
            set_error("hipMemcpy of net weights failed");
            rc = SPAI_ERR_DEVICE;
        }
    };
    up(n->w_stem, ws);
    up(n->b_stem, bs);
    if (blocks > 0) {
        up(n->w_res, wr);
        up(n->b_res, br);
    }
    up(n->w_head, wh);
    up(n->b_head, bh);
    up(n->w_pol, std::vector<float>(pol_w, pol_w + 7 * kPolIn));
    up(n->b_pol, std::vector<float>(pol_b, pol_b + 7));
    up(n->w_val, std::vector<float>(val_w, val_w + kValIn));
    up(n->b_val, std::vector<float>(val_b, val_b + 1));
    if (rc != SPAI_OK) {
        net_destroy(n);
        return rc;
    }
    *out = n;
    return SPAI_OK;
}

void net_destroy(spai_net *n) {
    if (!n) return;
    for (auto *b : {&n->w_stem, &n->w_res, &n->w_head}) b->release();
    for (auto *b : {&n->b_stem, &n->b_res, &n->b_head, &n->w_pol, &n->b_pol, &n->w_val, &n->b_val, &n->io_x,
                    &n->io_logits, &n->io_value, &n->io_priors})
        b->release();
    n->io_mine.release();
    n->io_theirs.release();
    n->io_count.release();
    delete n;
}

static NetParams params_of(const spai_net *n) {
    NetParams P;
    P.w_stem = (const uint4 *)n->w_stem.p;
    P.w_res = (const uint4 *)n->w_res.p;
    P.w_head = (const uint4 *)n->w_head.p;
    P.b_stem = n->b_stem.p;
    P.b_res = n->b_res.p;
    P.b_head = n->b_head.p;
    P.w_pol = n->w_pol.p;
    P.b_pol = n->b_pol.p;
    P.w_val = n->w_val.p;
    P.b_val = n->b_val.p;
    P.blocks = n->blocks;
    return P;
}

int net_eval_batch(spai_net *net, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint64_t *mine,
                   const uint64_t *theirs, float *priors, float *value) {
    if (!max_n) return SPAI_OK;
    const uint32_t grid = (max_n + kS - 1) / kS;
    k_forward<false><<<grid, kThreads, 0, st>>>(d_count, max_n, mine, theirs, nullptr, params_of(net), priors, value,
                                                nullptr);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

static int ensure(spai_net *n, uint32_t cnt) {
    if (n->io_value.n >= cnt) return SPAI_OK;
    SPAI_TRY(n->io_x.alloc((size_t)cnt * 126));
    SPAI_TRY(n->io_logits.alloc((size_t)cnt * 7));
    SPAI_TRY(n->io_value.alloc(cnt));
    SPAI_TRY(n->io_priors.alloc((size_t)cnt * kPriorStride));
    SPAI_TRY(n->io_mine.alloc(cnt));
    SPAI_TRY(n->io_theirs.alloc(cnt));
    return SPAI_OK;
}

int net_forward_x(spai_net *n, uint32_t cnt, const float *x, float *logits, float *value) {
    if (!cnt) return SPAI_OK;
    SPAI_TRY(ensure(n, cnt));
    hipStream_t st = n->eng->stream;
    SPAI_HIP(hipMemcpyAsync(n->io_x.p, x, (size_t)cnt * 126 * 4, hipMemcpyHostToDevice, st));
    k_forward<true><<<(cnt + kS - 1) / kS, kThreads, 0, st>>>(nullptr, cnt, nullptr, nullptr, n->io_x.p, params_of(n),
                                                             nullptr, n->io_value.p, n->io_logits.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(logits, n->io_logits.p, (size_t)cnt * 28, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipMemcpyAsync(value, n->io_value.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

int net_predict(spai_net *n, uint32_t cnt, const spai_c4_state *states, float *priors, float *values) {
    if (!cnt) return SPAI_OK;
    SPAI_TRY(ensure(n, cnt));
    std::vector<uint64_t> m(cnt), t(cnt);
    for (uint32_t i = 0; i < cnt; ++i) {
        bool xm = c4::x_to_move(states[i].num_actions_played);
        m[i] = xm ? states[i].x : states[i].o;
        t[i] = xm ? states[i].o : states[i].x;
    }
    hipStream_t st = n->eng->stream;
    SPAI_HIP(hipMemcpyAsync(n->io_mine.p, m.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(n->io_theirs.p, t.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    k_forward<false><<<(cnt + kS - 1) / kS, kThreads, 0, st>>>(nullptr, cnt, n->io_mine.p, n->io_theirs.p, nullptr,
                                                              params_of(n), n->io_priors.p, n->io_value.p, nullptr);
    SPAI_HIP(hipGetLastError());
    std::vector<float> pr((size_t)cnt * kPriorStride);
    SPAI_HIP(hipMemcpyAsync(pr.data(), n->io_priors.p, pr.size() * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipMemcpyAsync(values, n->io_value.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < cnt; ++i) {
        const bool ended = states[i].status != c4::kOngoing;   // no valid actions -> 0/0 (connect_four.rs:276)
        for (int a = 0; a < 7; ++a) priors[(size_t)i * 7 + a] = ended ? NAN : pr[(size_t)i * kPriorStride + a];
    }
    return SPAI_OK;
}

}  // namespace spai

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
//  * wave W owns 21 of the 84 (position tile, co tile) tasks of a 64-channel layer
// Algorithmic FLOPs per position (6 blocks x 64): 39,016,572.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "spai_internal.h"

namespace spai {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

constexpr int kHid = 64;
constexpr int kS = 8;                      // max positions per workgroup group
constexpr int kP = kS * c4::kCells;        // 336 board cells (LDS rows) at S = 8
// position tiles (16 LDS rows each) for a group of S positions
__host__ __device__ constexpr int npt_of(int S) { return (S * c4::kCells + 15) / 16; }
constexpr int kWaves = 4;                  // plan waves: the work split of every layer
// SPAI_W8 (experimental build): two waves per SIMD.  Waves W and W + 4 run plan
// wave W's tasks of every trunk conv over the two halves of K (the k-steps of
// input channels 0-31 and 32-63 of each tap: the same weight bytes per CU, half
// each), exchange half their partial sums through LDS and each finishes half
// the tasks; the stem, head and linear run on waves 0-3.  Group sizes <= 5 only
// (the partial-sum buffer must fit beside the activations).
#ifdef SPAI_W8
constexpr int kPhysWaves = 8;
#else
constexpr int kPhysWaves = 4;
#endif
constexpr int kThreads = kPhysWaves * 64;
constexpr int kStemThreads = kWaves * 64;   // the per-position setup work (stem weights, planes)
constexpr int kKStepsRes = 18;             // 576 / 32
constexpr int kHeadC = 35;                 // 32 policy + 3 value channels
constexpr int kPolIn = 32 * c4::kCells;    // 1344
constexpr int kValIn = 3 * c4::kCells;     // 126

// LDS carve (bytes)
constexpr int kZ = 0;                      // 256 B of zeros just below X (out-of-board taps)
constexpr int kX = 256;                    // [336][128 B] bf16 activations (256-B aligned)
constexpr int kZ1 = kX + kP * 128;         // 256 B of zeros just below Y
constexpr int kY = kZ1 + 256;              // second activation buffer
// Head features in LDS: H[s][cell*36 + c] (c < 35: 32 policy + 3 value channels,
// c = 35 is a zero pad), so the head conv's epilogue stores 4 channels of a cell
// as one 8-B word.  The fused linear runs over this cell-major K order (the host
// permutes the linear weights from the reference's c*42 + cell flatten to it).
constexpr int kHC = 36;                    // channels per cell in H
constexpr int kLinFeat = kHC * 42;         // 1512
constexpr int kLinK = 1536;                // padded to 48 k-steps of 32
constexpr int kLinKSteps = kLinK / 32;     // 48
constexpr int kLinPitch = kLinK + 16;      // the largest head-feature pitch (lin_pitch) sizes the overlay
// The fused linear has 8 outputs (7 logits + the value), so an MFMA B fragment
// of 16 columns would be half zeros.  The two K halves are packed into the 16
// columns instead: column n = (output n & 7, K half n >> 3), A row m =
// (position m & 7, K half m >> 3), and the diagonal blocks of D are the two
// halves' partial sums -- 24 k-steps and 24 KiB of weights, not 48.
constexpr int kLinHalves = 2;
constexpr int kLinBSteps = kLinKSteps / kLinHalves;   // B-fragment k-steps (1 KiB each)
constexpr int kH = kY;                     // bf16 head features [8][kLinPitch] overlay Y
constexpr int kHBytes = kP * 128;          // (all of Y)
constexpr int kB = kH + kHBytes;           // 8 x (mine, theirs)
constexpr int kL = kB + kS * 16;           // linear partials [4 waves][halves][8][8] f32
constexpr int kMaxBlocks = 20;
constexpr int kBiasFloats = kHid + 2 * kMaxBlocks * kHid + kHid;   // stem, residual convs, head (64 padded)
constexpr int kBias = kL + kWaves * kLinHalves * 64 * 4; // all conv biases, staged once per workgroup
constexpr int kBiasPer = (kBiasFloats + kStemThreads - 1) / kStemThreads;   // per thread
constexpr int kPlanes = kBias + kBiasFloats * 4;   // stem neighbour planes [8][34] u64 (272-B rows: positions
                                                   // in different 16-B bank groups)
constexpr int kPlaneRow = 34;
constexpr int kWStem = kPlanes + kS * kPlaneRow * 8;   // stem weight fragments [4 ct][64 lanes] x 16 B, staged once
constexpr int kTab = kWStem + 4 * 64 * 16;         // k_geo_init: one S's row-group table [42] x 16 B (NetParams::geo)
// The fused linear's B fragments: each wave loads its 6 k-steps straight into
// registers at the head conv's start (an LDS-DMA copy made the compiler wait
// vmcnt(0) at the head k-loop's first weight use).
constexpr int kLinWPer = kLinBSteps / kWaves;      // B fragments per wave
#ifdef SPAI_W8
constexpr int kSRun = 5;                   // largest group size this build runs
constexpr int kSplitMaxN = 14;             // most tasks of a plan wave at S <= kSRun (S = 5, position-major)
constexpr int kPart = kTab + 42 * 16;      // split-K partial sums [4 plan waves][kSplitMaxN][64 lanes] x 16 B
constexpr int kLdsBytes = kPart + kWaves * kSplitMaxN * 1024;
#else
constexpr int kSRun = kS;
constexpr int kLdsBytes = kTab + 42 * 16;
#endif
#ifdef SPAI_DIAG_KSTEP
constexpr int kStamps = 48;                // + 24..41: after each k-step of block 1 conv 1, 42 before its barrier, 43
                                           // after it, 44 at its start (diagnostic k-step build)
#else
constexpr int kStamps = 24;                // phase stamps per wave in the diagnostic mode (17..19: inside block 0 conv1;
#endif
                                           // 20/21: s_memtime / s_memrealtime at kernel entry, 22: s_memrealtime at the
                                           // first group's stamp 0, 23: s_memrealtime after the last group)
static_assert(kS * kLinPitch * 2 <= kHBytes, "head features fit in Y");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct NetParams {
    const uint4 *w_stem;   // [4 ct][64 lanes] 16 B fragments
    const uint4 *w_res;    // [2*blocks][18 ks][4 ct][64]
    const uint4 *w_head;   // [18][4][64]: a 64-channel layer whose co tile 3 is never computed
    const float *b_conv;   // conv biases, BN folded: [64 stem | 2*blocks x 64 residual convs | 64 head conv]
    const uint4 *w_lin;    // [48 ks][64] B fragments of the fused policy|value linear
    const float *b_pol;    // [7]
    const float *b_val;    // [1]
    // per group size S and row group idx (= LDS row / S): {cell, then the row group
    // holding each 3x3 tap's neighbour cell as 9 bytes (0xFF off the board)} x 16 B
    const uint4 *geo;             // [9][42]
    const uint4 *lane_geo;        // per-lane geometry of every (S, wave, tile): lane_geo_at, k_geo_init
    unsigned long long *stamps;   // diagnostic: [grid][4 waves][kStamps] s_memtime, or null
    int blocks;
};

// Phase stamps exist only in the diagnostic build (-DSPAI_DIAG): the branch
// around the store would otherwise cost the production kernel precise
// vmcnt tracking (hipcc waits vmcnt(0) after such control flow).
#ifdef SPAI_DIAG_HEAD
constexpr bool kDiagHead = true;   // stamps 17..19 time the head instead of block 0 conv 1
#else
constexpr bool kDiagHead = false;
#endif
// SPAI_DIAG_ENTRY (diagnostic builds): stamps 17..19 time the launch prologue
// instead -- 17 constants in LDS, 18 first group's geometry and bitboards loaded,
// 19 its planes stored (each behind a full wait, so the phases are serialised)
#ifdef SPAI_DIAG_ENTRY
constexpr bool kDiagEntry = true;
#else
[[maybe_unused]] constexpr bool kDiagEntry = false;
#endif
__device__ __forceinline__ void stamp(const NetParams &P, int wave, int lane, int k) {
#ifdef SPAI_DIAG
    if (P.stamps && lane == 0 && wave >= 0) P.stamps[((size_t)blockIdx.x * kWaves + wave) * kStamps + k] = __builtin_amdgcn_s_memtime();
#endif
}
// wall-clock stamp (100 MHz constant clock), diagnostic build only
__device__ __forceinline__ void stamp_real(const NetParams &P, int wave, int lane, int k) {
#ifdef SPAI_DIAG
    if (P.stamps && lane == 0 && wave >= 0)
        P.stamps[((size_t)blockIdx.x * kWaves + wave) * kStamps + k] = __builtin_amdgcn_s_memrealtime();
#endif
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// relu(round_bf16(a)), relu(round_bf16(b)) packed: ReLU on the packed bf16 pair is a
// signed 16-bit max with 0 (a negative value rounds to a negative bf16 or -0,
// both of which clamp to +0), so it costs one v_pk_max_i16 per two channels.
__device__ __forceinline__ uint32_t pack_relu_bf16x2(float a, float b) {
    const i16x2 h = __builtin_bit_cast(i16x2, __builtin_convertvector((f32x2){a, b}, bf16x2));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, (i16x2){0, 0}));
}

// ---------------------------------------------------------------- cell order and skipped taps
// Row layout of a group of S positions in the activation buffers:
//  * S <= 3, position-major: row r holds cell r % 42 of position r / 42 (cell =
//    board row * 7 + column), so a 3x3 tap is a contiguous shift of the rows;
//  * S >= 4, cell-major: row r holds cell kCellOrder[S][r / S] of position r % S.
//    The orders group board-edge cells so that some 16-row position tiles have NO
//    on-board neighbour for a tap: tap_skip(S, t) is the mask of such taps (bit
//    (dh+1)*3 + (dw+1)) of tile t, and their MFMAs and B-fragment reads are skipped
//    -- every product they would add is an exact zero (an out-of-board tap reads
//    the zeroed block), so the results are the same.
// Generated by scripts/gen_cell_orders.py (balanced over the four waves' task
// plans; at S = 4 the order index's parity is the cell's checkerboard colour,
// which keeps the permuted B reads conflict-free); max MFMA (tile, tap) pairs per
// wave and layer:
// S=1: position-major rows, identity order
// S=2: position-major rows, identity order
// S=3: position-major rows, identity order
// S=4: max MFMA tile-taps per wave and trunk layer 90 -> 84 [84, 84, 84, 84], head 72 -> 72
// S=5: max MFMA tile-taps per wave and trunk layer 126 -> 114 [114, 102, 114, 106], head 99 -> 84
// S=6: max MFMA tile-taps per wave and trunk layer 144 -> 132 [128, 132, 132, 132], head 108 -> 99
// S=7: max MFMA tile-taps per wave and trunk layer 171 -> 146 [146, 144, 144, 142], head 126 -> 111
// S=8: max MFMA tile-taps per wave and trunk layer 189 -> 159 [153, 159, 159, 153], head 144 -> 123
constexpr uint8_t kCellOrder[9][42] = {   // host: packed into NetParams::geo at net_create
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41},
    {22, 33, 10, 23, 24, 11, 26, 17, 8, 25, 18, 5, 6, 3, 4, 1, 34, 13, 20, 27, 30, 9, 16, 7, 38, 37, 40, 41, 0, 21, 14, 35, 32, 31, 12, 29, 28, 19, 2, 15, 36, 39},
    {13, 5, 30, 10, 23, 12, 38, 40, 37, 36, 0, 32, 27, 41, 20, 34, 2, 4, 3, 1, 16, 18, 26, 33, 39, 31, 22, 11, 28, 21, 14, 7, 8, 9, 15, 19, 24, 17, 35, 25, 29, 6},
    {37, 20, 40, 33, 22, 13, 25, 24, 35, 39, 38, 7, 10, 32, 19, 17, 27, 34, 41, 8, 16, 11, 36, 12, 2, 0, 4, 6, 26, 28, 1, 29, 30, 3, 15, 9, 31, 5, 23, 18, 21, 14},
    {8, 22, 4, 3, 1, 13, 20, 9, 33, 7, 21, 14, 25, 18, 19, 24, 35, 28, 0, 2, 5, 31, 32, 12, 16, 38, 36, 40, 39, 37, 26, 17, 27, 6, 34, 11, 30, 15, 23, 29, 10, 41},
    {28, 21, 41, 37, 18, 26, 1, 2, 16, 29, 22, 31, 15, 17, 5, 6, 24, 8, 13, 20, 4, 3, 33, 30, 27, 34, 0, 35, 12, 25, 23, 10, 36, 39, 19, 11, 32, 9, 38, 40, 7, 14},
};
__host__ __device__ constexpr uint16_t tap_skip(int S, int t) {
    constexpr uint16_t m1[21] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    constexpr uint16_t m2[21] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    constexpr uint16_t m3[21] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    constexpr uint16_t m4[21] = {0, 0, 0, 7, 292, 0, 448, 73, 0, 0, 448, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    constexpr uint16_t m5[21] = {0, 0, 448, 0, 292, 7, 0, 0, 0, 73, 0, 0, 0, 295, 0, 0, 0, 0, 0, 0, 0};
    constexpr uint16_t m6[21] = {256, 0, 0, 448, 0, 0, 292, 0, 0, 7, 0, 0, 0, 0, 0, 73, 0, 0, 0, 0, 0};
    constexpr uint16_t m7[21] = {0, 7, 4, 0, 73, 0, 0, 73, 7, 0, 0, 448, 448, 0, 292, 0, 0, 0, 484, 0, 0};
    constexpr uint16_t m8[21] = {73, 448, 0, 7, 0, 0, 0, 7, 0, 292, 7, 0, 292, 73, 0, 0, 448, 0, 0, 448, 73};
    return S == 1 ? m1[t] : S == 2 ? m2[t] : S == 3 ? m3[t] : S == 4 ? m4[t] : S == 5 ? m5[t] : S == 6 ? m6[t] : S == 7 ? m7[t] : m8[t];
}
__host__ __device__ constexpr bool cell_major(int S) { return S >= 4; }
// head-feature row pitch (bf16 elements): the head conv's 8-B stores of a tile hit
// distinct banks with 772 words at S = 8 and 776 words at S = 4
__host__ __device__ constexpr int lin_pitch(int S) { return S == 4 ? 1552 : 1544; }
// the first k-step of tile t whose tap is not skipped: its MFMA takes the bias
__host__ __device__ constexpr int first_kstep(int S, int t) {
    int tap = 0;
    while ((tap_skip(S, t) >> tap) & 1) ++tap;   // the centre tap is always on the board
    return 2 * tap;
}

// Work split: a conv layer is NPT position tiles x CT co tiles = NPT*CT
// tile-tasks over the four waves.  Three task orders, picked per layer shape:
//  * position-major (head conv, CT = 3, and the largest groups, where the
//    other orders run out of registers): wave W owns tasks [TT*W/4, TT*(W+1)/4)
//    of task = pos_tile*CT + co_tile: ~NPT/4 position tiles, every co tile, so
//    each wave streams all CT weight fragments per k-step;
//  * co-major (NPT <= SPAI_CO_MAJOR_MAX_NPT): in the 64-channel layers wave W
//    owns co tile W over all NPT position tiles, so the CU fetches each weight
//    fragment once per k-step (4 KiB) at NPT LDS reads per wave; in the head
//    (CT = 3) a wave's contiguous task range spans at most 2 co tiles;
//  * pair split (64-channel layers, NPT <= SPAI_PAIR_MAX_NPT): wave (j = W>>1, h = W&1) owns co
//    tiles {2j, 2j+1} over position tiles [h*m, h*m+m) (m = NPT/2) plus, for
//    odd NPT, the last tile in co tile 2j+h: NPT tasks per wave, 2 weight
//    fragments per wave and k-step (8 KiB per CU), ~NPT/2 LDS reads.
// The per-CU weight stream is what bounds small groups: the vector-memory
// path delivers ~64 B/clk/CU, i.e. 16 KiB per k-step costs ~256 cycles.
// Position tiles are addressed through a local index t < NT; gpt(t) is the
// group's position tile, pt(i) the local tile and co(i) the co tile of task i.
#ifndef SPAI_CO_MAJOR_MAX_NPT
#define SPAI_CO_MAJOR_MAX_NPT 8
#endif
#ifndef SPAI_PAIR_MAX_NPT
#define SPAI_PAIR_MAX_NPT 11
#endif
#ifndef SPAI_HEAD_CO_MAJOR_MAX_NPT
#define SPAI_HEAD_CO_MAJOR_MAX_NPT 8   // the head conv (CT = 3) in co-major order up to this many tiles
#endif
// Deferred epilogue (SPAI_DEFER_EPI).  A trunk conv's fused epilogue (ReLU, bf16 pack,
// LDS store: 8 VALU + a store per task) cannot hide in the last tap's MFMA gaps (an
// MFMA leaves 8 issue cycles free, a task's epilogue needs ~44), so at the
// position-major group sizes (S >= 5) the tasks of co tiles 2 and 3 -- output
// channels 32-63 -- keep their fp32 accumulators into the NEXT layer, which runs the
// K-half-0 k-steps of every tap (input channels 0-31) first and does those deferred
// epilogues in their MFMA gaps; a barrier then publishes channels 32-63 before the
// K-half-1 k-steps read them.  The K order is the same at every group size (the sums,
// and so the results, do not depend on S).
#ifdef SPAI_DEFER_EPI
constexpr bool kDefer = true;
#else
constexpr bool kDefer = false;
#endif
// k-step executed j-th in a layer (k = tap * 2 + K half)
__host__ __device__ constexpr int kstep_of(int j) { return kDefer ? (j < 9 ? 2 * j : 2 * (j - 9) + 1) : j; }

template <int W, int CT, int NPT>
struct Plan {
    static constexpr int MODE = NPT <= (CT == 3 ? SPAI_HEAD_CO_MAJOR_MAX_NPT : SPAI_CO_MAJOR_MAX_NPT) ? 1
                                : CT == 4 && NPT <= SPAI_PAIR_MAX_NPT                              ? 2
                                                                                                    : 0;
    static constexpr int TT = NPT * CT;
    // position-major / co-major: a contiguous task range
    static constexpr int first = TT * W / 4;
    static constexpr int nr = TT * (W + 1) / 4 - first;
    static constexpr int last = first + nr - 1;
    // pair split
    static constexpr int m = NPT / 2, r = NPT % 2, pj = W >> 1, ph = W & 1;

    static constexpr int n = MODE == 2 ? 2 * m + r : nr;   // tasks of this wave
    static constexpr int C0 = MODE == 2 ? 2 * pj : MODE == 1 ? first / NPT : 0;   // first co tile loaded
    static constexpr int CTL = MODE == 2 ? 2 : MODE == 1 ? last / NPT - C0 + 1 : CT;   // co tiles per k-step
    static constexpr int T0 = MODE == 2 ? ph * m
                              : MODE == 1 ? (CTL == 1 ? first % NPT : 0)
                                          : first / CT;
    static constexpr int NT = MODE == 2 ? m + r : MODE == 1 ? (CTL == 1 ? nr : NPT) : last / CT - T0 + 1;
    static constexpr int gpt(int t) { return MODE == 2 && t == m ? NPT - 1 : T0 + t; }
    static constexpr int pt(int i) {
        return MODE == 2 ? (i < 2 * m ? i / 2 : m) : (MODE == 1 ? (first + i) % NPT : (first + i) / CT) - T0;
    }
    static constexpr int co(int i) {
        return MODE == 2 ? (i < 2 * m ? 2 * pj + (i & 1) : 2 * pj + ph)
                         : MODE == 1 ? (first + i) / NPT : (first + i) % CT;
    }
    // deferred epilogue: the position-major 64-channel plans defer their co-tile 2/3 tasks
    static constexpr bool DEFER = kDefer && CT == 4 && MODE == 0;
    static constexpr int count_deferred() {
        int c = 0;
        for (int i = 0; i < n; ++i) c += co(i) >= 2;
        return c;
    }
    static constexpr int ND = DEFER ? count_deferred() : 0;
    // the deferred accumulators are indexed by task (dacc[i], only the deferred ones live):
    // every index stays a plain expression of the unrolled loop counters, so the arrays are
    // scalarised into registers (a loop-valued task map left them on the scratch stack)
    static constexpr int NDA = ND > 0 ? n : 1;
    static constexpr bool deferred(int i) { return DEFER && co(i) >= 2; }
};

// Per-lane LDS geometry, computed once per kernel (positions are the same for
// every layer).  For tile t and tap (dh,dw) the B-fragment address relative to
// the activation buffer is rel[t][tap] (k-step half 0; half 1 = rel ^ 64, the
// swizzled chunk index flips bit 2).  With the XOR swizzle every 3x3 shift of a
// 16-row tile is conflict-free for ds_read_b128; an out-of-board tap points
// into the zeroed 256-B block below the buffer, so the k-loop needs no select.  epi[t] is the
// relative address of this lane's 4 output channels of co tile 0 at its
// position (co tile c: epi ^ (c << 5)).
// rel is stored biased by +256 (the zero block becomes 0..255) as 16-bit halves,
// two taps per register (tap 2j low, 2j+1 high): 5 registers per tile instead of
// 9, which lets the pair split hold 11 position tiles without spilling.
template <int NT>
struct Geo {
    uint32_t rel2[NT][5];
    int epi[NT];
    // B-fragment offset of tile t, tap `tap`, relative to (buffer - 256)
    __device__ __forceinline__ uint32_t b(int t, int tap) const {
        return (tap & 1) ? rel2[t][tap >> 1] >> 16 : rel2[t][tap >> 1] & 0xFFFFu;
    }
};

// LDS row p of a group of S positions -> (position s, cell, order index idx)
struct RowCell {
    int s, cell, idx;   // cell < 0: a padding row past S * 42
};
template <int S>
__device__ __forceinline__ RowCell row_cell(const uint8_t *smem, int p) {
    if (p >= S * c4::kCells) return RowCell{0, -1, 0};
    if constexpr (!cell_major(S)) {
        const int s = p / c4::kCells, cell = p - s * c4::kCells;
        return RowCell{s, cell, cell};
    } else {
        const int idx = p / S;
        return RowCell{p - idx * S, (int)((const uint32_t *)(smem + kTab))[idx * 4], idx};
    }
}

template <int W, int CT, int NPT, int S>
__device__ __forceinline__ void make_geo(const uint8_t *smem, int lane, Geo<Plan<W, CT, NPT>::NT> &g) {
    using PL = Plan<W, CT, NPT>;
    const int col = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < PL::NT; ++t) {
        const int p = PL::gpt(t) * 16 + col;
        if constexpr (!cell_major(S)) {   // position-major rows: a tap is a contiguous shift
            const int cell = p % c4::kCells;
            const int h = cell / c4::kCols, w = cell - h * c4::kCols;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int dh = tap / 3 - 1, dw = tap % 3 - 1;
                const int r = p + dh * c4::kCols + dw;
                const bool ok = (unsigned)(h + dh) < (unsigned)c4::kRows && (unsigned)(w + dw) < (unsigned)c4::kCols;
                const int full = r * 128 + ((q ^ (r & 7)) << 4);
                // an out-of-board tap reads the zero block below the buffer at the same
                // 16-B granule its row would use, so it never adds a bank conflict
                const uint32_t v = (uint32_t)((ok ? full : (full & 255) - 256) + 256);
                if (tap & 1) g.rel2[t][tap >> 1] |= v << 16;
                else g.rel2[t][tap >> 1] = v;
            }
        } else {   // cell-major rows through the staged table {cell, neighbour row groups}
            const bool real = p < S * c4::kCells;
            const int idx = real ? p / S : 0, s = p - idx * S;
            const uint4 e = *(const uint4 *)(smem + kTab + idx * 16);
            const int own = p * 128 + ((q ^ (p & 7)) << 4);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const uint32_t word = tap < 4 ? e.y : tap < 8 ? e.z : e.w;
                const int nb = (int)((word >> (8 * (tap & 3))) & 255u);
                int v;
                if (real && nb != 255) {   // the neighbour cell's row for this position
                    const int r = nb * S + s;
                    v = r * 128 + ((q ^ (r & 7)) << 4) + 256;
                } else if (S == 4) {       // the zero block, at the granule an on-board neighbour of this
                                           // colour would use (row group parity = checkerboard colour)
                    const int r = (((idx ^ (tap / 3 + tap % 3)) & 1) << 2) + s;
                    v = (r * 128 + ((q ^ (r & 7)) << 4)) & 255;
                } else {                   // the zero block, at this row's own granule
                    v = own & 255;
                }
                if (tap & 1) g.rel2[t][tap >> 1] |= (uint32_t)v << 16;
                else g.rel2[t][tap >> 1] = (uint32_t)v;
            }
        }
        g.epi[t] = p * 128 + ((((q >> 1)) ^ (p & 7)) << 4) + ((q & 1) << 3);
    }
}

// Per-lane geometry table (NetParams::lane_geo), built once per net by
// k_geo_init from make_geo: computing it in the forward cost ~10 VALU per
// (tile, tap), some 900 cycles per position tile before the first MFMA.  Entry
// (S, W, t) of the 64-channel layers' plan (the head conv runs on it too) holds
// 64 lanes x 32 B: {rel2[5], epi, aux, 0}; aux = s | (bit col*7+row) << 8 for the
// stem and the head-feature offsets (padding rows: s = S, a zeroed plane row).
#ifndef SPAI_GEO_NT
#define SPAI_GEO_NT 8
#endif
constexpr int kGeoNT = SPAI_GEO_NT;   // the most position tiles a wave holds (S = 3, co-major; 11 for a pair split at S = 8)
__host__ __device__ constexpr size_t lane_geo_at(int S, int W, int t) {
    return (((size_t)(S - 1) * kWaves + W) * kGeoNT + t) * 64 * 2;   // in uint4
}
constexpr size_t kLaneGeoU4 = lane_geo_at(kS + 1, 0, 0);

template <int W, int NPT, int S>
__device__ __forceinline__ void load_geo(const NetParams &P, int lane, Geo<Plan<W, 4, NPT>::NT> &g,
                                         int (&aux)[Plan<W, 4, NPT>::NT]) {
    constexpr int NT = Plan<W, 4, NPT>::NT;
    static_assert(NT <= kGeoNT, "lane geometry table depth");
    const uint4 *src = P.lane_geo + lane_geo_at(S, W, 0) + 2 * lane;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint4 a = src[t * 128], b = src[t * 128 + 1];
        g.rel2[t][0] = a.x;
        g.rel2[t][1] = a.y;
        g.rel2[t][2] = a.z;
        g.rel2[t][3] = a.w;
        g.rel2[t][4] = b.x;
        g.epi[t] = (int)b.y;
        aux[t] = (int)b.z;
    }
}

template <int S, int W>
__device__ void geo_init_one(const uint8_t *smem, uint4 *out, int lane) {
    constexpr int NPT = npt_of(S);
    using PL = Plan<W, 4, NPT>;
    Geo<PL::NT> g;
    make_geo<W, 4, NPT, S>(smem, lane, g);
    uint4 *dst = out + lane_geo_at(S, W, 0) + 2 * lane;
    for (int t = 0; t < PL::NT; ++t) {
        const RowCell rc = row_cell<S>(smem, PL::gpt(t) * 16 + (lane & 15));
        const int h = rc.cell / c4::kCols, w = rc.cell - h * c4::kCols;
        const int aux = rc.cell < 0 ? S : rc.s | (w * 7 + h) << 8;
        dst[t * 128] = make_uint4(g.rel2[t][0], g.rel2[t][1], g.rel2[t][2], g.rel2[t][3]);
        dst[t * 128 + 1] = make_uint4(g.rel2[t][4], (uint32_t)g.epi[t], (uint32_t)aux, 0u);
    }
}

template <int S>
__device__ void geo_init_s(const uint8_t *smem, uint4 *out, int W, int lane) {
    if (W == 0) geo_init_one<S, 0>(smem, out, lane);
    else if (W == 1) geo_init_one<S, 1>(smem, out, lane);
    else if (W == 2) geo_init_one<S, 2>(smem, out, lane);
    else geo_init_one<S, 3>(smem, out, lane);
}

// one 64-thread workgroup per (S, wave): blockIdx.x = (S - 1) * 4 + W
__global__ __launch_bounds__(64) void k_geo_init(const uint4 *__restrict__ geo, uint4 *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kLdsBytes];
    const int S = blockIdx.x / kWaves + 1, W = blockIdx.x % kWaves, lane = threadIdx.x;
    if (lane < c4::kCells) ((uint4 *)(smem + kTab))[lane] = geo[S * c4::kCells + lane];
    __syncthreads();
    switch (S) {
    case 1: geo_init_s<1>(smem, out, W, lane); break;
    case 2: geo_init_s<2>(smem, out, W, lane); break;
    case 3: geo_init_s<3>(smem, out, W, lane); break;
    case 4: geo_init_s<4>(smem, out, W, lane); break;
    case 5: geo_init_s<5>(smem, out, W, lane); break;
    case 6: geo_init_s<6>(smem, out, W, lane); break;
    case 7: geo_init_s<7>(smem, out, W, lane); break;
    default: geo_init_s<8>(smem, out, W, lane); break;
    }
}

// Prefetch depths per group size: a small group has few MFMAs per k-step to
// hide a weight load (L2) or an LDS read behind, but registers to spare.
// (DA must divide the 18 k-steps of a layer: the ring carries the next layer's
// first DA-1 k-steps in the slots a fresh layer expects.)
// scheduling of an ordinary k-step (knobs, round 6): the MFMA / VALU / LDS / VMEM
// interleave hints, and the scheduling fence that closes each k-step
// the fused last tap's per-task hints and fence (final_tap_epilogue; knobs)
#ifndef SPAI_FINAL_HINTS
#define SPAI_FINAL_HINTS 1
#endif
#ifndef SPAI_FINAL_FENCE
#define SPAI_FINAL_FENCE 1
#endif
#ifndef SPAI_ISSUE_HINTS
#define SPAI_ISSUE_HINTS 0   // 1: the round-3 interleave hints (-2.5 % sims/s in round 6, profiles/r06/sched)
#endif
#ifndef SPAI_KSTEP_FENCE
#define SPAI_KSTEP_FENCE 1
#endif
#ifndef SPAI_DA4
#define SPAI_DA4 6   // A ring at S = 4 (tuning knob)
#endif
#ifndef SPAI_DB4
#define SPAI_DB4 2   // B ring at S = 4 (tuning knob)
#endif
#ifndef SPAI_DA8
#ifdef SPAI_FINAL2
#define SPAI_DA8 6   // the two-tap final phase (final_phase2) holds k-steps 14-17 in four ring slots
#else
#define SPAI_DA8 3   // A ring at S >= 5 (tuning knob)
#endif
#endif
#ifndef SPAI_DB8
#define SPAI_DB8 3   // B ring at S >= 5 (tuning knob; 3 since round 6 without the issue hints: +0.5 %, profiles/r06/sched)
#endif
__host__ __device__ constexpr int a_depth(int S) { return S <= 2 ? 9 : S <= 3 ? 6 : S <= 4 ? SPAI_DA4 : SPAI_DA8; }
__host__ __device__ constexpr int b_depth(int S) { return S <= 2 ? 4 : S <= 3 ? 3 : S <= 4 ? SPAI_DB4 : SPAI_DB8; }

// implicit-GEMM 3x3 conv over the LDS activations at IN for wave W's tasks.
// Software pipeline: A (weights, global/L2) DA-1 k-steps ahead, B (LDS) DB-1
// k-steps ahead; sched_group_barrier interleaves the prefetch with the MFMAs
// (and keeps the scheduler from sinking loads onto their uses).  The first
// k-step takes the bias as its C operand, so the accumulators need no zeroing
// and the epilogue no bias add.  The A ring is the caller's: A[0..DA-2] arrive
// holding k-steps 0..DA-2, and the last DA-1 k-steps refill them with the first
// k-steps of the next layer (`wn`, may be null), so consecutive layers stream
// weights without a cold start.  `wn` is always a valid layer (the current one
// when nothing follows): an unconditional prefetch keeps the vmcnt bookkeeping
// free of branches.
// Timing-only deletion experiments (diagnostic builds; wrong results):
// SPAI_EXP_NOA replaces the k-loop's weight loads by a register value, SPAI_EXP_NOB
// its activation reads, SPAI_EXP_NOBAR drops the barrier between trunk layers.
__device__ __forceinline__ uint4 exp_a(const uint4 &src, int lane, int k) {
#ifdef SPAI_EXP_NOA
    (void)src;
    return make_uint4(0x3F803F80u ^ (uint32_t)(lane + k), 0x3F803F80u, 0x3F803F80u, (uint32_t)k);
#else
    (void)lane, (void)k;
    return src;
#endif
}
__device__ __forceinline__ uint4 exp_b(const uint8_t *p, int lane, int k) {
#ifdef SPAI_EXP_NOB
    (void)p;
    return make_uint4(0x3F803F80u ^ (uint32_t)(lane * 3 + k), 0x3F803F80u, 0x3F803F80u, (uint32_t)k);
#else
    (void)lane, (void)k;
    return *(const uint4 *)p;
#endif
}
__device__ __forceinline__ void layer_barrier() {
#ifndef SPAI_EXP_NOBAR
    __syncthreads();
#endif
}

// The last tap of a 64-channel layer, task-major, with the epilogue fused
// (conv_mfma EPI > 0): k-steps 16 and 17 of task i (and, EPI = 2, the residual
// identity MFMA on the center-tap fragment of the block input at OUT), then
// relu/bf16 of task i - 2 into OUT.
template <int W, int CT, int NPT, int S, int DA, int DB, int EPI, int OUT>
__device__ __forceinline__ void final_tap_epilogue(uint8_t *smem, const Geo<Plan<W, CT, NPT>::NT> &g, int lane,
                                                   const uint4 (&A)[DA][Plan<W, CT, NPT>::CTL],
                                                   const uint4 (&B)[DB][Plan<W, CT, NPT>::NT],
                                                   const f32x4 (&bv)[Plan<W, CT, NPT>::CTL],
                                                   f32x4 (&acc)[Plan<W, CT, NPT>::n],
                                                   const int (&hoff)[Plan<W, CT, NPT>::NT],
                                                   f32x4 (&dacc)[Plan<W, CT, NPT>::NDA]) {
    using PL = Plan<W, CT, NPT>;
    // (EPI 1/2 with a deferring plan: the co-tile 2/3 tasks hand their accumulators on instead)
    auto defer = [](int i) { return EPI < 3 && PL::deferred(i); };
#ifdef SPAI_EXP_EPI_LAG
    constexpr int n = PL::n, k0 = kKStepsRes - 2, D = SPAI_EXP_EPI_LAG;   // timing experiment: epilogue lag
#else
    constexpr int n = PL::n, k0 = kKStepsRes - 2, D = 2;
#endif
    static_assert(CT == 4, "fused epilogue: 64-channel layers");
    auto live = [](int t, int ks) { return !((tap_skip(S, PL::gpt(t)) >> (ks >> 1)) & 1); };
    auto task_on = [](int i) { return !(EPI == 3 && PL::co(i) == 3); };   // the head has no co tile 3
    // Residual add as one more MFMA per task: acc += I * x, B = the center-tap
    // fragment of the 32-channel block that holds the task's co tile (read from
    // OUT, which still holds the block input x), A = an identity selecting its 16
    // channels.  One exact product 1 * x plus zero products and a single fp32
    // rounding: the value of the VALU add it replaces, for 8 issue cycles per task
    // instead of ~8 VALU instructions.
    uint4 id[2];   // the residual identities
    uint4 rb[3];   // residual B fragments, two tasks ahead
    if (EPI == 2) {
        const int m = lane & 15, q = lane >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = 16 * h + m - 8 * q;
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = j == 2 * e ? 0x3F80u : j == 2 * e + 1 ? 0x3F800000u : 0u;
            id[h] = make_uint4(w[0], w[1], w[2], w[3]);
        }
#pragma unroll
        for (int i = 0; i < 2 && i < n; ++i)
            rb[i] = *(const uint4 *)(smem + (OUT - 256) + (g.b(PL::pt(i), 4) ^ ((PL::co(i) >> 1) << 6)));
    }
#pragma unroll
    for (int i = 0; i < n + D; ++i) {
        int nm = 0, nv = 0, nw = 0, nrd = 0;
        if (i < n) {
            if (EPI == 2 && i + 2 < n) {
                rb[(i + 2) % 3] = *(const uint4 *)(smem + (OUT - 256) + (g.b(PL::pt(i + 2), 4) ^ ((PL::co(i + 2) >> 1) << 6)));
                ++nrd;
            }
            const int t = PL::gpt(PL::pt(i)), c = PL::co(i) - PL::C0;
#pragma unroll
            for (int j = k0; j < kKStepsRes; ++j) {
                const int ks = kstep_of(j);
                if (task_on(i) && live(PL::pt(i), ks)) {
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[j % DA][c]), as_bf16x8(B[j % DB][PL::pt(i)]),
                                                                    ks == first_kstep(S, t) ? bv[c] : acc[i], 0, 0, 0);
                    ++nm;
                }
            }
            if (EPI == 2) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(id[PL::co(i) & 1]), as_bf16x8(rb[i % 3]), acc[i],
                                                                0, 0, 0);
                ++nm;
            }
        }
        if (i >= D && EPI < 3 && !defer(i - D)) {
            const int j = i - D;
            const int off = OUT + (g.epi[PL::pt(j)] ^ (PL::co(j) << 5));
#if defined(SPAI_EXP_NOEPI) || defined(SPAI_EXP_NOEPI_ALL)
            // timing-only deletion experiments (wrong results): no conversion VALU (the accumulator
            // kept alive in its AGPRs), zeros stored -- or (NOEPI_ALL) no store either
            asm volatile("" ::"a"(acc[j]));
#ifdef SPAI_EXP_NOEPI
            *(uint2 *)(smem + off) = make_uint2(0u, (uint32_t)off);
            nw = 1;
#endif
            nv = 0;
#elif defined(SPAI_EXP_STORE_B128)
            // timing-only experiment (wrong results): the same bytes as half as many 16-B
            // stores (task pairs; the second task of a pair stores nothing)
            if ((j & 1) == 0) {
                const uint32_t a0 = pack_relu_bf16x2(acc[j][0], acc[j][1]), a1 = pack_relu_bf16x2(acc[j][2], acc[j][3]);
                const int j2 = j + 1 < PL::n ? j + 1 : j;
                const uint32_t b0 = pack_relu_bf16x2(acc[j2][0], acc[j2][1]), b1 = pack_relu_bf16x2(acc[j2][2], acc[j2][3]);
                *(uint4 *)(smem + (off & ~15)) = make_uint4(a0, a1, b0, b1);
                nw = 1;
            }
            nv = 5;
#elif defined(SPAI_EXP_STORE_LIN)
            // timing-only experiment (wrong results): the same stores at bank-conflict-free
            // addresses (each 16-lane group writes 128 contiguous bytes)
            (void)off;
            *(uint2 *)(smem + OUT + j * 512 + lane * 8) = make_uint2(pack_relu_bf16x2(acc[j][0], acc[j][1]),
                                                                     pack_relu_bf16x2(acc[j][2], acc[j][3]));
            nv = 5;
            nw = 1;
#else
            *(uint2 *)(smem + off) = make_uint2(pack_relu_bf16x2(acc[j][0], acc[j][1]), pack_relu_bf16x2(acc[j][2], acc[j][3]));
            nv = 5;
            nw = 1;
#endif
        } else if (EPI == 3 && i >= D && task_on(i - D)) {   // the head: H[s][cell * 36 + c] for the 35 real channels
            const int j = i - D, co0 = PL::co(j) * 16 + 4 * (lane >> 4), off = hoff[PL::pt(j)];
            // a lane with nothing to store writes its own word of the (not yet used) linear partials
            const int addr = co0 < kHC && off >= 0 ? kH + 2 * (off + co0) : kL + 8 * lane;
            *(uint2 *)(smem + addr) = make_uint2(pack_relu_bf16x2(acc[j][0], acc[j][1]), pack_relu_bf16x2(acc[j][2], acc[j][3]));
            nv = 5;
            nw = 1;
        }
        // issue order: the MFMAs with the epilogue's 5 VALU in their gaps, then the store and the read
#if SPAI_FINAL_HINTS
        if (nm >= 1) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (nv) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        if (nm >= 2) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (nv) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        if (nm >= 3) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (nv) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
        if (nv) {
            if (nm == 0) __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            else if (nm == 1) __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
            else if (nm == 2) __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
        }
        if (nw) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        if (nrd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#else
        (void)nv;
        (void)nw;
        (void)nrd;
#endif
#if SPAI_FINAL_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
    if constexpr (EPI < 3 && PL::ND > 0) {
#pragma unroll
        for (int i = 0; i < PL::n; ++i)
            if (PL::deferred(i)) dacc[i] = acc[i];
    }
}

// SPAI_FINAL2: at the position-major group sizes (S >= 5) the last TWO taps (k-steps
// 14-17) run task-major with the epilogue fused, so the LDS stores of the finished
// tasks overlap twice as many MFMAs as in final_tap_epilogue (round 6: a trunk conv's
// ~750 cycles of epilogue stores otherwise outlast its last tap, profiles/r06).  Each
// task still adds its k-steps in order, so the results are those of the default.  The
// B fragments of k-steps 14-17 are read per position tile, one tile ahead; the weights
// of k-steps 14-17 sit in four distinct slots of the A ring (DA = 6).
#ifdef SPAI_FINAL2
constexpr bool kFinal2 = true;
#else
constexpr bool kFinal2 = false;
#endif
template <int W, int CT, int NPT, int S, int IN, int DA, int EPI, int OUT>
__device__ __forceinline__ void final_phase2(uint8_t *smem, const Geo<Plan<W, CT, NPT>::NT> &g, int lane,
                                             const uint4 (&A)[DA][Plan<W, CT, NPT>::CTL],
                                             f32x4 (&acc)[Plan<W, CT, NPT>::n]) {
    using PL = Plan<W, CT, NPT>;
    constexpr int n = PL::n, NT = PL::NT, k0 = kKStepsRes - 4, D = 2;
    static_assert(CT == 4 && PL::MODE == 0 && (EPI == 1 || EPI == 2), "final_phase2: position-major trunk convs");
    static_assert(DA >= 6, "final_phase2: k-steps 14-17 need four distinct A slots");
    auto live = [](int t, int ks) { return !((tap_skip(S, PL::gpt(t)) >> (ks >> 1)) & 1); };
    uint4 Bf[2][4];   // k-steps 14-17 of one local tile, double-buffered over the tiles
    auto read_tile = [&](int t) {
        int nr = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ks = k0 + k, tap = ks >> 1, flip = (ks & 1) << 6;
            if (live(t, ks)) {
                Bf[t & 1][k] = *(const uint4 *)(smem + (IN - 256) + (g.b(t, tap) ^ flip));
                ++nr;
            }
        }
        return nr;
    };
    uint4 id[2];   // the residual identities (final_tap_epilogue)
    uint4 rb[3];   // residual B fragments, two tasks ahead
    if (EPI == 2) {
        const int m = lane & 15, q = lane >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = 16 * h + m - 8 * q;
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = j == 2 * e ? 0x3F80u : j == 2 * e + 1 ? 0x3F800000u : 0u;
            id[h] = make_uint4(w[0], w[1], w[2], w[3]);
        }
#pragma unroll
        for (int i = 0; i < 2 && i < n; ++i)
            rb[i] = *(const uint4 *)(smem + (OUT - 256) + (g.b(PL::pt(i), 4) ^ ((PL::co(i) >> 1) << 6)));
    }
    read_tile(PL::pt(0));
#pragma unroll
    for (int i = 0; i < n + D; ++i) {
        int nm = 0, nv = 0, nw = 0, nrd = 0;
        if (i < n) {
            const int t = PL::pt(i), c = PL::co(i) - PL::C0;
            if ((i == 0 || PL::pt(i - 1) != t) && t + 1 < NT) nrd += read_tile(t + 1);   // the next tile, one tile ahead
            if (EPI == 2 && i + 2 < n) {
                rb[(i + 2) % 3] = *(const uint4 *)(smem + (OUT - 256) + (g.b(PL::pt(i + 2), 4) ^ ((PL::co(i + 2) >> 1) << 6)));
                ++nrd;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (live(t, k0 + k)) {   // (the bias went in with the first live k-step, <= 8)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[(k0 + k) % DA][c]),
                                                                    as_bf16x8(Bf[t & 1][k]), acc[i], 0, 0, 0);
                    ++nm;
                }
            if (EPI == 2) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(id[PL::co(i) & 1]), as_bf16x8(rb[i % 3]), acc[i],
                                                                0, 0, 0);
                ++nm;
            }
        }
        if (i >= D) {
            const int j = i - D;
            const int off = OUT + (g.epi[PL::pt(j)] ^ (PL::co(j) << 5));
            *(uint2 *)(smem + off) = make_uint2(pack_relu_bf16x2(acc[j][0], acc[j][1]), pack_relu_bf16x2(acc[j][2], acc[j][3]));
            nv = 9;
            nw = 1;
        }
        // issue order: each MFMA followed by 2 of the epilogue's VALU, then the rest, the
        // store and the reads
#pragma unroll
        for (int k = 0; k < 5; ++k)
            if (k < nm) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                if (nv) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
            }
        if (nv && nm < 5) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        if (nv && nm < 4) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        if (nv && nm < 3) __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        if (nw) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
#pragma unroll
        for (int k = 0; k < 5; ++k)
            if (k < nrd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// EPI > 0 fuses the layer's epilogue into its last tap (k-steps 16 and 17): the
// final tap runs task-major -- each task's two MFMAs back to back (EPI = 2: plus
// the residual MFMA of final_tap_epilogue), and the ReLU/bf16 pack and LDS store of
// task i - 2 ride in the MFMA gaps of task i instead of a serial epilogue after
// the k-loop.  Safe to store while other waves still run this layer: OUT is not
// this layer's input, and a residual read that meets another wave's fresh store
// in the other 16 channels of its 32-channel block multiplies it by zero.
template <int W, int CT, int NPT, int S, int IN, int DA, int DB, int EPI = 0, int OUT = 0>
__device__ __forceinline__ void conv_mfma(uint8_t *smem, const Geo<Plan<W, CT, NPT>::NT> &g, const float *bias,
                                          const uint4 *__restrict__ w, const uint4 *__restrict__ wn, int lane,
                                          uint4 (&A)[DA][Plan<W, CT, NPT>::CTL],
                                          f32x4 (&acc)[Plan<W, CT, NPT>::n],
                                          const int (&hoff)[Plan<W, CT, NPT>::NT],
                                          f32x4 (&dacc)[Plan<W, CT, NPT>::NDA],
                                          unsigned long long *kst = nullptr) {
    using PL = Plan<W, CT, NPT>;
    constexpr int NT = PL::NT, CTL = PL::CTL;
    (void)kst;
#ifdef SPAI_DIAG_KSTEP
    if (kst) kst[20] = __builtin_amdgcn_s_memtime();   // stamp 44: conv start
#endif
    static_assert(kKStepsRes % DA == 0, "the carried A ring needs DA | k-steps per layer");
    const int q = lane >> 4;
    f32x4 bv[CTL];
#pragma unroll
    for (int c = 0; c < CTL; ++c) {
        const float4 b = *(const float4 *)(bias + (PL::C0 + c) * 16 + 4 * q);
        bv[c] = f32x4{b.x, b.y, b.z, b.w};
    }
    const uint4 *wl = w + PL::C0 * 64 + lane;
    const uint4 *wnl = wn + PL::C0 * 64 + lane;
    // (tile, tap) pairs whose rows are all off the board for that tap are skipped
    // (tap_skip); the indices below are compile-time constants once unrolled
    // EPI = 3, the head conv: co tile 3 (channels 48..63) does not exist -- its
    // tasks, weight loads, and the B reads of tiles with no other task are dropped
    auto task_on = [](int i) { return !(EPI == 3 && PL::co(i) == 3); };
    auto tile_on = [&](int t) {
        bool on = false;
        for (int i = 0; i < PL::n; ++i) on = on || (PL::pt(i) == t && task_on(i));
        return on;
    };
    auto live = [&](int t, int ks) { return tile_on(t) && !((tap_skip(S, PL::gpt(t)) >> (ks >> 1)) & 1); };
#ifndef SPAI_DEFER_EPI   // the k-loop in k-step order (production)
    uint4 B[DB][NT];
#pragma unroll
    for (int kb = 0; kb < DB - 1; ++kb) {
        const int tap = kb >> 1, flip = (kb & 1) << 6;
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (live(t, kb)) B[kb][t] = *(const uint4 *)(smem + (IN - 256) + (g.b(t, tap) ^ flip));
    }
    constexpr int la = DA - 1, lb = DB - 1;
    // A for k-step ks + la (this layer's, or the next layer's first k-steps)
    auto load_a = [&](int ks) {
        if (ks + la < kKStepsRes) {
#pragma unroll
            for (int c = 0; c < CTL; ++c)
                if (!(EPI == 3 && PL::C0 + c == 3)) A[(ks + la) % DA][c] = exp_a(wl[((ks + la) * CT + c) * 64], lane, ks + c);
        } else if (EPI != 3) {   // (nothing follows the head)
#pragma unroll
            for (int c = 0; c < CTL; ++c) A[(ks + la) % DA][c] = exp_a(wnl[((ks + la - kKStepsRes) * CT + c) * 64], lane, ks + c);
        }
    };
    // k-steps in the task-major final phase: 4 with SPAI_FINAL2 at the position-major sizes
    constexpr int KF = (EPI == 1 || EPI == 2) && kFinal2 && PL::MODE == 0 ? 4 : 2;
    constexpr int kBEnd = KF == 2 ? kKStepsRes : kKStepsRes - KF;   // the ring's B reads end here
#pragma unroll
    for (int ks = 0; ks < kKStepsRes; ++ks) {
        if constexpr (KF == 4) if (ks == kKStepsRes - 4) {
            // the next layer's second k-step's weights go to the slot k-step 13 left; the
            // slots of k-steps 14-16 refill after the final phase
            load_a(ks);
            final_phase2<W, CT, NPT, S, IN, DA, EPI, OUT>(smem, g, lane, A, acc);
            load_a(ks + 1);
            load_a(ks + 2);
            load_a(ks + 3);
#ifdef SPAI_DIAG_KSTEP
            if (kst) kst[ks] = __builtin_amdgcn_s_memtime();
#endif
            break;
        }
        if constexpr (EPI > 0 && KF == 2) if (ks == kKStepsRes - 2) {
            // B reads of the last k-step (if not issued yet), then the fused final tap;
            // k-step 17's A prefetch waits for the MFMAs that read the slot it refills
            if (ks + lb < kKStepsRes) {
                const int tap = (ks + lb) >> 1, flip = ((ks + lb) & 1) << 6;
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    if (live(t, ks + lb)) B[(ks + lb) % DB][t] = *(const uint4 *)(smem + (IN - 256) + (g.b(t, tap) ^ flip));
            }
            load_a(ks);
            final_tap_epilogue<W, CT, NPT, S, DA, DB, EPI, OUT>(smem, g, lane, A, B, bv, acc, hoff, dacc);
            load_a(ks + 1);
#ifdef SPAI_DIAG_KSTEP
            if (kst) kst[ks] = __builtin_amdgcn_s_memtime();
#endif
            break;
        }
        load_a(ks);
        int nr = 0;   // B reads issued this k-step (for the issue-order hints)
        if (ks + lb < kBEnd) {
            const int tap = (ks + lb) >> 1, flip = ((ks + lb) & 1) << 6;
#pragma unroll
            for (int t = 0; t < NT; ++t)
                if (live(t, ks + lb)) {
                    B[(ks + lb) % DB][t] = exp_b(smem + (IN - 256) + (g.b(t, tap) ^ flip), lane, ks + t);
                    ++nr;
                }
        }
        int nm = 0;
#pragma unroll
        for (int i = 0; i < PL::n; ++i)
            if (task_on(i) && live(PL::pt(i), ks)) {
                const int t = PL::gpt(PL::pt(i));
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[ks % DA][PL::co(i) - PL::C0]),
                                                                as_bf16x8(B[ks % DB][PL::pt(i)]),
                                                                ks == first_kstep(S, t) ? bv[PL::co(i) - PL::C0]
                                                                                        : acc[i], 0, 0, 0);
                ++nm;
            }
        // issue order for this k-step: each MFMA followed by up to 2 VALU, one
        // LDS read (next B) and one weight load (A, DA-1 ahead)
        const int ng = nm > nr ? nm : nr;
#if SPAI_ISSUE_HINTS
#pragma unroll
        for (int i = 0; i < PL::n; ++i) {
            if (i < ng) {
                if (i < nm) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                if (i < nr) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (i < CTL) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
#else
        (void)ng;
#endif
#if SPAI_KSTEP_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
#ifdef SPAI_DIAG_KSTEP
        if (kst) kst[ks] = __builtin_amdgcn_s_memtime();
#endif
    }
#else   // SPAI_DEFER_EPI: K-half-0 k-steps first, the previous layer's deferred epilogue in their gaps
    uint4 B[DB][NT];
    // B fragments of the j-th executed k-step (its tap and K half)
    auto read_b = [&](int j) {
        const int ks = kstep_of(j), tap = ks >> 1, flip = (ks & 1) << 6;
        int nr = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (live(t, ks)) {
                B[j % DB][t] = exp_b(smem + (IN - 256) + (g.b(t, tap) ^ flip), lane, j + t);
                ++nr;
            }
        return nr;
    };
#pragma unroll
    for (int kb = 0; kb < DB - 1; ++kb) read_b(kb);
    constexpr int la = DA - 1, lb = DB - 1;
    // A for the k-step executed (j + la)-th (this layer's, or the next layer's first ones)
    auto load_a = [&](int j) {
        if (j + la < kKStepsRes) {
            const int ks = kstep_of(j + la);
#pragma unroll
            for (int c = 0; c < CTL; ++c)
                if (!(EPI == 3 && PL::C0 + c == 3)) A[(j + la) % DA][c] = exp_a(wl[(ks * CT + c) * 64], lane, j + c);
        } else if (EPI != 3) {   // (nothing follows the head)
            const int ks = kstep_of(j + la - kKStepsRes);
#pragma unroll
            for (int c = 0; c < CTL; ++c) A[(j + la) % DA][c] = exp_a(wnl[(ks * CT + c) * 64], lane, j + c);
        }
    };
    // deferred epilogue of the previous layer (its co-tile 2/3 tasks, output channels
    // 32-63 of IN) in the MFMA gaps of the K-half-0 k-steps; the barrier at the top of
    // step jb publishes them before the first K-half-1 B reads (issued lb steps ahead)
    constexpr int jb = 9 - lb;
    constexpr bool din = PL::ND > 0;
#pragma unroll
    for (int j = 0; j < kKStepsRes; ++j) {
        const int ks = kstep_of(j);
        if constexpr (din) if (j == jb) __syncthreads();
        if constexpr (EPI > 0) if (j == kKStepsRes - 2) {
            // B reads of the last k-step (if not issued yet), then the fused final tap;
            // the last k-step's A prefetch waits for the MFMAs that read the slot it refills
            if (j + lb < kKStepsRes) read_b(j + lb);
            load_a(j);
            final_tap_epilogue<W, CT, NPT, S, DA, DB, EPI, OUT>(smem, g, lane, A, B, bv, acc, hoff, dacc);
            load_a(j + 1);
#ifdef SPAI_DIAG_KSTEP
            if (kst) kst[j] = __builtin_amdgcn_s_memtime();
#endif
            break;
        }
        load_a(j);
        const int nr = j + lb < kKStepsRes ? read_b(j + lb) : 0;   // B reads issued this k-step (issue hints)
        int nm = 0;
#pragma unroll
        for (int i = 0; i < PL::n; ++i)
            if (task_on(i) && live(PL::pt(i), ks)) {
                const int t = PL::gpt(PL::pt(i));
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[j % DA][PL::co(i) - PL::C0]),
                                                                as_bf16x8(B[j % DB][PL::pt(i)]),
                                                                ks == first_kstep(S, t) ? bv[PL::co(i) - PL::C0]
                                                                                        : acc[i], 0, 0, 0);
                ++nm;
            }
        int ndw = 0;   // deferred epilogue tasks stored this k-step (tasks [j n / jb, (j + 1) n / jb))
        if constexpr (din) {
#pragma unroll
            for (int i = 0; i < PL::n; ++i)
                if (j < jb && i >= j * PL::n / jb && i < (j + 1) * PL::n / jb && PL::deferred(i)) {
                    const int off = IN + (g.epi[PL::pt(i)] ^ (PL::co(i) << 5));
                    *(uint2 *)(smem + off) = make_uint2(pack_relu_bf16x2(dacc[i][0], dacc[i][1]),
                                                        pack_relu_bf16x2(dacc[i][2], dacc[i][3]));
                    ++ndw;
                }
        }
        // issue order for this k-step: each MFMA followed by up to 2 VALU, one
        // LDS read (next B) and one weight load (A, DA-1 ahead); deferred stores last
        const int ng = nm > nr ? nm : nr;
#pragma unroll
        for (int i = 0; i < PL::n; ++i) {
            if (i < ng) {
                if (i < nm) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                if (i < nr) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (i < CTL) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
        if constexpr (din) {
#pragma unroll
            for (int k = 0; k < PL::n; ++k)
                if (k < ndw) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#ifdef SPAI_DIAG_KSTEP
        if (kst) kst[j] = __builtin_amdgcn_s_memtime();
#endif
    }
#endif
}

template <int CT, int C0, int CTL, int DA>
__device__ __forceinline__ void load_a_first(const uint4 *__restrict__ w, int lane, uint4 (&A)[DA][CTL]) {
#pragma unroll
    for (int k = 0; k < DA - 1; ++k)
#pragma unroll
        for (int c = 0; c < CTL; ++c) A[k][c] = w[(kstep_of(k) * CT + C0 + c) * 64 + lane];
}

// epilogue for a 64-channel bf16 output: relu(acc) -> LDS at OUT (the stem's;
// the trunk and head convs fuse theirs into the last tap, final_tap_epilogue)
template <int W, int NPT, int OUT>
__device__ __forceinline__ void epilogue_act(uint8_t *smem, const Geo<Plan<W, 4, NPT>::NT> &g, f32x4 (&acc)[Plan<W, 4, NPT>::n],
                                             f32x4 (&dacc)[Plan<W, 4, NPT>::NDA]) {
    using PL = Plan<W, 4, NPT>;
#pragma unroll
    for (int i = 0; i < PL::n; ++i) {
        if (PL::deferred(i)) {   // stored by the first trunk conv's K-half-0 k-steps
            dacc[i] = acc[i];
            continue;
        }
        const int off = OUT + (g.epi[PL::pt(i)] ^ (PL::co(i) << 5));
        *(uint2 *)(smem + off) = make_uint2(pack_relu_bf16x2(acc[i][0], acc[i][1]), pack_relu_bf16x2(acc[i][2], acc[i][3]));
    }
}

// stem: one k-step, k = tap*3 + plane (27 of 32 used).  Bitboard path: the
// neighbour planes N[s][k] (one u64 per sample/tap/plane, built at kernel start)
// hold at bit col*7+row the value of that cell's (dh,dw) neighbour, so lane
// element j of a position is bit (col*7+row) of N[s][8q+j].  FROM_X path
// (Net::forward on arbitrary inputs): gather the fp32 input tensor.
template <int W, int S, bool FROM_X>
__device__ __forceinline__ void stem(uint8_t *smem, const NetParams &P, const float *__restrict__ x, int base_slot,
                                     int valid, int lane, const Geo<Plan<W, 4, npt_of(S)>::NT> &g,
                                     const int (&aux)[Plan<W, 4, npt_of(S)>::NT],
                                     f32x4 (&dacc)[Plan<W, 4, npt_of(S)>::NDA]) {
    constexpr int NPT = npt_of(S);
    using PL = Plan<W, 4, NPT>;
    constexpr int NT = PL::NT;
    const int q = lane >> 4;
    uint4 a[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = ((const uint4 *)(smem + kWStem))[c * 64 + lane];
    uint4 bv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int s = aux[t] & 255, b = aux[t] >> 8;   // b = col*7 + row of the row's cell
        uint16_t e[8];
        if (!FROM_X) {
            const uint4 *np = (const uint4 *)(smem + kPlanes) + s * (kPlaneRow / 2) + q * 4;   // N[s][8q .. 8q+7]
#pragma unroll
            for (int j2 = 0; j2 < 4; ++j2) {
                const uint4 w4 = np[j2];
                const uint64_t n0 = (uint64_t)w4.x | ((uint64_t)w4.y << 32), n1 = (uint64_t)w4.z | ((uint64_t)w4.w << 32);
                e[2 * j2] = ((n0 >> b) & 1ull) ? 0x3F80u : 0u;
                e[2 * j2 + 1] = ((n1 >> b) & 1ull) ? 0x3F80u : 0u;
            }
        } else {
            const int h = b % c4::kCols, wc = b / c4::kCols;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int kk = 8 * q + j;
                float v = 0.f;
                if (kk < 27) {
                    const int tap = kk / 3, ch = kk - tap * 3;
                    const int hh = h + tap / 3 - 1, ww = wc + tap % 3 - 1;
                    if ((unsigned)hh < (unsigned)c4::kRows && (unsigned)ww < (unsigned)c4::kCols && s < valid)
                        v = x[((size_t)(base_slot + s) * 3 + ch) * c4::kCells + hh * c4::kCols + ww];
                }
                e[j] = __builtin_bit_cast(uint16_t, (__bf16)v);
            }
        }
        bv[t] = make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16, e[4] | (uint32_t)e[5] << 16,
                           e[6] | (uint32_t)e[7] << 16);
    }
    const float *bias = (const float *)(smem + kBias);
    f32x4 b4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float4 b = *(const float4 *)(bias + c * 16 + 4 * q);
        b4[c] = f32x4{b.x, b.y, b.z, b.w};
    }
    f32x4 acc[PL::n];
#pragma unroll
    for (int i = 0; i < PL::n; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[PL::co(i)]), as_bf16x8(bv[PL::pt(i)]),
                                                        b4[PL::co(i)], 0, 0, 0);
    epilogue_act<W, NPT, kX>(smem, g, acc, dacc);
}

// The head conv (64 -> 32 policy + 3 value channels) on the 64-channel layers'
// plan, geometry and A ring: the last residual conv prefetches its first
// weights, and co tile 3 is dropped (conv_mfma EPI = 3), whose fused epilogue
// writes relu(bf16) features to H[s][cell * 36 + c].
template <int W, int S, int DA>
__device__ __forceinline__ void head_layer(uint8_t *smem, const NetParams &P, int lane,
                                           const Geo<Plan<W, 4, npt_of(S)>::NT> &g,
                                           const int (&aux)[Plan<W, 4, npt_of(S)>::NT],
                                           uint4 (&A)[DA][Plan<W, 4, npt_of(S)>::CTL],
                                           uint4 (&wlin)[kLinWPer],
                                           f32x4 (&dacc)[Plan<W, 4, npt_of(S)>::NDA]) {
    constexpr int NPT = npt_of(S);
    using PL = Plan<W, 4, NPT>;
    int hoff[PL::NT];   // head-feature offset of each tile's row (-1: padding)
#pragma unroll
    for (int t = 0; t < PL::NT; ++t) {
        const int s = aux[t] & 255, b = aux[t] >> 8;   // b = col*7 + row
        hoff[t] = s < S ? s * lin_pitch(S) + ((b % c4::kCols) * c4::kCols + b / c4::kCols) * kHC : -1;
    }
#pragma unroll
    for (int i = 0; i < kLinWPer; ++i) wlin[i] = P.w_lin[(W * kLinWPer + i) * 64 + lane];   // consumed after the head conv
    f32x4 acc[PL::n];
    conv_mfma<W, 4, NPT, S, kX, DA, b_depth(S), 3, kH>(smem, g, (const float *)(smem + kBias) + kHid * (1 + 2 * P.blocks),
                                                      P.w_head, P.w_head, lane, A, acc, hoff, dacc);
#ifdef SPAI_DIAG
    if (kDiagHead) stamp(P, W, lane, 17);
#endif
    // K padding [1512, 1536) of each row: 6 words of 8 B
    uint16_t *H = (uint16_t *)(smem + kH);
    if (W == 0 && lane < S * 6)
        *(uint2 *)(H + (lane / 6) * lin_pitch(S) + kLinFeat + 4 * (lane % 6)) = make_uint2(0u, 0u);
#ifdef SPAI_DIAG
    if (kDiagHead) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp(P, W, lane, 18);
    }
#endif
}

// fused policy|value linear on MFMA: out[s][o] = sum_k H[s][k] * Wl[o][k]
// (o < 7 policy logits over k < 1344, o = 7 value pre-activation over
// 1344 <= k < 1470; connect_four.rs:63-64,69-70), the two K halves packed into
// one 16-column B fragment (kLinHalves).  Wave W takes B k-steps [6W, 6W+6) of
// 24, their fragments held in registers (wlin); partial sums go to LDS.
template <int W, int S>
__device__ __forceinline__ void linear_mfma(uint8_t *smem, int lane, const uint4 (&wlin)[kLinWPer]) {
    constexpr int k0 = (kLinBSteps / kWaves) * W, k1 = k0 + kLinBSteps / kWaves;
    const int m = lane & 15, q = lane >> 4;
    // A row m: position m & 7 over K half m >> 3
    const int s = m & 7, kh = m >> 3;
    const uint8_t *hrow = s < S ? smem + kH + (s * lin_pitch(S) + kh * (kLinK / 2)) * 2 + q * 16 : smem + kZ + q * 16;
    const int hstep = s < S ? 64 : 0;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = k0; ks < k1; ++ks) {
        const uint4 a = *(const uint4 *)(hrow + ks * hstep);
        const uint4 b = wlin[ks - k0];
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a), as_bf16x8(b), acc, 0, 0, 0);
    }
    // D[row 4q + r][col n = lane & 15]
    float *L = (float *)(smem + kL) + W * kLinHalves * 64;
    if ((q >> 1) == (m >> 3)) {   // keep the diagonal blocks: row half (q >> 1) == column half (n >> 3)
#pragma unroll
        for (int r = 0; r < 4; ++r) L[(q >> 1) * 64 + (4 * (q & 1) + r) * 8 + (m & 7)] = acc[r];
    }
}


// ---------------------------------------------------------------- split-K trunk conv (SPAI_W8)
// Plan wave W's tasks over half of K: KH = 1 the k-steps of input channels 0-31
// of every tap (even k-steps), KH = 2 those of channels 32-63 (odd).  The A
// ring runs over the wave's 9 local k-steps (DA | 9) and carries the next
// layer's first ones across the boundary.  Then the two waves of the pair swap
// partial sums through LDS: each finishes half of the tasks as
// (first-half sum incl. bias) + (second-half sum), adds the residual by the
// identity MFMA (EPI = 2) and stores relu/bf16 to OUT.
template <int W, int NPT>
__device__ __forceinline__ int split_keep_lo() {
    return (Plan<W, 4, NPT>::n + 1) / 2;   // tasks [0, h) finish on the KH = 1 wave, [h, n) on the KH = 2 wave
}
template <int W, int NPT, int S, int IN, int DA, int DB, int EPI, int OUT, int KH>
__device__ __forceinline__ void conv_split(uint8_t *smem, const Geo<Plan<W, 4, NPT>::NT> &g, const float *bias,
                                           const uint4 *__restrict__ w, const uint4 *__restrict__ wn, int lane,
                                           uint4 (&A)[DA][Plan<W, 4, NPT>::CTL], f32x4 (&acc)[Plan<W, 4, NPT>::n]) {
#ifdef SPAI_W8
    using PL = Plan<W, 4, NPT>;
    constexpr int NT = PL::NT, CTL = PL::CTL, n = PL::n, KL = kKStepsRes / 2, par = KH - 1;
    static_assert(KH == 1 || KH == 2, "split half");
    static_assert(KL % DA == 0, "the carried A ring needs DA | local k-steps");
    static_assert(n <= kSplitMaxN, "partial-sum buffer");
    const int q = lane >> 4;
    f32x4 bv[CTL];
#pragma unroll
    for (int c = 0; c < CTL; ++c) {
        if (KH == 1) {
            const float4 b = *(const float4 *)(bias + (PL::C0 + c) * 16 + 4 * q);
            bv[c] = f32x4{b.x, b.y, b.z, b.w};
        } else {
            bv[c] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    const uint4 *wl = w + PL::C0 * 64 + lane;
    const uint4 *wnl = wn + PL::C0 * 64 + lane;
    auto live = [](int t, int j) { return !((tap_skip(S, PL::gpt(t)) >> j) & 1); };   // local step j = tap j
    constexpr int la = DA - 1, lb = DB - 1;
    uint4 B[DB][NT];
#pragma unroll
    for (int j = 0; j < lb; ++j)
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (live(t, j)) B[j][t] = *(const uint4 *)(smem + (IN - 256) + (g.b(t, j) ^ (par << 6)));
    auto load_a = [&](int j) {
        const int jj = j + la;
#pragma unroll
        for (int c = 0; c < CTL; ++c)
            A[jj % DA][c] = jj < KL ? wl[((2 * jj + par) * 4 + c) * 64] : wnl[((2 * (jj - KL) + par) * 4 + c) * 64];
    };
#pragma unroll
    for (int j = 0; j < KL; ++j) {
        load_a(j);
        int nr = 0;
        if (j + lb < KL) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
                if (live(t, j + lb)) {
                    B[(j + lb) % DB][t] = *(const uint4 *)(smem + (IN - 256) + (g.b(t, j + lb) ^ (par << 6)));
                    ++nr;
                }
        }
        int nm = 0;
#pragma unroll
        for (int i = 0; i < n; ++i)
            if (live(PL::pt(i), j)) {
                const int t = PL::gpt(PL::pt(i));
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(A[j % DA][PL::co(i) - PL::C0]),
                                                                as_bf16x8(B[j % DB][PL::pt(i)]),
                                                                2 * j == first_kstep(S, t) ? bv[PL::co(i) - PL::C0]
                                                                                           : acc[i], 0, 0, 0);
                ++nm;
            }
        const int ng = nm > nr ? nm : nr;
#pragma unroll
        for (int i = 0; i < n; ++i) {
            if (i < ng) {
                if (i < nm) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
                if (i < nr) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                if (i < CTL) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // swap half of the partial sums with the partner wave
    constexpr int h = (n + 1) / 2;
    constexpr int g0 = KH == 1 ? h : 0, g1 = KH == 1 ? n : h;   // given away
    constexpr int k0 = KH == 1 ? 0 : h, k1 = KH == 1 ? h : n;   // kept and finished here
    f32x4 *part = (f32x4 *)(smem + kPart) + (size_t)W * kSplitMaxN * 64 + lane;
#pragma unroll
    for (int i = g0; i < g1; ++i) part[i * 64] = acc[i];
    __syncthreads();
    uint4 id[2];
    if (EPI == 2) {
        const int m = lane & 15;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int jj = 16 * hh + m - 8 * q;
            uint32_t wv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) wv[e] = jj == 2 * e ? 0x3F80u : jj == 2 * e + 1 ? 0x3F800000u : 0u;
            id[hh] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
    }
#pragma unroll
    for (int i = k0; i < k1; ++i) {
        const f32x4 p = part[i * 64];
        f32x4 a = KH == 1 ? acc[i] + p : p + acc[i];   // (first K half) + (second K half)
        if (EPI == 2) {
            const uint4 rb = *(const uint4 *)(smem + (OUT - 256) + (g.b(PL::pt(i), 4) ^ ((PL::co(i) >> 1) << 6)));
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(id[PL::co(i) & 1]), as_bf16x8(rb), a, 0, 0, 0);
        }
        const int off = OUT + (g.epi[PL::pt(i)] ^ (PL::co(i) << 5));
        *(uint2 *)(smem + off) = make_uint2(pack_relu_bf16x2(a[0], a[1]), pack_relu_bf16x2(a[2], a[3]));
    }
#else
    (void)smem, (void)g, (void)bias, (void)w, (void)wn, (void)lane, (void)A, (void)acc;
#endif
}

template <int KH, int CTL, int C0, int DA>
__device__ __forceinline__ void load_a_first_split(const uint4 *__restrict__ w, int lane, uint4 (&A)[DA][CTL]) {
#pragma unroll
    for (int j = 0; j < DA - 1; ++j)
#pragma unroll
        for (int c = 0; c < CTL; ++c) A[j][c] = w[((2 * j + KH - 1) * 4 + C0 + c) * 64 + lane];
}

template <int W, int S, bool FROM_X, int KH>
__device__ __forceinline__ void torso_and_heads(uint8_t *smem, const NetParams &P, const float *__restrict__ x,
                                                int base, int valid, int lane, const Geo<Plan<W, 4, npt_of(S)>::NT> &g,
                                                const int (&aux)[Plan<W, 4, npt_of(S)>::NT]) {
    constexpr int NPT = npt_of(S);
    using PL4 = Plan<W, 4, NPT>;
    constexpr size_t kLayer = (size_t)kKStepsRes * 4 * 64;
    const float *bias = (const float *)(smem + kBias);
    if constexpr (KH > 0) {   // SPAI_W8: split-K trunk on 8 waves, stem / head / linear on waves 0-3
        constexpr int DA = 3, DB = b_depth(S), SW = KH == 2 ? -1 : W;
        uint4 A[DA][PL4::CTL];
        if (P.blocks > 0) load_a_first_split<KH, PL4::CTL, PL4::C0, DA>(P.w_res, lane, A);
        static_assert(!kDefer, "SPAI_W8 has no deferred epilogue");
        f32x4 dacc[PL4::NDA];
        if (KH == 1) stem<W, S, FROM_X>(smem, P, x, base, valid, lane, g, aux, dacc);
        __syncthreads();
        stamp(P, SW, lane, 1);
        for (int b = 0; b < P.blocks; ++b) {
            f32x4 acc[PL4::n];
            const int l1 = 2 * b, l2 = 2 * b + 1;
            conv_split<W, NPT, S, kX, DA, DB, 1, kY, KH>(smem, g, bias + kHid * (1 + l1), P.w_res + l1 * kLayer,
                                                        P.w_res + l2 * kLayer, lane, A, acc);
            layer_barrier();
            if (l1 < 12) stamp(P, SW, lane, 2 + l1);
            conv_split<W, NPT, S, kY, DA, DB, 2, kX, KH>(smem, g, bias + kHid * (1 + l2), P.w_res + l2 * kLayer,
                                                        b + 1 < P.blocks ? P.w_res + (l2 + 1) * kLayer : P.w_res + l2 * kLayer,
                                                        lane, A, acc);
            layer_barrier();
            if (l2 < 12) stamp(P, SW, lane, 2 + l2);
        }
        uint4 wlin[kLinWPer];
        if (KH == 1) {
            constexpr int DH = a_depth(S);
            uint4 Ah[DH][PL4::CTL];
            load_a_first<4, PL4::C0, PL4::CTL, DH>(P.w_head, lane, Ah);
            head_layer<W, S, DH>(smem, P, lane, g, aux, Ah, wlin, dacc);
        }
        __syncthreads();
        stamp(P, SW, lane, 14);
        if (KH == 1) linear_mfma<W, S>(smem, lane, wlin);
        return;
    }
    constexpr int DA = a_depth(S), DB = b_depth(S);
    uint4 A[DA][PL4::CTL];
    load_a_first<4, PL4::C0, PL4::CTL, DA>(P.blocks > 0 ? P.w_res : P.w_head, lane, A);
    f32x4 dacc[PL4::NDA];   // deferred epilogue accumulators, handed from each layer to the next
    stem<W, S, FROM_X>(smem, P, x, base, valid, lane, g, aux, dacc);
    __syncthreads();
    stamp(P, W, lane, 1);
#ifdef SPAI_C4_BLOCK_UNROLL
#pragma unroll SPAI_C4_BLOCK_UNROLL
#endif
    for (int b = 0; b < P.blocks; ++b) {   // relu(x + BN(conv(relu(BN(conv(x)))))), model/mod.rs:152-165
        f32x4 acc[Plan<W, 4, NPT>::n];
        const int l1 = 2 * b, l2 = 2 * b + 1;
        unsigned long long *kst = nullptr;
#ifdef SPAI_DIAG_KSTEP
        if (b == 1 && P.stamps && lane == 0) kst = P.stamps + ((size_t)blockIdx.x * kWaves + W) * kStamps + 24;
#endif
        conv_mfma<W, 4, NPT, S, kX, DA, DB, 1, kY>(smem, g, bias + kHid * (1 + l1), P.w_res + l1 * kLayer,
                                                                    P.w_res + l2 * kLayer, lane, A, acc, aux, dacc, kst);
#ifdef SPAI_DIAG_KSTEP
        if (kst) kst[18] = __builtin_amdgcn_s_memtime();
#endif
#ifdef SPAI_DIAG
        if (b == 0 && !kDiagHead && !kDiagEntry) {   // make the k-loop's results visible before the stamp
            asm volatile("" ::"v"(acc[0][0]), "v"(acc[PL4::n - 1][3]));
            stamp(P, W, lane, 17);
        }
#endif
#ifdef SPAI_DIAG
        if (b == 0 && !kDiagHead && !kDiagEntry) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            stamp(P, W, lane, 18);
        }
#endif
        layer_barrier();
#ifdef SPAI_DIAG_KSTEP
        if (kst) kst[19] = __builtin_amdgcn_s_memtime();
#endif
#ifdef SPAI_DIAG
        if (b == 0 && !kDiagHead && !kDiagEntry) stamp(P, W, lane, 19);
#endif
        if (l1 < 12) stamp(P, W, lane, 2 + l1);
        conv_mfma<W, 4, NPT, S, kY, DA, DB, 2, kX>(smem, g, bias + kHid * (1 + l2), P.w_res + l2 * kLayer,
                            b + 1 < P.blocks ? P.w_res + (l2 + 1) * kLayer : P.w_head, lane, A, acc, aux, dacc);
        layer_barrier();
        if (l2 < 12) stamp(P, W, lane, 2 + l2);
    }
    if (kDiagHead) stamp(P, W, lane, 19);   // diagnostic head mode: 19 = before the head, 17 = head k-loop, 18 = H written
    uint4 wlin[kLinWPer];
    head_layer<W, S, DA>(smem, P, lane, g, aux, A, wlin, dacc);
    __syncthreads();
    stamp(P, W, lane, 14);
    linear_mfma<W, S>(smem, lane, wlin);
}

// Group size for `count` leaves on `grid` workgroups: the fewest rounds R of at
// most kS positions per workgroup, then the smallest S that still fits R rounds
// (a group's latency grows with its npt_of(S) position tiles, so e.g. 3000
// leaves run as 2 rounds of S = 6 (16 tiles), not 2 rounds of S = 8 (21 tiles)).
__host__ __device__ inline int group_size(uint32_t count, uint32_t grid) {
    const uint32_t cap = grid * (uint32_t)kSRun;
    const uint32_t rounds = count ? (count + cap - 1) / cap : 1u;
    const uint32_t per = grid * rounds;
    const int g = (int)((count + per - 1) / per);
    return g < 1 ? 1 : g > kSRun ? kSRun : g;
}

// Group size when `conc` search chains' forwards share the CUs (conc > 1): their
// workgroups queue for the same CUs, so the iteration is bound by the forwards'
// summed CU time as much as by one chain's forward latency plus its tree
// kernels.  From the latency-optimal size upwards, the size minimising
// max(conc x CU cycles / grid, forward latency + kChainCycles) on the measured
// per-group cycles (profiles/r04/search_ab/phases_pro.txt) is taken: larger
// groups cost fewer CU cycles per leaf (29k at S = 1, 15.7k at S = 4, 12.6k at
// S = 8).  The results do not depend on S.
constexpr float kGroupCycles[kS + 1] = {0.f, 29200.f, 45500.f, 58600.f, 62900.f, 81200.f, 86200.f, 94700.f, 100500.f};
constexpr float kLaunchCycles = 4200.f;   // kernel entry to the first group (~2 us)
#ifndef SPAI_CONC_CHAIN_CYCLES
#define SPAI_CONC_CHAIN_CYCLES 31000.f
#endif
#ifndef SPAI_CONC_MIN_COUNT
#define SPAI_CONC_MIN_COUNT 600
#endif
constexpr float kChainCycles = SPAI_CONC_CHAIN_CYCLES;   // the chain's tree kernels and launch gaps per iteration (~15 us)
// below this many leaves the chains' forwards are short and the model's CU term
// overstates their contention: measured slower there (moves 26-41 of a bench step,
// profiles/r04/group_policy)
constexpr uint32_t kConcMinCount = SPAI_CONC_MIN_COUNT;
__host__ __device__ inline int group_size_conc(uint32_t count, uint32_t grid, int conc) {
    const int s0 = group_size(count, grid);
    if (conc <= 1 || count < kConcMinCount) return s0;
    float best = 3.0e38f;
    int bs = s0;
    for (int S = s0; S <= kSRun; ++S) {
        const uint32_t wgs = (count + S - 1) / S, rounds = (wgs + grid - 1) / grid;
        const float cu = (float)wgs * kGroupCycles[S] + (float)(wgs < grid ? wgs : grid) * kLaunchCycles;
        const float lat = (float)rounds * kGroupCycles[S] + kLaunchCycles;
        const float t = fmaxf((float)conc * cu / (float)grid, lat + kChainCycles);
        if (t < best) {
            best = t;
            bs = S;
        }
    }
    return bs;
}

// The group loop of one (wave, group size) variant.
template <int W, int S, bool FROM_X, int KH>
__device__ __forceinline__ void run_groups(uint8_t *smem, const NetParams &P, uint32_t count, int ngroups,
                                           const uint64_t *__restrict__ mine, const uint64_t *__restrict__ theirs,
                                           const float *__restrict__ x, float *__restrict__ priors,
                                           float *__restrict__ value, float *__restrict__ logits, int tid) {
    constexpr int wave = KH == 2 ? -1 : W;   // (stamps: one wave of each SIMD pair)
    const int lane = tid & 63;
    for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        // hide the lane id from loop-invariant code motion: the trunk geometry (and
        // every layer's per-lane addressing) hoisted out of the loop would stay live
        // through the head, and the forward's register footprint decides whether the
        // other search chain's tree kernels can run beside it (scripts/kernel_regs.py)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        ln &= 63;   // restore the known range for the compiler
        Geo<Plan<W, 4, npt_of(S)>::NT> g;
        int aux[Plan<W, 4, npt_of(S)>::NT];
        load_geo<W, npt_of(S), S>(P, ln, g, aux);   // before the bitboard loads: the two latencies overlap
        const int base = grp * S;
        const int valid = min(S, (int)count - base);
        if (tid < kS) {
            uint64_t m = 0, t = 0;
            if (!FROM_X && tid < valid) {
                m = mine[base + tid];
                t = theirs[base + tid];
            }
            ((uint64_t *)(smem + kB))[2 * tid] = m;
            ((uint64_t *)(smem + kB))[2 * tid + 1] = t;
        }
#ifdef SPAI_DIAG_ENTRY
        if (grp == (int)blockIdx.x) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stamp(P, wave, lane, 18);
        }
#endif
        if (!FROM_X && tid < kStemThreads) {   // neighbour planes N[s][k]: k = tap*3 + plane, shifted so bit b = value at b's neighbour
            const int s = tid >> 5, k = tid & 31;
            uint64_t v = 0;
            if (k < 27 && s < valid) {
                const uint64_t m = mine[base + s], t = theirs[base + s];
                const int tap = k / 3, ch = k - tap * 3;
                const uint64_t plane = ch == 0 ? m : ch == 1 ? t : (~(m | t) & c4::kBoard);
                const int off = (tap % 3 - 1) * 7 + (tap / 3 - 1);
                v = off >= 0 ? plane >> off : plane << -off;
            }
            ((uint64_t *)(smem + kPlanes))[s * kPlaneRow + k] = v;
        }
#ifdef SPAI_DIAG_ENTRY
        if (grp == (int)blockIdx.x) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            stamp(P, wave, lane, 19);
        }
#endif
        __syncthreads();
        stamp(P, wave, lane, 0);
        if (grp == (int)blockIdx.x) stamp_real(P, wave, lane, 22);
        torso_and_heads<W, S, FROM_X, KH>(smem, P, x, base, valid, ln, g, aux);
        __syncthreads();
        stamp(P, wave, lane, 15);
        if (tid < valid) {
            const float *L = (const float *)(smem + kL);
            const int slot = base + tid;
            float sum8[8];
#pragma unroll
            for (int o = 0; o < 8; ++o)
                sum8[o] = 0.f;
#pragma unroll
            for (int pp = 0; pp < kWaves * kLinHalves; ++pp)   // fixed order: wave-major, K half
#pragma unroll
                for (int o = 0; o < 8; ++o) sum8[o] += L[pp * 64 + tid * 8 + o];
            float lg[c4::kActions];
            float mx = -INFINITY;
#pragma unroll
            for (int a = 0; a < c4::kActions; ++a) {
                lg[a] = sum8[a] + P.b_pol[a];
                mx = fmaxf(mx, lg[a]);
            }
            const float v = tanhf(sum8[7] + P.b_val[0]);
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
        stamp(P, wave, lane, 16);
        __syncthreads();   // kB / planes / L are rewritten by the next group
    }
}

template <int S, bool FROM_X>
__device__ __forceinline__ void dispatch_wave(uint8_t *smem, const NetParams &P, uint32_t count, int ngroups,
                                              const uint64_t *__restrict__ mine, const uint64_t *__restrict__ theirs,
                                              const float *__restrict__ x, float *__restrict__ priors,
                                              float *__restrict__ value, float *__restrict__ logits, int wave, int tid) {
#ifdef SPAI_W8
    constexpr int K0 = 1, K1 = 2;   // waves 0-3: the first K half of each tap, 4-7: the second
#else
    constexpr int K0 = 0;
#endif
    switch (wave) {
    case 0: run_groups<0, S, FROM_X, K0>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    case 1: run_groups<1, S, FROM_X, K0>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    case 2: run_groups<2, S, FROM_X, K0>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    case 3: run_groups<3, S, FROM_X, K0>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
#ifdef SPAI_W8
    case 4: run_groups<0, S, FROM_X, K1>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    case 5: run_groups<1, S, FROM_X, K1>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    case 6: run_groups<2, S, FROM_X, K1>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
    default: run_groups<3, S, FROM_X, K1>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, tid); break;
#else
    default: break;
#endif
    }
}

// Persistent forward: the grid is at most one workgroup per CU; each workgroup
// loops over groups of S positions (S from the device-side leaf count, see
// group_size / group_size_conc for conc concurrent search chains; FROM_X and the
// diagnostic mode use S = force_s).
template <bool FROM_X>
__global__ __launch_bounds__(kThreads) void k_forward(const uint32_t *__restrict__ count_ptr, uint32_t count_imm,
                                                      int force_s, int conc, const uint64_t *__restrict__ mine,
                                                      const uint64_t *__restrict__ theirs, const float *__restrict__ x,
                                                      NetParams P, float *__restrict__ priors,
                                                      float *__restrict__ value, float *__restrict__ logits) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[kLdsBytes];
    stamp(P, threadIdx.x >> 6, threadIdx.x & 63, 20);
    stamp_real(P, threadIdx.x >> 6, threadIdx.x & 63, 21);
    const int tid = threadIdx.x;
    // launch constants (stem weights, every conv bias): their loads are issued
    // together, beside the leaf count's, and land in LDS before the group loop
    // (staged inside it they were two more dependent round trips per launch)
    const bool setup = kThreads == kStemThreads || tid < kStemThreads;
    const uint4 ws = setup ? P.w_stem[tid] : make_uint4(0u, 0u, 0u, 0u);   // 256 x 16 B
    const int nbias = setup ? (2 * P.blocks + 2) * kHid : 0;
    float bv[kBiasPer];
#pragma unroll
    for (int j = 0; j < kBiasPer; ++j) bv[j] = tid + j * kStemThreads < nbias ? P.b_conv[tid + j * kStemThreads] : 0.f;
    const uint32_t count = count_ptr ? *count_ptr : count_imm;
    const int S = force_s > 0 ? min(force_s, kSRun) : group_size_conc(count, gridDim.x, conc);
    const int ngroups = (int)((count + S - 1) / S);
    if ((int)blockIdx.x >= ngroups) return;
    if (tid < 64) ((uint32_t *)(smem + kZ))[tid] = 0u;   // the zero blocks below X and Y
    else if (tid < 128) ((uint32_t *)(smem + kZ1))[tid - 64] = 0u;
    if (setup) ((uint4 *)(smem + kWStem))[tid] = ws;
#pragma unroll
    for (int j = 0; j < kBiasPer; ++j)
        if (tid + j * kStemThreads < nbias) ((float *)(smem + kBias))[tid + j * kStemThreads] = bv[j];
#ifdef SPAI_DIAG_ENTRY
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    stamp(P, tid >> 6, tid & 63, 17);
#endif
#ifdef SPAI_FWD_PRIO
    __builtin_amdgcn_s_setprio(SPAI_FWD_PRIO);   // experiment: issue priority against co-resident tree kernels
#endif
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    if constexpr (FROM_X) {
        dispatch_wave<kSRun, true>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid);
    } else {
#ifdef SPAI_ONLY_S
        dispatch_wave<SPAI_ONLY_S, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid);
#else
        switch (S) {
        case 1: dispatch_wave<1, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        case 2: dispatch_wave<2, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        case 3: dispatch_wave<3, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        case 4: dispatch_wave<4, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
#ifdef SPAI_W8
        default: dispatch_wave<5, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
#else
        case 5: dispatch_wave<5, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        case 6: dispatch_wave<6, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        case 7: dispatch_wave<7, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
        default: dispatch_wave<8, false>(smem, P, count, ngroups, mine, theirs, x, priors, value, logits, wave, tid); break;
#endif
        }
#endif
    }
    stamp_real(P, wave, tid & 63, 23);
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

int net_create(spai_engine *e, int blocks, int hidden, const float *params, size_t nparams, int dtype,
               spai_net **out) {
    SPAI_CHECK(e->game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "device net: only Connect4 is built");
    SPAI_CHECK(dtype == SPAI_DTYPE_BF16 || dtype == SPAI_DTYPE_F32, SPAI_ERR_INVALID, "unknown dtype %d", dtype);
    SPAI_CHECK(hidden == kHid, SPAI_ERR_UNSUPPORTED, "device net: hidden must be 64 (got %d)", hidden);
    SPAI_CHECK(blocks >= 0 && blocks <= kMaxBlocks, SPAI_ERR_UNSUPPORTED, "device net: 0..%d blocks (got %d)",
               kMaxBlocks, blocks);
    SPAI_CHECK(params && nparams == net_num_params(e->game, blocks, hidden), SPAI_ERR_INVALID,
               "expected %zu params, got %zu", net_num_params(e->game, blocks, hidden), nparams);
    if (dtype == SPAI_DTYPE_F32) {   // the reference's fp32 arithmetic (net_c4_f32.hip)
        spai_net *n = new spai_net();
        n->eng = e;
        n->blocks = blocks;
        n->hidden = hidden;
        n->dtype = SPAI_DTYPE_F32;
        const int rc = net_create_f32(n, params);
        if (rc != SPAI_OK) {
            net_destroy(n);
            return rc;
        }
        *out = n;
        return SPAI_OK;
    }
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
    std::vector<uint16_t> wh((size_t)kKStepsRes * 4 * 64 * 8, 0);
    std::vector<float> bh(kHid, 0.f);
    for (int ks = 0; ks < kKStepsRes; ++ks)
        for (int ct = 0; ct < 4; ++ct)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    int co = ct * 16 + (l & 15), k = ks * 32 + 8 * (l >> 4) + j;
                    int tap = k / kHid, ci = k % kHid;
                    float v = 0.f;
                    if (co < 32) v = pw[((size_t)co * kHid + ci) * 9 + tap];
                    else if (co < kHeadC) v = vw[((size_t)(co - 32) * kHid + ci) * 9 + tap];
                    wh[(((size_t)ks * 4 + ct) * 64 + l) * 8 + j] = f2bf(v);
                }
    for (int o = 0; o < 32; ++o) bh[o] = pb[o];
    for (int o = 0; o < 3; ++o) bh[32 + o] = vb[o];

    spai_net *n = new spai_net();
    n->eng = e;
    if (hipDeviceGetAttribute(&n->n_cu, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || n->n_cu < 1)
        n->n_cu = 256;
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
    if (blocks > 0) up(n->w_res, wr);
    up(n->w_head, wh);
    {
        std::vector<float> bc(bs);
        bc.insert(bc.end(), br.begin(), br.end());
        bc.insert(bc.end(), bh.begin(), bh.end());
        up(n->b_conv, bc);
    }
    // fused linear as MFMA B fragments with the K halves packed: [ks 24][lane 64][8],
    // lane -> o = lane & 7, k = (lane >> 3 & 1) * 768 + ks*32 + 8*(lane >> 4) + j over
    // the head features H[s][cell*36 + c]; the reference flattens c*42 + cell
    // (policy c < 32 -> logits 0..6, value c = 32..34 -> o = 7)
    std::vector<uint16_t> wlin((size_t)kLinBSteps * 64 * 8, 0);
    for (int ks = 0; ks < kLinBSteps; ++ks)
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j) {
                const int o = l & 7;
                const int k = ((l >> 3) & 1) * (kLinK / 2) + ks * 32 + 8 * (l >> 4) + j;
                const int cell = k / kHC, c = k % kHC;
                float v = 0.f;
                if (k < kLinFeat && o < 7 && c < 32) v = pol_w[(size_t)o * kPolIn + c * c4::kCells + cell];
                else if (k < kLinFeat && o == 7 && c >= 32 && c < kHeadC) v = val_w[(c - 32) * c4::kCells + cell];
                wlin[((size_t)ks * 64 + l) * 8 + j] = f2bf(v);
            }
    up(n->w_lin, wlin);
    // geometry table: per S and row group idx, the cell and each tap's neighbour row group
    std::vector<uint32_t> geo((size_t)9 * c4::kCells * 4, 0);
    for (int S = 1; S <= kS; ++S) {
        int idx_of[c4::kCells];
        for (int i = 0; i < c4::kCells; ++i) idx_of[kCellOrder[S][i]] = i;
        for (int i = 0; i < c4::kCells; ++i) {
            const int cell = kCellOrder[S][i], h = cell / c4::kCols, w = cell % c4::kCols;
            uint32_t *e = &geo[((size_t)S * c4::kCells + i) * 4];
            e[0] = (uint32_t)cell;
            for (int tap = 0; tap < 9; ++tap) {
                const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
                const bool ok = hh >= 0 && hh < c4::kRows && ww >= 0 && ww < c4::kCols;
                const uint32_t nb = ok ? (uint32_t)idx_of[hh * c4::kCols + ww] : 255u;
                e[1 + tap / 4] |= nb << (8 * (tap % 4));
            }
        }
    }
    up(n->geo, geo);
    if (rc == SPAI_OK) rc = n->lane_geo.alloc(kLaneGeoU4 * 4);
    if (rc == SPAI_OK) {
        k_geo_init<<<kS * kWaves, 64, 0, e->stream>>>((const uint4 *)n->geo.p, (uint4 *)n->lane_geo.p);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess) {
            set_error("lane geometry kernel failed");
            rc = SPAI_ERR_DEVICE;
        }
    }
    up(n->b_pol, std::vector<float>(pol_b, pol_b + 7));
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
    for (auto *b : {&n->w_stem, &n->w_res, &n->w_head, &n->w_lin}) b->release();
    for (auto *b : {&n->b_conv, &n->b_pol, &n->b_val, &n->f32, &n->io_x,
                    &n->io_logits, &n->io_value, &n->io_priors})
        b->release();
    n->io_mine.release();
    n->io_theirs.release();
    n->io_count.release();
    n->geo.release();
    n->lane_geo.release();
    delete n;
}

static NetParams params_of(const spai_net *n) {
    NetParams P;
    P.w_stem = (const uint4 *)n->w_stem.p;
    P.w_res = (const uint4 *)n->w_res.p;
    P.w_head = (const uint4 *)n->w_head.p;
    P.b_conv = n->b_conv.p;
    P.w_lin = (const uint4 *)n->w_lin.p;
    P.b_pol = n->b_pol.p;
    P.b_val = n->b_val.p;
    P.geo = (const uint4 *)n->geo.p;
    P.lane_geo = (const uint4 *)n->lane_geo.p;
    P.stamps = nullptr;
    P.blocks = n->blocks;
    return P;
}

int ensure_io(spai_net *n, uint32_t cnt) {
    if (n->io_value.n >= cnt) return SPAI_OK;
    SPAI_TRY(n->io_x.alloc((size_t)cnt * 126));
    SPAI_TRY(n->io_logits.alloc((size_t)cnt * 7));
    SPAI_TRY(n->io_value.alloc(cnt));
    SPAI_TRY(n->io_priors.alloc((size_t)cnt * kPriorStride));
    SPAI_TRY(n->io_mine.alloc(cnt));
    SPAI_TRY(n->io_theirs.alloc(cnt));
    return SPAI_OK;
}

// random reachable, ongoing positions (player-to-move view) for the forward benchmarks
static void random_positions(uint32_t cnt, std::vector<uint64_t> &m, std::vector<uint64_t> &t) {
    m.resize(cnt);
    t.resize(cnt);
    uint64_t h = 0x1234;
    for (uint32_t i = 0; i < cnt; ++i) {
        c4::State s{0, 0, 0, c4::kOngoing};
        h = c4::splitmix64(h);
        for (int k = 0, plies = (int)(h % 30); k < plies; ++k) {
            uint32_t lm = c4::legal_mask(s.x, s.o, s.status);
            h = c4::splitmix64(h);
            c4::State r;
            c4::next_state(s, c4::kth_bit(lm, (int)(h % c4::popc32(lm))), r);
            if (r.status != c4::kOngoing) break;
            s = r;
        }
        const bool xm = c4::x_to_move(s.n);
        m[i] = xm ? s.x : s.o;
        t[i] = xm ? s.o : s.x;
    }
}

// Device time of the search's forward launch alone (net_eval_batch with a
// device-side leaf count, as in search) on `cnt` random positions: mean of
// `iters` back-to-back launches between two HIP events on the engine stream.
int net_bench(spai_net *n, uint32_t cnt, uint32_t iters, double *ms, int conc) {
    SPAI_CHECK(cnt > 0 && iters > 0, SPAI_ERR_INVALID, "need cnt > 0 and iters > 0");
    SPAI_TRY(ensure_io(n, cnt));
    if (!n->io_count.p) SPAI_TRY(n->io_count.alloc(1));
    hipStream_t st = n->eng->stream;
    std::vector<uint64_t> m, t;
    random_positions(cnt, m, t);
    SPAI_HIP(hipMemcpyAsync(n->io_mine.p, m.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(n->io_theirs.p, t.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(n->io_count.p, &cnt, 4, hipMemcpyHostToDevice, st));
    for (int w = 0; w < 3; ++w)
        SPAI_TRY(net_eval_batch(n, st, n->io_count.p, cnt, n->io_mine.p, n->io_theirs.p, n->io_priors.p, n->io_value.p,
                                0, conc));
    hipEvent_t a, b;
    SPAI_HIP(hipEventCreate(&a));
    SPAI_HIP(hipEventCreate(&b));
    SPAI_HIP(hipEventRecord(a, st));
    for (uint32_t i = 0; i < iters; ++i)
        SPAI_TRY(net_eval_batch(n, st, n->io_count.p, cnt, n->io_mine.p, n->io_theirs.p, n->io_priors.p, n->io_value.p,
                                0, conc));
    SPAI_HIP(hipEventRecord(b, st));
    SPAI_HIP(hipEventSynchronize(b));
    float f = 0;
    SPAI_HIP(hipEventElapsedTime(&f, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *ms = f / iters;
    return SPAI_OK;
}

int net_phase_stamps(spai_net *n, uint32_t cnt, double *cycles) {
#ifndef SPAI_DIAG
    (void)n;
    (void)cycles;
    SPAI_CHECK(false, SPAI_ERR_UNSUPPORTED, "phase stamps need the diagnostic build (make -C self-play-ai_amd diag)");
#endif
    SPAI_CHECK(cnt > 0, SPAI_ERR_INVALID, "need cnt > 0");
    SPAI_CHECK(n->dtype == SPAI_DTYPE_BF16, SPAI_ERR_UNSUPPORTED, "phase stamps time the bf16 kernel");
    SPAI_TRY(ensure_io(n, cnt));
    hipStream_t st = n->eng->stream;
    std::vector<uint64_t> m, t;
    random_positions(cnt, m, t);
    const char *es = std::getenv("SPAI_PHASE_S");   // diagnostic: group size to time (default 8)
    const int S = es ? std::max(1, std::min(kSRun, std::atoi(es))) : kSRun;
    uint32_t grid = (cnt + S - 1) / S;
    if (const char *eg = std::getenv("SPAI_PHASE_GRID"))   // fewer workgroups: the stamps keep each one's LAST group
        grid = std::min<uint32_t>(grid, (uint32_t)std::max(1, std::atoi(eg)));
    DevBuf<unsigned long long> d;
    SPAI_TRY(d.alloc((size_t)grid * kWaves * kStamps));
    SPAI_HIP(hipMemsetAsync(d.p, 0, d.n * 8, st));
    SPAI_HIP(hipMemcpyAsync(n->io_mine.p, m.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(n->io_theirs.p, t.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    NetParams P = params_of(n);
    P.stamps = d.p;
    for (int rep = 0; rep < 3; ++rep)   // last launch warm
        k_forward<false><<<grid, kThreads, 0, st>>>(nullptr, cnt, S, 1, n->io_mine.p, n->io_theirs.p, nullptr, P,
                                                   n->io_priors.p, n->io_value.p, nullptr);
    SPAI_HIP(hipGetLastError());
    std::vector<unsigned long long> hs(d.n);
    SPAI_HIP(hipMemcpyAsync(hs.data(), d.p, d.n * 8, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    // cycles[k], k < 20: mean over workgroups/waves of stamp[k] - stamp[0] (shader clock).
    // Wall clock (s_memrealtime, 100 MHz): cycles[20] = mean entry -> first group start in
    // shader cycles, [21] the same in ns, [22] mean first group start -> end in ns, [23] the
    // launch span (latest end - earliest entry over all workgroups) in ns.
    for (int k = 0; k < kStamps; ++k) cycles[k] = 0;
    double cntw = 0;
    unsigned long long first_in = ~0ull, last_out = 0;
    for (uint32_t g = 0; g < grid; ++g)
        for (int w = 0; w < kWaves; ++w) {
            const unsigned long long *sp = hs.data() + ((size_t)g * kWaves + w) * kStamps;
            if (!sp[0] || !sp[16]) continue;   // (a workgroup with no group)
            for (int k = 0; k < 20; ++k) cycles[k] += sp[k] ? (double)(long long)(sp[k] - sp[0]) : 0.0;
            for (int k = 24; k < kStamps; ++k) cycles[k] += sp[k] ? (double)(long long)(sp[k] - sp[0]) : 0.0;
            cycles[20] += (double)(sp[0] - sp[20]);   // (the last group's stamp 0: one group per workgroup in the sweeps)
            cycles[21] += 10.0 * (double)(sp[22] - sp[21]);
            cycles[22] += 10.0 * (double)(sp[23] - sp[22]);
            first_in = std::min(first_in, sp[21]);
            last_out = std::max(last_out, sp[23]);
            cntw += 1;
        }
    for (int k = 0; k < kStamps; ++k)
        if (k != 23) cycles[k] /= cntw > 0 ? cntw : 1;
    cycles[23] = last_out > first_in ? 10.0 * (double)(last_out - first_in) : 0.0;
    return SPAI_OK;
}

int net_eval_batch(spai_net *net, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint64_t *mine,
                   const uint64_t *theirs, float *priors, float *value, uint32_t grid_cap_call, int conc) {
    if (!max_n) return SPAI_OK;
    if (net->dtype == SPAI_DTYPE_F32) return net_f32_launch(net, st, d_count, max_n, mine, theirs, nullptr, priors, value, nullptr);
    // SPAI_FWD_GRID caps the persistent grid (tuning knob: fewer workgroups -> larger groups S)
    static const uint32_t grid_cap = [] {
        const char *v = std::getenv("SPAI_FWD_GRID");
        return v ? (uint32_t)std::max(1, std::atoi(v)) : 0u;
    }();
    uint32_t grid = std::min<uint32_t>(max_n, (uint32_t)net->n_cu);
    if (grid_cap) grid = std::min(grid, grid_cap);
    if (grid_cap_call) grid = std::min(grid, grid_cap_call);
    // SPAI_FWD_CONC=0: the latency-optimal group size whatever the chains (A/B knob)
    static const bool conc_policy = [] {
        const char *v = std::getenv("SPAI_FWD_CONC");
        return !v || std::atoi(v) != 0;
    }();
    // SPAI_FWD_S=k: every launch at group size k (A/B knob; the results do not depend on S)
    static const int force_s = [] {
        const char *v = std::getenv("SPAI_FWD_S");
        return v ? std::max(0, std::min(kSRun, std::atoi(v))) : 0;
    }();
    k_forward<false><<<grid, kThreads, 0, st>>>(d_count, max_n, force_s, conc_policy ? conc : 1, mine, theirs, nullptr,
                                                params_of(net), priors, value, nullptr);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}


int net_forward_x(spai_net *n, uint32_t cnt, const float *x, float *logits, float *value) {
    if (!cnt) return SPAI_OK;
    SPAI_TRY(ensure_io(n, cnt));
    hipStream_t st = n->eng->stream;
    SPAI_HIP(hipMemcpyAsync(n->io_x.p, x, (size_t)cnt * 126 * 4, hipMemcpyHostToDevice, st));
    if (n->dtype == SPAI_DTYPE_F32) {
        SPAI_TRY(net_f32_launch(n, st, nullptr, cnt, nullptr, nullptr, n->io_x.p, nullptr, n->io_value.p, n->io_logits.p));
    } else {
        k_forward<true><<<(cnt + kSRun - 1) / kSRun, kThreads, 0, st>>>(nullptr, cnt, kSRun, 1, nullptr, nullptr, n->io_x.p,
                                                                 params_of(n), nullptr, n->io_value.p, n->io_logits.p);
        SPAI_HIP(hipGetLastError());
    }
    SPAI_HIP(hipMemcpyAsync(logits, n->io_logits.p, (size_t)cnt * 28, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipMemcpyAsync(value, n->io_value.p, (size_t)cnt * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

int net_predict(spai_net *n, uint32_t cnt, const spai_c4_state *states, float *priors, float *values) {
    if (!cnt) return SPAI_OK;
    SPAI_TRY(ensure_io(n, cnt));
    std::vector<uint64_t> m(cnt), t(cnt);
    for (uint32_t i = 0; i < cnt; ++i) {
        bool xm = c4::x_to_move(states[i].num_actions_played);
        m[i] = xm ? states[i].x : states[i].o;
        t[i] = xm ? states[i].o : states[i].x;
    }
    hipStream_t st = n->eng->stream;
    SPAI_HIP(hipMemcpyAsync(n->io_mine.p, m.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(n->io_theirs.p, t.data(), (size_t)cnt * 8, hipMemcpyHostToDevice, st));
    if (n->dtype == SPAI_DTYPE_F32) {
        SPAI_TRY(net_f32_launch(n, st, nullptr, cnt, n->io_mine.p, n->io_theirs.p, nullptr, n->io_priors.p,
                                n->io_value.p, nullptr));
    } else {
        k_forward<false><<<std::min<uint32_t>(cnt, (uint32_t)n->n_cu), kThreads, 0, st>>>(
            nullptr, cnt, 0, 1, n->io_mine.p, n->io_theirs.p, nullptr, params_of(n), n->io_priors.p, n->io_value.p,
            nullptr);
        SPAI_HIP(hipGetLastError());
    }
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

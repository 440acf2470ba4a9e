// c4.h — Connect4 rules on 64-bit bitboards, shared by the HIP kernels and the
// host runtime.  Restates game/connect_four.rs (reference root) on a layout
// built for the device: bit (col*7 + row) per stone, row 0 = bottom, bit 6 of
// each column is a permanently clear sentinel so column carries and shifts
// never wrap.
//
//   legal actions   connect_four.rs:213-225  top cell (row 5) empty, ascending
//   drop row        connect_four.rs:128-136  lowest empty cell = (occ + bottom) & column
//   winner          connect_four.rs:140-179  H, V and (+1 row,+1 col) diagonal only:
//                                            shifts {7, 1, 8}; the anti-diagonal
//                                            (shift 6) is NOT checked (quirk Q1)
//   status          connect_four.rs:200-204  Won before Tied (n == 42)
//   value           connect_four.rs:231-240  Won -> -1, Tied -> 0 (player-to-move view)
//   encoding        connect_four.rs:242-259  [mine, theirs, empty][row][col]
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SPAI_HD __host__ __device__ __forceinline__
#else
#define SPAI_HD inline
#endif

namespace spai {
namespace c4 {

constexpr int kRows = 6;
constexpr int kCols = 7;
constexpr int kActions = 7;
constexpr int kCells = 42;
constexpr int kMaxPlies = 42;
constexpr uint64_t kBottom = 0x0040810204081ull;      // bit 7c for c in 0..6
constexpr uint64_t kTop = kBottom << 5;                // bit 7c+5
constexpr uint64_t kColMask = 0x3Full;                 // 6 cells of one column
constexpr uint64_t kBoard = kBottom * kColMask;        // all 42 cells

enum : uint8_t { kOngoing = 0, kTied = 1, kWon = 2 };

SPAI_HD uint32_t popc64(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __popcll(v);
#else
    return (uint32_t)__builtin_popcountll(v);
#endif
}

SPAI_HD uint32_t popc32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __popc(v);
#else
    return (uint32_t)__builtin_popcount(v);
#endif
}

// 7-bit mask of columns whose top cell is empty (status must be checked by caller)
SPAI_HD uint32_t open_columns(uint64_t occ) {
    uint64_t free_top = ~occ & kTop;                   // bit 7c+5 set if column c open
    // gather bits 5,12,19,26,33,40,47 -> 0..6
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < kCols; ++c) m |= (uint32_t)((free_top >> (7 * c + 5)) & 1ull) << c;
    return m;
}

SPAI_HD uint32_t legal_mask(uint64_t x, uint64_t o, uint8_t status) {
    return status == kOngoing ? open_columns(x | o) : 0u;
}

// cell the next stone in `col` lands on (0 if the column is full)
SPAI_HD uint64_t drop_bit(uint64_t occ, int col) {
    return (occ + (1ull << (7 * col))) & (kColMask << (7 * col));
}

// four in a row horizontally (7), vertically (1) or on the (+1,+1) diagonal (8)
SPAI_HD bool has_line(uint64_t b) {
    uint64_t m = b & (b >> 7);
    if (m & (m >> 14)) return true;
    m = b & (b >> 1);
    if (m & (m >> 2)) return true;
    m = b & (b >> 8);
    if (m & (m >> 16)) return true;
    return false;
}

// k-th (0-based) set bit of a 7-bit mask = action of the k-th child (children are
// created in ascending legal-action order, mcts.rs:127)
SPAI_HD int kth_bit(uint32_t mask, int k) {
    for (int i = 0; i < k; ++i) mask &= mask - 1;
#if defined(__HIP_DEVICE_COMPILE__)
    return __ffs(mask) - 1;
#else
    return __builtin_ctz(mask);
#endif
}

struct State {
    uint64_t x, o;
    uint8_t n, status;
};

SPAI_HD bool x_to_move(uint8_t n) { return (n & 1u) == 0; }

// get_next_state.  Returns 0, -2 (column full) or -3 (game over); out untouched on error.
SPAI_HD int next_state(const State &s, int col, State &out) {
    if (s.status != kOngoing) return -3;
    if (col < 0 || col >= kCols) return -1;
    uint64_t bit = drop_bit(s.x | s.o, col);
    if (!bit) return -2;
    State r = s;
    uint64_t mover;
    if (x_to_move(s.n)) { r.x |= bit; mover = r.x; }
    else { r.o |= bit; mover = r.o; }
    r.n = (uint8_t)(s.n + 1);
    r.status = has_line(mover) ? kWon : (r.n == kCells ? kTied : kOngoing);
    out = r;
    return 0;
}

SPAI_HD float terminal_value(uint8_t status) { return status == kWon ? -1.0f : 0.0f; }

// ---------------------------------------------------------------------------
// Deterministic stub evaluators (not in the reference; pins search/self-play
// against oracle/spai_oracle.c or_hash_eval_raw + mask_invalid_actions).
// All f32 arithmetic is on small integers or single correctly-rounded
// divisions, so host and device agree bit for bit (build with -ffp-contract=off).
// ---------------------------------------------------------------------------
SPAI_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// mask_invalid_actions (connect_four.rs:261-279): p*mask / sum(p*mask), the sum
// in ndarray's order (sequential for 7 elements)
SPAI_HD void mask_renorm(const float *p, uint32_t legal, float *out) {
    float m[kActions];
    float s = 0.0f;
#pragma unroll
    for (int a = 0; a < kActions; ++a) {
        m[a] = p[a] * (((legal >> a) & 1u) ? 1.0f : 0.0f);
        s = s + m[a];
    }
#pragma unroll
    for (int a = 0; a < kActions; ++a) out[a] = m[a] / s;
}

SPAI_HD void stub_eval(int kind, uint64_t x, uint64_t o, uint8_t n, float *priors, float *value) {
    float raw[kActions];
    if (kind == 1) {  // SPAI_EVAL_UNIFORM
#pragma unroll
        for (int a = 0; a < kActions; ++a) raw[a] = 1.0f / (float)kActions;
        *value = 0.0f;
    } else {          // SPAI_EVAL_HASH
        uint64_t h = splitmix64(x ^ (o * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)n << 58));
        float w[kActions];
        float s = 0.0f;
#pragma unroll
        for (int a = 0; a < kActions; ++a) {
            w[a] = (float)(1 + ((h >> (5 * a)) & 31));
            s = s + w[a];
        }
#pragma unroll
        for (int a = 0; a < kActions; ++a) raw[a] = w[a] / s;
        *value = (float)((int)((h >> 48) & 255) - 127) / 128.0f;
    }
    mask_renorm(raw, open_columns(x | o), priors);
}

}  // namespace c4
}  // namespace spai

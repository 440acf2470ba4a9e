// philox.h — move sampling for self-play (host, and the device for Connect4).
//
// The reference samples a root child with rand::thread_rng and
// WeightedIndex over visit_count^temperature (learner_concurrent.rs:177,189-193),
// which is unseeded.  Here the uniform comes from Philox4x32-10 keyed by
// (seed, game id, move number), so a game's trajectory does not depend on how
// games are batched or sharded across GPUs; the weights, their running sum and
// the draw follow rand 0.8's WeightedIndex<f32> exactly (f32 arithmetic).
// oracle/spai_oracle.c (or_u01_f32, or_policy_sample) restates the same
// definition for the parity tests.
#pragma once
#include <stdint.h>

#include <cmath>
#include <vector>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SPAI_PHX __host__ __device__ inline
#else
#define SPAI_PHX inline
#endif

namespace spai {

SPAI_PHX void philox4x32(uint32_t c[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

SPAI_PHX double sample_uniform(uint64_t seed, uint64_t game_id, uint64_t move_no) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)move_no, (uint32_t)(move_no >> 32), (uint32_t)game_id, (uint32_t)(game_id >> 32)};
    uint32_t out[4];
    philox4x32(ctr, key, out);
    uint64_t bits = (((uint64_t)out[0] << 21) ^ ((uint64_t)out[1] >> 11)) & ((1ull << 53) - 1);
    return (double)bits * (1.0 / 9007199254740992.0);
}

// rand 0.8's UniformFloat<f32> draw (Uniform::new(0, total).sample): the top 23
// bits of a Philox word as a float in [1, 2), minus 1 -- a uniform in [0, 1)
SPAI_PHX float sample_u01_f32(uint64_t seed, uint64_t game_id, uint64_t move_no) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)move_no, (uint32_t)(move_no >> 32), (uint32_t)game_id, (uint32_t)(game_id >> 32)};
    uint32_t out[4];
    philox4x32(ctr, key, out);
    return __builtin_bit_cast(float, (out[0] >> 9) | 0x3F800000u) - 1.0f;
}

// WeightedIndex::<f32>::new(w) then sample (rand 0.8, learner_concurrent.rs:192-193):
// the running f32 total before each later weight, Uniform::new(0, total) shrinking
// its scale one ulp at a time while scale * (1 - 2^-23) >= total, chosen = u01 *
// scale + 0, and the index = the number of running totals <= chosen (so a zero
// weight is never picked).  -1: no item, an invalid (negative / NaN) weight or an
// infinite total (the reference panics); -2: all weights zero (panics too)
SPAI_PHX int weighted_index_f32(const float *w, int n, float u01) {
    if (n <= 0) return -1;
    float total = 0.0f;
    for (int i = 0; i < n; ++i) {
        if (!(w[i] >= 0.0f)) return -1;
        total = i ? total + w[i] : w[i];
    }
    if (total == 0.0f) return -2;
    if (!(total <= 3.40282347e38f)) return -1;
    const float max_rand = 1.0f - 1.1920929e-7f;
    float scale = total;
    while (scale * max_rand >= total) scale = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, scale) - 1u);
    const float chosen = u01 * scale + 0.0f;
    int idx = 0;
    float run = 0.0f;
    for (int i = 0; i + 1 < n; ++i) {
        run = i ? run + w[i] : w[i];
        if (run <= chosen) idx = i + 1;
    }
    return idx;
}

// the move draw of SelfPlayWorker::self_play over child visit counts: weights
// (visit_count as f32).powf(temperature), host powf (glibc, as Rust's f32::powf)
inline int weighted_index(const float *visits, int n, float temperature, float u01) {
    float w[512];
    if (n <= 0 || n > 512) return -1;
    for (int i = 0; i < n; ++i) w[i] = ::powf(visits[i], temperature);
    return weighted_index_f32(w, n, u01);
}

}  // namespace spai

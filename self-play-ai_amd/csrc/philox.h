// philox.h — move sampling for self-play (host, and the device for Connect4).
//
// The reference samples a root child with rand::thread_rng and
// WeightedIndex over visit_count^temperature (learner_concurrent.rs:177,189-193),
// which is unseeded.  Here the uniform comes from Philox4x32-10 keyed by
// (seed, game id, move number), so a game's trajectory does not depend on how
// games are batched or sharded across GPUs; the weights and their running sum
// are kept in double.  oracle/spai_oracle.c (or_uniform, or_weighted_index)
// restates the same definition for the parity tests.
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

// index of the sampled child, -1 if n is out of range, -2 if all weights are 0
// visits^temperature for the integer visit counts of a self-play run, each
// computed once by the same std::pow (so the weights are the same bits); any
// other value goes to std::pow directly
struct PowCache {
    double temperature = -1.0;
    std::vector<double> tab;
    double operator()(float v, float t) {
        if ((double)t != temperature) {
            temperature = (double)t;
            tab.clear();
        }
        if (!(v >= 0.f) || v >= 1.0e6f || v != (float)(uint32_t)v) return std::pow((double)v, (double)t);
        const uint32_t k = (uint32_t)v;
        while (tab.size() <= k) tab.push_back(std::pow((double)tab.size(), (double)t));
        return tab[k];
    }
};

// the sampled index from the running sums cum[0..n) of the weights (total = cum[n-1])
SPAI_PHX int weighted_index_cum(const double *cum, int n, double total, double u) {
    if (!(total > 0.0)) return -2;
    double x = u * total;
    int last = 0;   // last index whose cumulative weight increased (rand never picks a zero weight)
    for (int i = 0; i < n; ++i) {
        if (cum[i] > x) return i;
        if (i == 0 ? cum[0] > 0.0 : cum[i] > cum[i - 1]) last = i;
    }
    return last;   // u * total rounded up to total
}

template <class Pow>
inline int weighted_index_with(const float *visits, int n, float temperature, double u, Pow &&pw) {
    double cum[512];
    double total = 0.0;
    if (n <= 0 || n > 512) return -1;
    for (int i = 0; i < n; ++i) {
        total += pw(visits[i], temperature);
        cum[i] = total;
    }
    return weighted_index_cum(cum, n, total, u);
}

inline int weighted_index(const float *visits, int n, float temperature, double u) {
    return weighted_index_with(visits, n, temperature, u,
                               [](float v, float t) { return std::pow((double)v, (double)t); });
}

}  // namespace spai

// policy.cpp — the reference's Policy trait methods on flat policy arrays
// (game/mod.rs:35-44; bodies in connect_four.rs:96-125, tictactoe.rs:96-125,
// chess.rs:518-545).  Host code: these run once per move on a 7/9/4672-entry
// array the search already copied back, so there is nothing to offload.
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "spai_internal.h"

namespace {

// ndarray's sum of a contiguous f32 array (numeric_util::unrolled_fold):
// eight running lanes, combined (0+4)+(1+5)+(2+6)+(3+7), then the tail.
float nd_sum(const float *x, uint32_t n) {
    float p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t i = 0;
    for (; n - i >= 8; i += 8)
        for (int k = 0; k < 8; ++k) p[k] = p[k] + x[i + k];
    float acc = 0.0f;
    acc = acc + (p[0] + p[4]);
    acc = acc + (p[1] + p[5]);
    acc = acc + (p[2] + p[6]);
    acc = acc + (p[3] + p[7]);
    for (; i < n; ++i) acc = acc + x[i];
    return acc;
}

// f32::total_cmp key: flip the magnitude bits of negatives, compare as i32
int32_t total_key(float f) {
    int32_t b;
    std::memcpy(&b, &f, 4);
    return b ^ (int32_t)((uint32_t)(b >> 31) >> 1);
}

float next_down(float f) {   // f > 0, finite
    uint32_t b;
    std::memcpy(&b, &f, 4);
    --b;
    std::memcpy(&f, &b, 4);
    return f;
}

}  // namespace

extern "C" {

int spai_policy_normalize(float *p, uint32_t n) {
    SPAI_CHECK(p || !n, SPAI_ERR_INVALID, "p must not be NULL");
    const float s = nd_sum(p, n);
    for (uint32_t i = 0; i < n; ++i) p[i] = p[i] / s;
    return SPAI_OK;
}

int spai_policy_best_action(const float *p, uint32_t n, uint32_t *index) {
    SPAI_CHECK(p && index, SPAI_ERR_INVALID, "p and index must not be NULL");
    SPAI_CHECK(n > 0, SPAI_ERR_INVALID, "empty policy (the reference unwraps None)");
    // Iterator::max_by keeps the later element on ties
    uint32_t best = 0;
    int32_t bk = total_key(p[0]);
    for (uint32_t i = 1; i < n; ++i) {
        const int32_t k = total_key(p[i]);
        if (k >= bk) {
            bk = k;
            best = i;
        }
    }
    *index = best;
    return SPAI_OK;
}

int spai_policy_sample(const float *p, uint32_t n, float temperature, float u01, uint32_t *index) {
    SPAI_CHECK(p && index, SPAI_ERR_INVALID, "p and index must not be NULL");
    SPAI_CHECK(n > 0, SPAI_ERR_INVALID, "WeightedError::NoItem");
    SPAI_CHECK(u01 >= 0.0f && u01 < 1.0f, SPAI_ERR_INVALID, "u01 must lie in [0, 1)");
    // WeightedIndex::new (rand 0.8): running f32 totals before each later weight
    std::vector<float> cum;
    cum.reserve(n - 1);
    float total = 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        const float w = std::pow(p[i], temperature);   // mapv(|x| x.powf(temperature))
        SPAI_CHECK(w >= 0.0f, SPAI_ERR_INVALID, "WeightedError::InvalidWeight at %u", i);
        if (i) cum.push_back(total);
        total = i ? total + w : w;
    }
    SPAI_CHECK(total != 0.0f, SPAI_ERR_INVALID, "WeightedError::AllWeightsZero");
    SPAI_CHECK(std::isfinite(total), SPAI_ERR_INVALID, "Uniform::new: range overflow");
    // UniformFloat::<f32>::new(0, total): shrink scale until the largest draw stays below total
    const float max_rand = 1.0f - 1.1920929e-7f;
    float scale = total;
    while (scale * max_rand >= total) scale = next_down(scale);
    const float chosen = u01 * scale + 0.0f;
    // first cumulative weight greater than the chosen weight
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (cum[mid] <= chosen) lo = mid + 1;
        else hi = mid;
    }
    *index = lo;
    return SPAI_OK;
}

}  // extern "C"

/* A plain C99 client of include/spai.h, linked against libspai.so the way a
 * Rust/Go/JNI binding would be (no C++ or torch types cross the boundary).
 *   abi_client host    host-only entry points (version, Policy helpers, errors)
 *   abi_client gpu N   + one Connect4 search of N sims over 3 trees with the
 *                        hash evaluator; prints visit counts per tree */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "spai.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_ != SPAI_OK) {                                                      \
            fprintf(stderr, "%s -> %d: %s\n", #x, rc_, spai_last_error());         \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char **argv) {
    const float p[4] = {0.1f, 0.5f, 0.5f, 0.2f};
    uint32_t idx = 99;
    printf("version %s\n", spai_version());
    CHECK(spai_policy_best_action(p, 4, &idx));
    printf("best_action %u\n", idx);
    CHECK(spai_policy_sample(p, 4, 1.0f, 0.5f, &idx));
    printf("sample %u\n", idx);
    if (spai_policy_best_action(p, 0, &idx) != SPAI_ERR_INVALID) return 2;
    printf("empty_error %s\n", spai_last_error());
    if (argc < 2 || strcmp(argv[1], "gpu") != 0) return 0;

    const uint32_t sims = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
    spai_config cfg;
    CHECK(spai_config_default(SPAI_GAME_CONNECT4, &cfg));
    cfg.num_searches = sims;
    cfg.max_trees = 3;
    cfg.eval = SPAI_EVAL_HASH;
    spai_engine *e = NULL;
    CHECK(spai_engine_create(SPAI_GAME_CONNECT4, &cfg, 0, &e));
    CHECK(spai_trees_create(e, 3));
    const uint32_t trees[3] = {0, 1, 2};
    float policy[3 * 7], visits[3 * 7];
    uint32_t ids[3 * 7], nch[3];
    CHECK(spai_search(e, 3, trees, sims, policy, ids, visits, nch));
    for (int t = 0; t < 3; ++t) {
        printf("tree %d children %u visits", t, nch[t]);
        for (uint32_t k = 0; k < nch[t]; ++k) printf(" %.0f", visits[t * 7 + k]);
        printf("\n");
    }
    CHECK(spai_engine_destroy(e));
    return 0;
}

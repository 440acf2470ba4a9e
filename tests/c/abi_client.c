/* A plain C99 client of include/spai.h, linked against libspai.so the way a
 * Rust/Go/JNI binding would be (no C++ or torch types cross the boundary).
 *   abi_client host    host-only entry points (version, Policy helpers, errors)
 *   abi_client gpu N   + one Connect4 search of N sims over 3 trees with the
 *                        hash evaluator; prints visit counts per tree
 *   abi_client net PARAMS NPARAMS BLOCKS BOARDS N
 *                      Model::predict (model/mod.rs:36-98) through spai_net_create
 *                      + spai_predict on N positions, fp32 and bf16 nets: PARAMS is
 *                      raw f32 in construction order, BOARDS raw [N][3] u64 (x, o,
 *                      moves played); prints priors and value per position (%a)
 *   abi_client selfplay GAMES SIMS SEED
 *                      SelfPlayWorker::self_play (learner_concurrent.rs:169-242)
 *                      through spai_selfplay_run with a C sink callback, hash
 *                      evaluator; prints every emitted sample exactly
 *   abi_client nan     an engine error through the boundary: a net whose value
 *                      bias is NaN makes spai_search return SPAI_ERR_NAN (the
 *                      reference panics, mcts.rs:106-109), then a clean net on
 *                      fresh trees searches normally */
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

/* the sink receives each finished game's samples (spai_sample_sink): the game id,
 * its moves, and per position the value, the visit policy and the encoding as two
 * bit masks of its 126 planes (each entry is 0 or 1), all printed exactly */
static void sink(void *user, uint32_t game_id, uint32_t n, const float *enc, const float *pol, const float *val,
                 const int32_t *moves) {
    uint32_t *count = (uint32_t *)user;
    *count += 1;
    printf("game %u %u", game_id, n);
    for (uint32_t i = 0; i < n; ++i) printf(" %d", moves[i]);
    printf("\n");
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t lo = 0, hi = 0;
        for (int k = 0; k < 126; ++k)
            if (enc[i * 126 + k] != 0.0f) {
                if (k < 64) lo |= 1ull << k;
                else hi |= 1ull << (k - 64);
            }
        printf("pos %a %016llx %016llx", val[i], (unsigned long long)lo, (unsigned long long)hi);
        for (int a = 0; a < 7; ++a) printf(" %a", pol[i * 7 + a]);
        printf("\n");
    }
}

static int read_file(const char *path, void *buf, size_t bytes) {
    FILE *f = fopen(path, "rb");
    if (!f) return 0;
    const size_t got = fread(buf, 1, bytes, f);
    fclose(f);
    return got == bytes;
}

static int net_mode(char **argv) {
    const size_t np = (size_t)atol(argv[3]);
    const int blocks = atoi(argv[4]);
    const uint32_t n = (uint32_t)atoi(argv[6]);
    size_t want = 0;
    CHECK(spai_net_num_params(SPAI_GAME_CONNECT4, blocks, 64, &want));
    if (want != np) return 3;
    float *params = malloc(np * sizeof(float));
    uint64_t *boards = malloc((size_t)n * 3 * sizeof(uint64_t));
    spai_c4_state *st = calloc(n, sizeof(spai_c4_state));
    float *priors = malloc((size_t)n * 7 * sizeof(float)), *values = malloc(n * sizeof(float));
    if (!params || !boards || !st || !priors || !values) return 4;
    if (!read_file(argv[2], params, np * sizeof(float)) || !read_file(argv[5], boards, (size_t)n * 24)) return 5;
    for (uint32_t i = 0; i < n; ++i) {
        st[i].x = boards[3 * i];
        st[i].o = boards[3 * i + 1];
        st[i].num_actions_played = (uint8_t)boards[3 * i + 2];
        st[i].status = SPAI_ONGOING;
    }
    spai_config cfg;
    CHECK(spai_config_default(SPAI_GAME_CONNECT4, &cfg));
    cfg.max_trees = 1;
    cfg.num_searches = 1;
    spai_engine *e = NULL;
    CHECK(spai_engine_create(SPAI_GAME_CONNECT4, &cfg, 0, &e));
    const int dtypes[2] = {SPAI_DTYPE_F32, SPAI_DTYPE_BF16};
    for (int d = 0; d < 2; ++d) {
        spai_net *net = NULL;
        CHECK(spai_net_create(e, blocks, 64, params, np, dtypes[d], &net));
        CHECK(spai_predict(net, n, st, priors, values));
        for (uint32_t i = 0; i < n; ++i) {
            printf("predict %s %u %a", d == 0 ? "f32" : "bf16", i, values[i]);
            for (int a = 0; a < 7; ++a) printf(" %a", priors[i * 7 + a]);
            printf("\n");
        }
        CHECK(spai_net_destroy(net));
    }
    CHECK(spai_engine_destroy(e));
    free(params), free(boards), free(st), free(priors), free(values);
    return 0;
}

static int selfplay_mode(char **argv) {
    spai_config cfg;
    CHECK(spai_config_default(SPAI_GAME_CONNECT4, &cfg));
    const uint32_t games = (uint32_t)atoi(argv[2]);
    cfg.num_searches = (uint32_t)atoi(argv[3]);
    cfg.seed = (uint64_t)atoll(argv[4]);
    cfg.max_trees = games;
    cfg.eval = SPAI_EVAL_HASH;
    spai_engine *e = NULL;
    CHECK(spai_engine_create(SPAI_GAME_CONNECT4, &cfg, 0, &e));
    uint32_t finished = 0;
    spai_selfplay_stats stats;
    CHECK(spai_selfplay_run(e, games, 0, sink, &finished, &stats));
    printf("stats %u %.0f %.0f %.0f\n", finished, stats.games, stats.sims, stats.positions);
    CHECK(spai_engine_destroy(e));
    return 0;
}

static int nan_mode(void) {
    spai_config cfg;
    CHECK(spai_config_default(SPAI_GAME_CONNECT4, &cfg));
    cfg.num_searches = 8;
    cfg.max_trees = 64;
    cfg.eval = SPAI_EVAL_NET;
    cfg.seed = 1;
    spai_engine *e = NULL;
    CHECK(spai_engine_create(SPAI_GAME_CONNECT4, &cfg, 0, &e));
    size_t np = 0;
    CHECK(spai_net_num_params(SPAI_GAME_CONNECT4, 2, 64, &np));
    float *p = malloc(np * sizeof(float));
    if (!p) return 4;
    CHECK(spai_net_init_params(SPAI_GAME_CONNECT4, 2, 64, 3, p));
    const float clean_bias = p[np - 1];
    p[np - 1] = __builtin_nanf("");   /* value-head linear bias (model/connect_four.rs:69-70) */
    spai_net *net = NULL;
    CHECK(spai_net_create(e, 2, 64, p, np, SPAI_DTYPE_BF16, &net));
    CHECK(spai_engine_set_net(e, net));
    CHECK(spai_trees_create(e, 64));
    uint32_t trees[64], ids[64 * 7], nch[64];
    float policy[64 * 7], visits[64 * 7];
    for (uint32_t t = 0; t < 64; ++t) trees[t] = t;
    const int rc = spai_search(e, 64, trees, 8, policy, ids, visits, nch);
    printf("nan_rc %d %s\n", rc, rc == SPAI_OK ? "" : spai_last_error());
    CHECK(spai_net_destroy(net));
    p[np - 1] = clean_bias;   /* the engine recovers: a clean net on fresh trees */
    CHECK(spai_net_create(e, 2, 64, p, np, SPAI_DTYPE_BF16, &net));
    CHECK(spai_engine_set_net(e, net));
    CHECK(spai_trees_create(e, 64));
    CHECK(spai_search(e, 64, trees, 8, policy, ids, visits, nch));
    float vsum = 0.f;
    for (uint32_t t = 0; t < 64; ++t)
        for (uint32_t k = 0; k < nch[t]; ++k) vsum += visits[t * 7 + k];
    printf("recovered %.0f\n", vsum);
    CHECK(spai_net_destroy(net));
    CHECK(spai_engine_destroy(e));
    free(p);
    return 0;
}

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
    if (argc >= 7 && strcmp(argv[1], "net") == 0) return net_mode(argv);
    if (argc >= 5 && strcmp(argv[1], "selfplay") == 0) return selfplay_mode(argv);
    if (argc >= 2 && strcmp(argv[1], "nan") == 0) return nan_mode();
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

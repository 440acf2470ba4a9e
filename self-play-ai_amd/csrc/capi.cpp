// capi.cpp — extern "C" entry points of include/spai.h.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>

#include "philox.h"
#include "spai_internal.h"

namespace spai {
namespace {
thread_local char g_err[1024] = "";
}

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// net_init_params: tch 0.13 default initialisers (see DESIGN.md "Random init"),
// the same Philox stream as oracle/spai_oracle.c or_net_init_params.
namespace {
float philox_unit(uint64_t seed, uint32_t tensor, uint64_t idx) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), tensor, 0x5EEDu};
    uint32_t out[4];
    philox4x32(ctr, key, out);
    return (float)(out[0] >> 8) * (1.0f / 16777216.0f);
}
}  // namespace
}  // namespace spai

namespace spai {
void net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params) {
    (void)game;
    uint32_t t = 0;
    float *p = params;
    auto uni = [&](size_t n, float lo, float hi) {
        for (size_t i = 0; i < n; ++i) p[i] = lo + (hi - lo) * philox_unit(seed, t, i);
        p += n;
        ++t;
    };
    auto cst = [&](size_t n, float v) {
        for (size_t i = 0; i < n; ++i) p[i] = v;
        p += n;
        ++t;
    };
    auto conv = [&](int ci, int co) {
        const float b = (float)std::sqrt(6.0 / (double)(ci * 9));
        uni((size_t)co * ci * 9, -b, b);
        cst(co, 0.f);
    };
    auto bn = [&](int c) {
        uni(c, 0.f, 1.f);
        cst(c, 0.f);
        cst(c, 0.f);
        cst(c, 1.f);
    };
    auto lin = [&](int in, int out) {
        const float b = (float)std::sqrt(6.0 / (double)in), bb = (float)(1.0 / std::sqrt((double)in));
        uni((size_t)out * in, -b, b);
        uni(out, -bb, bb);
    };
    conv(3, hidden);
    bn(hidden);
    for (int i = 0; i < blocks; ++i) {
        conv(hidden, hidden);
        bn(hidden);
        conv(hidden, hidden);
        bn(hidden);
    }
    conv(hidden, 32);
    bn(32);
    lin(32 * c4::kCells, c4::kActions);
    conv(hidden, 3);
    bn(3);
    lin(3 * c4::kCells, 1);
}
}  // namespace spai

using namespace spai;

#define ENG_CHECK(e)                                                           \
    do {                                                                       \
        if (!(e)) {                                                            \
            set_error("null engine handle");                                   \
            return SPAI_ERR_INVALID;                                           \
        }                                                                      \
        if (hipSetDevice((e)->device) != hipSuccess) {                         \
            set_error("hipSetDevice(%d) failed", (e)->device);                 \
            return SPAI_ERR_DEVICE;                                            \
        }                                                                      \
    } while (0)

#define PTR_CHECK(p)                                                           \
    do {                                                                       \
        if (!(p)) {                                                            \
            set_error("%s must not be NULL", #p);                              \
            return SPAI_ERR_INVALID;                                           \
        }                                                                      \
    } while (0)

extern "C" {

const char *spai_last_error(void) { return g_err; }

const char *spai_version(void) { return "spai 0.2 (gfx950)"; }

int spai_device_count(int *count) {
    PTR_CHECK(count);
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return SPAI_OK;
}

int spai_config_default(int game, spai_config *cfg) {
    PTR_CHECK(cfg);
    SPAI_CHECK(game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "device engine: only Connect4 is built (game %d)", game);
    *cfg = spai_config{};
    cfg->c = 2.0f;              // mcts.rs:49
    cfg->num_searches = 600;    // mcts.rs:50
    cfg->temperature = 1.25f;   // mcts.rs:51
    cfg->max_trees = 100;       // num_batched_self_play_games, learner_concurrent.rs:56
    cfg->max_moves = c4::kMaxPlies;
    cfg->eval = SPAI_EVAL_NET;
    cfg->seed = 0;
    return SPAI_OK;
}

int spai_engine_create(int game, const spai_config *cfg, int device, spai_engine **out) {
    PTR_CHECK(cfg);
    PTR_CHECK(out);
    SPAI_CHECK(game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "device engine: only Connect4 is built (game %d)", game);
    SPAI_CHECK(cfg->eval <= SPAI_EVAL_HASH, SPAI_ERR_INVALID, "bad eval kind %u", cfg->eval);
    SPAI_CHECK(cfg->max_moves <= c4::kMaxPlies, SPAI_ERR_INVALID, "max_moves %u > 42", cfg->max_moves);
    int ndev = 0;
    SPAI_HIP(hipGetDeviceCount(&ndev));
    SPAI_CHECK(device >= 0 && device < ndev, SPAI_ERR_DEVICE, "device %d not present (%d visible)", device, ndev);
    SPAI_HIP(hipSetDevice(device));
    // SPAI_BLOCKING_SYNC=1 (A/B knob): host waits on the device sleep instead of spinning,
    // so a rank's self-play host loop needs less than a core beside its GPU (DESIGN.md §6:
    // the host-core budget of an 8-GPU node).  Takes effect only before the device's
    // first use in the process.
    static const bool blocking_sync = [] {
        const char *v = std::getenv("SPAI_BLOCKING_SYNC");
        return v && std::atoi(v) != 0;
    }();
    if (blocking_sync) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    spai_engine *e = new (std::nothrow) spai_engine();
    SPAI_CHECK(e, SPAI_ERR_INVALID, "out of host memory");
    e->game = game;
    e->device = device;
    e->cfg = *cfg;
    bool ok = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) == hipSuccess && e->err.alloc(1) == SPAI_OK;
    for (int h = 1; h < spai_engine::kChains && ok; ++h)
        ok = hipStreamCreateWithFlags(&e->chain_stream[h], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&e->ev_join[h], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        set_error("engine stream / scratch allocation failed");
        delete e;
        return SPAI_ERR_DEVICE;
    }
    e->chain_stream[0] = e->stream;
    *out = e;
    return SPAI_OK;
}

int spai_engine_destroy(spai_engine *e) {
    if (!e) return SPAI_OK;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    Trees &T = e->trees;
    T.nodes.release();
    T.root.release();
    T.next_free.release();
    T.root_x.release();
    T.root_o.release();
    T.root_n.release();
    T.root_status.release();
    T.path.release();
    T.depth.release();
    T.slot.release();
    T.left.release();
    T.evals.release();
    for (Batch &B : e->batch) {
        B.tree.release();
        B.mine.release();
        B.theirs.release();
        B.priors.release();
        B.value.release();
        B.iter_counts.release();
        B.iter_more.release();
    }
    e->games.x.release();
    e->games.o.release();
    e->games.n.release();
    e->games.status.release();
    e->active.release();
    e->err.release();
    e->stats.release();
    e->pow_tab.release();
    e->move_out.release();
    for (uint32_t *&h : e->h_move)
        if (h) (void)hipHostFree(h);
    for (hipEvent_t ev : e->timer.ev) (void)hipEventDestroy(ev);
    for (int h = 1; h < spai_engine::kChains; ++h) {
        if (e->chain_stream[h]) (void)hipStreamSynchronize(e->chain_stream[h]);
        if (e->chain_stream[h]) (void)hipStreamDestroy(e->chain_stream[h]);
        if (e->ev_join[h]) (void)hipEventDestroy(e->ev_join[h]);
    }
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    (void)hipStreamDestroy(e->stream);
    delete e;
    return SPAI_OK;
}

int spai_engine_sync(spai_engine *e) {
    ENG_CHECK(e);
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int spai_games_resize(spai_engine *e, uint32_t n) { ENG_CHECK(e); return rules_resize(e, n); }
int spai_games_reset(spai_engine *e, uint32_t first, uint32_t n) { ENG_CHECK(e); return rules_reset(e, first, n); }
int spai_games_write(spai_engine *e, uint32_t first, uint32_t n, const spai_c4_state *s) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(s);
    return rules_write(e, first, n, s);
}
int spai_games_read(spai_engine *e, uint32_t first, uint32_t n, spai_c4_state *s) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(s);
    return rules_read(e, first, n, s);
}
int spai_legal_mask(spai_engine *e, uint32_t first, uint32_t n, uint32_t *mask) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(mask);
    return rules_legal(e, first, n, mask);
}
int spai_apply(spai_engine *e, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(actions);
    return rules_apply(e, first, n, actions, rc);
}
int spai_value_terminated(spai_engine *e, uint32_t first, uint32_t n, float *v, uint8_t *t) {
    ENG_CHECK(e);
    if (n) {
        PTR_CHECK(v);
        PTR_CHECK(t);
    }
    return rules_value_term(e, first, n, v, t);
}
int spai_encode(spai_engine *e, uint32_t first, uint32_t n, float *out) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(out);
    return rules_encode(e, first, n, out);
}
int spai_mask_invalid(spai_engine *e, uint32_t first, uint32_t n, const float *p, uint32_t len, float *out) {
    ENG_CHECK(e);
    if (n) {
        PTR_CHECK(p);
        PTR_CHECK(out);
    }
    return rules_mask(e, first, n, p, len, out);
}
int spai_rules_bench(spai_engine *e, uint32_t n, uint32_t iters, double *ms) {
    ENG_CHECK(e);
    PTR_CHECK(ms);
    return rules_bench(e, n, iters, ms);
}

int spai_net_num_params(int game, int blocks, int hidden, size_t *count) {
    PTR_CHECK(count);
    SPAI_CHECK(game == SPAI_GAME_CONNECT4 && blocks >= 0 && hidden > 0, SPAI_ERR_UNSUPPORTED,
               "net shape not supported (game %d, blocks %d, hidden %d)", game, blocks, hidden);
    *count = net_num_params(game, blocks, hidden);
    return SPAI_OK;
}

int spai_net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params) {
    PTR_CHECK(params);
    SPAI_CHECK(game == SPAI_GAME_CONNECT4 && blocks >= 0 && hidden > 0, SPAI_ERR_UNSUPPORTED,
               "net shape not supported");
    net_init_params(game, blocks, hidden, seed, params);
    return SPAI_OK;
}

int spai_net_create(spai_engine *e, int blocks, int hidden, const float *params, size_t nparams, int dtype,
                    spai_net **out) {
    ENG_CHECK(e);
    PTR_CHECK(out);
    return net_create(e, blocks, hidden, params, nparams, dtype, out);
}

int spai_net_destroy(spai_net *n) {
    if (!n) return SPAI_OK;
    if (n->eng) {
        (void)hipSetDevice(n->eng->device);
        (void)hipStreamSynchronize(n->eng->stream);
        if (n->eng->net == n) n->eng->net = nullptr;
    }
    net_destroy(n);
    return SPAI_OK;
}

int spai_net_forward(spai_net *n, uint32_t cnt, const float *x, float *logits, float *value) {
    PTR_CHECK(n);
    ENG_CHECK(n->eng);
    if (cnt) {
        PTR_CHECK(x);
        PTR_CHECK(logits);
        PTR_CHECK(value);
    }
    return net_forward_x(n, cnt, x, logits, value);
}

int spai_predict(spai_net *n, uint32_t cnt, const spai_c4_state *s, float *priors, float *values) {
    PTR_CHECK(n);
    ENG_CHECK(n->eng);
    if (cnt) {
        PTR_CHECK(s);
        PTR_CHECK(priors);
        PTR_CHECK(values);
    }
    return net_predict(n, cnt, s, priors, values);
}

int spai_engine_set_net(spai_engine *e, spai_net *n) {
    ENG_CHECK(e);
    SPAI_CHECK(!n || n->eng == e, SPAI_ERR_INVALID, "net belongs to another engine");
    e->net = n;
    return SPAI_OK;
}

int spai_trees_create(spai_engine *e, uint32_t n) { ENG_CHECK(e); return trees_create(e, n); }
int spai_tree_reset(spai_engine *e, uint32_t t, const spai_c4_state *root) { ENG_CHECK(e); return tree_reset(e, t, root); }
int spai_search(spai_engine *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                uint32_t *child_ids, float *child_visits, uint32_t *n_children) {
    ENG_CHECK(e);
    if (n) PTR_CHECK(tree_idx);
    return search(e, n, tree_idx, num_searches, policy, child_ids, child_visits, n_children, nullptr);
}
int spai_tree_use_subtree(spai_engine *e, uint32_t t, uint32_t child) { ENG_CHECK(e); return tree_use_subtree(e, t, child); }
int spai_tree_node(spai_engine *e, uint32_t t, uint32_t node, spai_c4_state *st, uint32_t *visits, float *w) {
    ENG_CHECK(e);
    return tree_node(e, t, node, st, visits, w);
}
int spai_tree_size(spai_engine *e, uint32_t t, uint32_t *nodes) {
    ENG_CHECK(e);
    PTR_CHECK(nodes);
    return tree_size(e, t, nodes);
}

int spai_selfplay_run(spai_engine *e, uint32_t n_games, uint64_t gid_base, spai_sample_sink sink, void *user,
                      spai_selfplay_stats *stats) {
    ENG_CHECK(e);
    SPAI_CHECK(n_games > 0 && n_games <= e->cfg.max_trees, SPAI_ERR_INVALID, "n_games %u not in [1, max_trees=%u]",
               n_games, e->cfg.max_trees);
    return selfplay_run(e, n_games, gid_base, sink, user, stats);
}

int spai_selfplay_stream(spai_engine *e, uint32_t n_games, uint32_t window, uint64_t gid_base, spai_sample_sink sink,
                         void *user, spai_selfplay_stats *stats) {
    ENG_CHECK(e);
    if (e->game != SPAI_GAME_CONNECT4) {
        set_error("self-play streaming: Connect4 engines");
        return SPAI_ERR_UNSUPPORTED;
    }
    if (window == 0) {
        set_error("window must be > 0");
        return SPAI_ERR_INVALID;
    }
    return selfplay_run(e, n_games, gid_base, sink, user, stats, window);
}

int spai_engine_set_timing(spai_engine *e, int enabled) {
    ENG_CHECK(e);
    KernelTimer &K = e->timer;
    K.enabled = enabled != 0;
    K.stride = enabled > 1 ? (uint32_t)enabled : 4u;
    for (int i = 0; i < 3; ++i) K.total_ms[i] = K.launches[i] = K.items[i] = 0;
    K.used = 0;
    K.which.clear();
    K.iter.clear();
    return SPAI_OK;
}

int spai_engine_timing(spai_engine *e, double *avg_ms, double *launches) {
    ENG_CHECK(e);
    KernelTimer &K = e->timer;
    for (int i = 0; i < 3; ++i) {
        if (avg_ms) avg_ms[i] = K.launches[i] ? K.total_ms[i] / K.launches[i] : 0.0;
        if (launches) launches[i] = K.launches[i];
    }
    return SPAI_OK;
}

int spai_net_phase_cycles(spai_net *n, uint32_t count, double *cycles) {
    PTR_CHECK(n);
    PTR_CHECK(cycles);
    ENG_CHECK(n->eng);
    return net_phase_stamps(n, count, cycles);
}

int spai_net_bench(spai_net *n, uint32_t count, uint32_t iters, double *ms) {
    PTR_CHECK(n);
    PTR_CHECK(ms);
    ENG_CHECK(n->eng);
    return net_bench(n, count, iters, ms);
}

int spai_net_bench_conc(spai_net *n, uint32_t count, uint32_t iters, int conc, double *ms) {
    PTR_CHECK(n);
    PTR_CHECK(ms);
    ENG_CHECK(n->eng);
    if (conc < 1) {
        set_error("conc %d < 1", conc);
        return SPAI_ERR_INVALID;
    }
    return net_bench(n, count, iters, ms, conc);
}

int spai_engine_timing_items(spai_engine *e, double *total_ms, double *items) {
    ENG_CHECK(e);
    for (int i = 0; i < 3; ++i) {
        if (total_ms) total_ms[i] = e->timer.total_ms[i];
        if (items) items[i] = e->timer.items[i];
    }
    return SPAI_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- learner
int spai_adam_config_default(spai_adam_config *cfg) {
    PTR_CHECK(cfg);
    cfg->lr = 1e-3f;   // Adam::default().build(vs, 1e-3) (model/mod.rs:107)
    cfg->beta1 = 0.9f;
    cfg->beta2 = 0.999f;
    cfg->eps = 1e-8f;
    cfg->bn_momentum = 0.1f;   // nn::batch_norm2d(.., Default::default())
    cfg->bn_eps = 1e-5f;
    return SPAI_OK;
}

int spai_learner_create(spai_engine *e, int blocks, int hidden, const float *params, size_t n,
                        const spai_adam_config *cfg, spai_learner **out) {
    ENG_CHECK(e);
    PTR_CHECK(params);
    PTR_CHECK(out);
    return learner_create(e, blocks, hidden, params, n, cfg, out);
}

int spai_learner_destroy(spai_learner *l) {
    if (!l) return SPAI_OK;
    learner_destroy(l);
    return SPAI_OK;
}

int spai_learner_train_batch(spai_learner *l, uint32_t n, const float *states, const float *policies,
                             const float *values, float *loss) {
    PTR_CHECK(l);
    PTR_CHECK(states);
    PTR_CHECK(policies);
    PTR_CHECK(values);
    ENG_CHECK(l->eng);
    return learner_train_batch(l, n, states, policies, values, loss);
}

int spai_learner_train_batches(spai_learner *l, uint32_t k, uint32_t n, const float *states, const float *policies,
                               const float *values, float *losses) {
    PTR_CHECK(l);
    PTR_CHECK(states);
    PTR_CHECK(policies);
    PTR_CHECK(values);
    ENG_CHECK(l->eng);
    return learner_train_batches(l, k, n, states, policies, values, losses);
}

int spai_learner_params(spai_learner *l, float *params, size_t n) {
    PTR_CHECK(l);
    PTR_CHECK(params);
    ENG_CHECK(l->eng);
    return learner_params(l, params, n, false);
}

int spai_learner_grads(spai_learner *l, float *grads, size_t n) {
    PTR_CHECK(l);
    PTR_CHECK(grads);
    ENG_CHECK(l->eng);
    return learner_params(l, grads, n, true);
}

int spai_learner_activation(spai_learner *l, int layer, float *out, size_t n) {
    PTR_CHECK(l);
    PTR_CHECK(out);
    ENG_CHECK(l->eng);
    return learner_activation(l, layer, out, n);
}

int spai_comm_unique_id(uint8_t *id) {
    PTR_CHECK(id);
    return comm_unique_id(id);
}

int spai_learner_set_comm(spai_learner *l, int rank, int world, const uint8_t *id) {
    PTR_CHECK(l);
    ENG_CHECK(l->eng);
    if (world > 1) PTR_CHECK(id);   // world 1: an id makes a 1-rank RCCL communicator, NULL none
    return learner_set_comm(l, rank, world, id);
}

int spai_learner_broadcast(spai_learner *l, int root) {
    PTR_CHECK(l);
    ENG_CHECK(l->eng);
    return learner_broadcast(l, root);
}

int spai_learner_set_host_comm(spai_learner *l, int rank, int world, spai_host_allreduce fn, void *user) {
    PTR_CHECK(l);
    ENG_CHECK(l->eng);
    return learner_set_host_comm(l, rank, world, fn, user);
}

int spai_learner_last_batch(spai_learner *l, uint32_t *n) {
    PTR_CHECK(l);
    PTR_CHECK(n);
    *n = l->last_batch;
    return SPAI_OK;
}

// ---------------------------------------------------------------- checkpoints
int spai_params_save_safetensors(int game, int blocks, int hidden, const float *params, size_t n, const char *path) {
    PTR_CHECK(params);
    PTR_CHECK(path);
    return params_save_safetensors(game, blocks, hidden, params, n, path);
}

int spai_params_load_safetensors(int game, int blocks, int hidden, const char *path, float *params, size_t n) {
    PTR_CHECK(params);
    PTR_CHECK(path);
    return params_load_safetensors(game, blocks, hidden, path, params, n);
}

// ---------------------------------------------------------------- replay + pipeline
int spai_replay_create(uint32_t capacity, spai_replay **out) {
    PTR_CHECK(out);
    return replay_create(capacity, out);
}

int spai_replay_destroy(spai_replay *r) {
    if (r) replay_destroy(r);
    return SPAI_OK;
}

int spai_replay_push(spai_replay *r, uint32_t n, const float *states, const float *policies, const float *values) {
    PTR_CHECK(r);
    if (n) {
        PTR_CHECK(states);
        PTR_CHECK(policies);
        PTR_CHECK(values);
    }
    return replay_push(r, n, states, policies, values);
}

int spai_replay_pop(spai_replay *r, uint32_t n, float *states, float *policies, float *values) {
    PTR_CHECK(r);
    if (n) {
        PTR_CHECK(states);
        PTR_CHECK(policies);
        PTR_CHECK(values);
    }
    return replay_pop_now(r, n, states, policies, values);
}

int spai_replay_size(spai_replay *r, uint32_t *n) {
    PTR_CHECK(r);
    PTR_CHECK(n);
    return replay_size(r, n);
}

int spai_choose_multiple(uint32_t n, uint32_t k, uint64_t seed, uint64_t stream, uint32_t *out) {
    PTR_CHECK(out);
    std::vector<uint32_t> v;
    choose_multiple(n, k, seed, stream, v);
    std::copy(v.begin(), v.end(), out);
    return SPAI_OK;
}

#define PIPE_CFG_CHECK(cfg)                                                                                  \
    SPAI_CHECK((cfg)->struct_size == sizeof(spai_pipeline_config), SPAI_ERR_INVALID,                        \
               "spai_pipeline_config.struct_size is %u, this library expects %zu (set it to "                \
               "sizeof(spai_pipeline_config) of the header the library was built with)",                   \
               (unsigned)(cfg)->struct_size, sizeof(spai_pipeline_config))

int spai_pipeline_config_default(spai_pipeline_config *cfg) {
    PTR_CHECK(cfg);
    PIPE_CFG_CHECK(cfg);
    static const int dev0 = 0;
    *cfg = spai_pipeline_config{};
    cfg->struct_size = sizeof(spai_pipeline_config);
    cfg->n_selfplay = 1;
    cfg->selfplay_devices = &dev0;
    cfg->learner_device = 0;
    cfg->games_per_batch = 100;   // SelfPlayArgs::default (learner_concurrent.rs:50-59)
    cfg->num_searches = 600;
    cfg->c = 2.0f;
    cfg->temperature = 1.25f;
    cfg->batch_size = 128;        // TrainingArgs::default (:61-69)
    cfg->batches_per_iter = 20;
    cfg->train_iters = 10;
    cfg->replay_capacity = 128 * 100;   // main.rs:142
    cfg->sample_fraction = 0.3f;        // learner_concurrent.rs:278
    cfg->blocks = 4;                    // model::connect_four::Args::default
    cfg->seed = 0;
    cfg->checkpoint_dir = nullptr;
    return SPAI_OK;
}

int spai_pipeline_run(const spai_pipeline_config *cfg, const float *init_params, size_t n_params,
                      spai_pipeline_stats *stats) {
    PTR_CHECK(cfg);
    PIPE_CFG_CHECK(cfg);
    PTR_CHECK(init_params);
    return pipeline_run(cfg, init_params, n_params, stats);
}

int spai_learner_train(spai_learner *l, uint32_t n, const float *states, const float *policies, const float *values,
                       uint32_t epochs, uint32_t batch, uint64_t seed, float *loss) {
    PTR_CHECK(l);
    PTR_CHECK(states);
    PTR_CHECK(policies);
    PTR_CHECK(values);
    ENG_CHECK(l->eng);
    return learner_train_epochs(l, n, states, policies, values, epochs, batch, seed, loss);
}

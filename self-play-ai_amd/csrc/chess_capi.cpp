// chess_capi.cpp — extern "C" entry points of the chess section of include/spai.h.
#include <cstring>
#include <new>

#include "chess_engine.h"

using namespace spai;
using namespace spai::chess;

#define CH_CHECK(e)                                                            \
    do {                                                                       \
        if (!(e)) {                                                            \
            set_error("null chess engine handle");                             \
            return SPAI_ERR_INVALID;                                           \
        }                                                                      \
        if (hipSetDevice((e)->device) != hipSuccess) {                         \
            set_error("hipSetDevice(%d) failed", (e)->device);                 \
            return SPAI_ERR_DEVICE;                                            \
        }                                                                      \
    } while (0)

#define CH_PTR(p)                                                              \
    do {                                                                       \
        if (!(p)) {                                                            \
            set_error("%s must not be NULL", #p);                              \
            return SPAI_ERR_INVALID;                                           \
        }                                                                      \
    } while (0)

namespace {
void release_all(spai_chess *e) {
    spai::chess::Slots &S = e->slots;
    S.board.release();
    S.hist.release();
    S.n_hist.release();
    S.moves.release();
    S.u32.release();
    S.i32.release();
    S.f32.release();
    S.f32b.release();
    spai::chess::Trees &T = e->trees;
    T.nodes.release();
    T.first.release();
    T.nhash.release();
    T.root.release();
    T.fill.release();
    T.half.release();
    T.root_board.release();
    T.root_reps.release();
    T.hist.release();
    T.hist_n.release();
    T.path.release();
    T.depth.release();
    T.leaf_moves.release();
    T.leaf_n.release();
    T.leaf_hash.release();
    T.leaf_key.release();
    T.st_nch.release();
    T.st_visits.release();
    T.st_ids.release();
    T.st_moves.release();
    T.adv_pick.release();
    T.adv_out.release();
    T.adv_board.release();
    spai::chess::Batch &B = e->batch;
    B.counts.release();
    B.tree.release();
    B.x.release();
    B.logits.release();
    B.value.release();
    e->active.release();
    e->err.release();
    for (hipEvent_t ev : e->timer.ev) (void)hipEventDestroy(ev);
    e->timer.ev.clear();
}
}  // namespace

extern "C" {

int spai_chess_config_default(spai_config *cfg) {
    CH_PTR(cfg);
    *cfg = spai_config{};
    cfg->c = 2.0f;              // mcts.rs:49
    cfg->num_searches = 400;    // BASELINE config 4 (chess, 400 sims/move)
    cfg->temperature = 1.25f;   // learner_concurrent.rs:53
    cfg->max_trees = 1024;      // BASELINE config 4 (1024 parallel games)
    // longest game: transposition-table entries per game.  The reference's rules end a
    // game by the fifty-move counter (chess.rs:124-144,154-166: a draw at 100 plies with
    // no pawn move, capture or castle-right change).  Pawn moves and captures alone bound
    // a game at 5,949 moves = 11,898 plies; the reference's extra reset on a castle-rights
    // change can happen at most 4 more times (each side loses its kingside and queenside
    // rights separately), each worth at most 100 further plies: 12,298 plies.  12,304
    // entries (96 KB per game) therefore cover the longest legal game; a longer one would
    // be reported as SPAI_ERR_CAPACITY ("game longer than cfg.max_moves").
    cfg->max_moves = 12304;
    cfg->eval = SPAI_EVAL_NET;
    cfg->seed = 0;
    return SPAI_OK;
}

int spai_chess_create(const spai_config *cfg, int device, spai_chess **out) {
    CH_PTR(cfg);
    CH_PTR(out);
    SPAI_CHECK(cfg->eval <= SPAI_EVAL_HASH, SPAI_ERR_INVALID, "bad eval kind %u", cfg->eval);
    SPAI_CHECK(cfg->max_moves >= 1 && cfg->max_trees >= 1 && cfg->num_searches >= 1, SPAI_ERR_INVALID,
               "max_moves, max_trees and num_searches must be >= 1");
    SPAI_CHECK(cfg->max_moves <= 65535, SPAI_ERR_INVALID, "max_moves %u > 65535", cfg->max_moves);
    int ndev = 0;
    SPAI_HIP(hipGetDeviceCount(&ndev));
    SPAI_CHECK(device >= 0 && device < ndev, SPAI_ERR_DEVICE, "device %d not present (%d visible)", device, ndev);
    SPAI_HIP(hipSetDevice(device));
    spai_chess *e = new (std::nothrow) spai_chess();
    SPAI_CHECK(e, SPAI_ERR_INVALID, "out of host memory");
    e->device = device;
    e->cfg = *cfg;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) e->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess || e->err.alloc(1) != SPAI_OK ||
        hipMemsetAsync(e->err.p, 0, 4, e->stream) != hipSuccess) {
        set_error("chess engine stream / scratch allocation failed");
        delete e;
        return SPAI_ERR_DEVICE;
    }
    *out = e;
    return SPAI_OK;
}

int spai_chess_destroy(spai_chess *e) {
    if (!e) return SPAI_OK;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    release_all(e);
    (void)hipStreamDestroy(e->stream);
    delete e;
    return SPAI_OK;
}

int spai_chess_sync(spai_chess *e) {
    CH_CHECK(e);
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int spai_chess_games_resize(spai_chess *e, uint32_t n) {
    CH_CHECK(e);
    return slots_resize(e, n, e->cfg.max_moves);
}

int spai_chess_games_write(spai_chess *e, uint32_t first, uint32_t n, const spai_chess_state *s) {
    CH_CHECK(e);
    if (n) CH_PTR(s);
    return slots_write(e, first, n, s);
}

int spai_chess_games_read(spai_chess *e, uint32_t first, uint32_t n, spai_chess_state *s) {
    CH_CHECK(e);
    if (n) CH_PTR(s);
    return slots_read(e, first, n, s);
}

int spai_chess_legal_moves(spai_chess *e, uint32_t first, uint32_t n, uint16_t *moves, uint32_t *counts) {
    CH_CHECK(e);
    return slots_legal(e, first, n, moves, counts);
}

int spai_chess_apply(spai_chess *e, uint32_t first, uint32_t n, const uint16_t *moves, int32_t *rc) {
    CH_CHECK(e);
    if (n) CH_PTR(moves);
    return slots_apply(e, first, n, moves, rc);
}

int spai_chess_status(spai_chess *e, uint32_t first, uint32_t n, uint8_t *status, uint32_t *reps, float *value,
                      uint8_t *terminated) {
    CH_CHECK(e);
    return slots_status(e, first, n, status, reps, value, terminated);
}

int spai_chess_rules_bench(spai_chess *e, uint32_t first, uint32_t n, uint32_t iters, double *ms) {
    CH_CHECK(e);
    CH_PTR(ms);
    return slots_rules_bench(e, first, n, iters, ms);
}

int spai_chess_perft(spai_chess *e, uint32_t slot, int depth, uint64_t *counts) {
    CH_CHECK(e);
    CH_PTR(counts);
    return perft(e, slot, depth, counts);
}

int spai_chess_encode(spai_chess *e, uint32_t first, uint32_t n, float *out) {
    CH_CHECK(e);
    if (n) CH_PTR(out);
    return slots_encode(e, first, n, out);
}

int spai_chess_mask_invalid(spai_chess *e, uint32_t first, uint32_t n, const float *policy, uint32_t len,
                            float *out) {
    CH_CHECK(e);
    if (n) {
        CH_PTR(policy);
        CH_PTR(out);
    }
    return slots_mask(e, first, n, policy, len, out);
}

int spai_chess_move_index(int side, uint16_t move, int32_t *index) {
    CH_PTR(index);
    SPAI_CHECK(side == 0 || side == 1, SPAI_ERR_INVALID, "side must be 0 or 1");
    SPAI_CHECK(((move >> 12) & 7) <= 4 && (move & 63) != ((move >> 6) & 63), SPAI_ERR_INVALID, "bad move code %u",
               move);
    *index = policy_index(side, move);
    return SPAI_OK;
}

int spai_chess_index_move(int side, int32_t index, uint16_t *move) {
    CH_PTR(move);
    SPAI_CHECK(side == 0 || side == 1, SPAI_ERR_INVALID, "side must be 0 or 1");
    SPAI_CHECK(index >= 0 && index < kPolicy, SPAI_ERR_INVALID, "index %d out of [0, 4672)", index);
    *move = (uint16_t)get_action_host(side, index);
    return SPAI_OK;
}

int spai_chess_net_num_params(int blocks, size_t *count) {
    CH_PTR(count);
    SPAI_CHECK(blocks >= 0, SPAI_ERR_INVALID, "blocks < 0");
    *count = net_num_params(blocks);
    return SPAI_OK;
}

int spai_chess_net_init_params(int blocks, uint64_t seed, float *params) {
    CH_PTR(params);
    SPAI_CHECK(blocks >= 0, SPAI_ERR_INVALID, "blocks < 0");
    net_init_params(blocks, seed, params);
    return SPAI_OK;
}

int spai_chess_net_create(spai_chess *e, int blocks, const float *params, size_t n_params, spai_chess_net **out) {
    CH_CHECK(e);
    CH_PTR(out);
    return net_create(e, blocks, params, n_params, out);
}

int spai_chess_net_destroy(spai_chess_net *net) {
    if (!net) return SPAI_OK;
    (void)hipSetDevice(net->eng->device);
    if (net->eng->net == net) net->eng->net = nullptr;
    net_destroy(net);
    return SPAI_OK;
}

int spai_chess_net_forward(spai_chess_net *net, uint32_t n, const float *x, float *logits, float *value) {
    CH_PTR(net);
    CH_CHECK(net->eng);
    if (n) {
        CH_PTR(x);
        CH_PTR(logits);
        CH_PTR(value);
    }
    return net_forward_host(net, n, x, logits, value);
}

int spai_chess_predict(spai_chess_net *net, uint32_t first, uint32_t n, float *priors, float *values) {
    CH_PTR(net);
    CH_CHECK(net->eng);
    if (n) {
        CH_PTR(priors);
        CH_PTR(values);
    }
    return net_predict(net, first, n, priors, values);
}

int spai_chess_set_net(spai_chess *e, spai_chess_net *net) {
    CH_CHECK(e);
    SPAI_CHECK(!net || net->eng == e, SPAI_ERR_INVALID, "net belongs to another engine");
    e->net = net;
    return SPAI_OK;
}

int spai_chess_trees_create(spai_chess *e, uint32_t n) {
    CH_CHECK(e);
    return trees_create(e, n);
}

int spai_chess_search(spai_chess *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                      uint32_t *child_ids, float *child_visits, uint16_t *child_moves, uint32_t *n_children) {
    CH_CHECK(e);
    CH_PTR(tree_idx);
    return search(e, n, tree_idx, num_searches, policy, child_ids, child_visits, child_moves, n_children, nullptr);
}

int spai_chess_tree_reset(spai_chess *e, uint32_t tree, uint32_t slot) {
    CH_CHECK(e);
    return tree_reset_from_slot(e, tree, slot);
}

int spai_chess_tree_use_subtree(spai_chess *e, uint32_t tree, uint32_t child_index) {
    CH_CHECK(e);
    return tree_use_subtree(e, tree, child_index);
}

int spai_chess_tree_root(spai_chess *e, uint32_t tree, spai_chess_state *root, uint32_t *visits, float *value_sum) {
    CH_CHECK(e);
    return tree_root(e, tree, root, visits, value_sum);
}

int spai_chess_trees_advance(spai_chess *e, uint32_t n, const uint32_t *tree_idx, const uint32_t *child_index,
                             uint8_t *status, uint32_t *reps) {
    CH_CHECK(e);
    CH_PTR(tree_idx);
    CH_PTR(child_index);
    return trees_advance(e, n, tree_idx, child_index, status, reps);
}

int spai_chess_selfplay_run(spai_chess *e, uint32_t n_games, uint64_t game_id_base, spai_chess_sample_sink sink,
                            void *user, spai_selfplay_stats *stats) {
    CH_CHECK(e);
    return selfplay_run(e, n_games, game_id_base, sink, user, stats);
}

int spai_chess_selfplay_stream(spai_chess *e, uint32_t n_games, uint32_t window, uint64_t game_id_base,
                               spai_chess_sample_sink sink, void *user, spai_selfplay_stats *stats) {
    CH_CHECK(e);
    if (window == 0) {
        set_error("window must be > 0");
        return SPAI_ERR_INVALID;
    }
    return selfplay_run(e, n_games, game_id_base, sink, user, stats, window);
}

int spai_chess_set_timing(spai_chess *e, int enabled) {
    CH_CHECK(e);
    KernelTimer &t = e->timer;
    t.enabled = enabled != 0;
    for (int k = 0; k < 3; ++k) t.total_ms[k] = t.launches[k] = t.items[k] = 0;
    t.used = 0;
    t.which.clear();
    return SPAI_OK;
}

int spai_chess_timing(spai_chess *e, double *avg_ms, double *launches, double *items) {
    CH_CHECK(e);
    const KernelTimer &t = e->timer;
    for (int k = 0; k < 3; ++k) {
        if (avg_ms) avg_ms[k] = t.launches[k] > 0 ? t.total_ms[k] / t.launches[k] : 0.0;
        if (launches) launches[k] = t.launches[k];
        if (items) items[k] = t.items[k];
    }
    return SPAI_OK;
}

}  // extern "C"

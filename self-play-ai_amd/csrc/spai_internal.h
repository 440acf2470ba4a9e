// spai_internal.h — engine state shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/spai.h"
#include "c4.h"

namespace spai {

void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define SPAI_HIP(expr)                                                                                  \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) {                                                                         \
            ::spai::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return SPAI_ERR_DEVICE;                                                                     \
        }                                                                                               \
    } while (0)

#define SPAI_CHECK(cond, code, ...)          \
    do {                                     \
        if (!(cond)) {                       \
            ::spai::set_error(__VA_ARGS__);  \
            return (code);                   \
        }                                    \
    } while (0)

#define SPAI_TRY(expr)             \
    do {                           \
        int rc_ = (expr);          \
        if (rc_ != SPAI_OK) return rc_; \
    } while (0)

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    int alloc(size_t count) {
        release();
        if (count == 0) return SPAI_OK;
        SPAI_HIP(hipMalloc((void **)&p, count * sizeof(T)));
        n = count;
        return SPAI_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// Node record, 16 B, one per tree node (mcts.rs:20-30 without the State clone):
//   x = visit_count (u32), y = value_sum (f32 bits), z = prior (f32 bits),
//   w = children: kNoChildren, or first_child (24 bits, per-tree index) | n_children << 24.
// Children of a node are contiguous and in legal-action order, so a child's
// action and state follow from its parent's state (no per-node State copy).
constexpr uint32_t kNoChildren = 0xFFFFFFFFu;
constexpr int kMaxDepth = 48;        // >= 42 plies + root
constexpr int kPriorStride = 8;      // priors [slot][8]

// Game slots for the batched rules API (SoA bitboards in HBM).
struct GameSlots {
    DevBuf<uint64_t> x, o;
    DevBuf<uint8_t> n, status;
    uint32_t count = 0;
};

// Device-resident MCTS trees, one arena of `cap` nodes per tree.
struct Trees {
    uint32_t n_trees = 0;
    uint32_t cap = 0;
    DevBuf<uint4> nodes;            // [n_trees * cap]
    DevBuf<uint32_t> root;          // root node index per tree
    DevBuf<uint32_t> next_free;     // arena fill per tree
    DevBuf<uint64_t> root_x, root_o;
    DevBuf<uint8_t> root_n, root_status;
    DevBuf<uint32_t> path;          // [n_trees * kMaxDepth]
    DevBuf<uint8_t> depth;          // [n_trees]
    DevBuf<uint32_t> slot;          // [n_trees] leaf slot in the current batch (select -> expand)
    DevBuf<uint32_t> left;          // [n_trees] search iterations left (tail run-on mode, search.hip)
    DevBuf<uint32_t> evals;         // [n_trees] live leaves of the current search call (tail-mode policy)
    DevBuf<uint64_t> slot_gid;      // [n_trees] self-play: the game id a tree slot plays (its sampling stream)
    DevBuf<uint32_t> slot_move;     // [n_trees] self-play: that game's move number (k_advance advances it)
    DevBuf<uint32_t> refill;        // [2 n_trees] self-play streaming: slots taking a new game, and the games
    // host mirrors of the root bookkeeping
    std::vector<uint32_t> h_root;
    std::vector<c4::State> h_root_state;
    std::vector<uint32_t> h_root_first;   // first child of the root after the last search
    std::vector<uint8_t> h_root_nch;
};

// A search chain's leaf batches (the evaluator's input/output), double-buffered
// by iteration parity: [2][cap] slots; iter_counts[it] is iteration it's slot counter.
struct Batch {
    uint32_t cap = 0;
    DevBuf<uint32_t> tree;          // slot -> tree
    DevBuf<uint64_t> mine, theirs;  // leaf position, player-to-move view
    DevBuf<float> priors;           // [cap][8] masked softmax
    DevBuf<float> value;            // [cap]
    DevBuf<uint32_t> iter_counts;   // per-iteration leaf counts of the current search
    DevBuf<uint32_t> iter_more;     // tail mode: per pass, set if a tree stopped at the run cap
};

struct KernelTimer {
    bool enabled = false;
    uint32_t stride = 4;            // sample every stride-th search iteration
    double total_ms[3] = {0, 0, 0};
    double launches[3] = {0, 0, 0};
    double items[3] = {0, 0, 0};
    std::vector<hipEvent_t> ev;     // pool, 2 per sampled launch
    size_t used = 0;
    std::vector<int> which;         // kernel index per sampled launch
    std::vector<uint32_t> iter;     // iteration per sampled launch
    std::vector<int> chain;         // search chain (stream) per sampled launch
};

}  // namespace spai

struct spai_net {
    spai_engine *eng = nullptr;
    int blocks = 0, hidden = 0;
    int n_cu = 256;                 // compute units: the persistent forward's grid
    // packed, BN-folded bf16 MFMA fragments + fp32 biases / head linears (see net_c4.hip)
    spai::DevBuf<uint16_t> w_stem, w_res, w_head, w_lin;
    spai::DevBuf<float> b_conv, b_pol, b_val;   // b_conv: stem | residual convs | head conv biases
    int dtype = SPAI_DTYPE_BF16;    // SPAI_DTYPE_F32: unfolded fp32 weights in `f32` (net_c4_f32.hip)
    spai::DevBuf<float> f32;
    spai::DevBuf<float> io_x, io_logits, io_value, io_priors;   // scratch for forward/predict calls
    spai::DevBuf<uint64_t> io_mine, io_theirs;
    spai::DevBuf<uint32_t> io_count;
    spai::DevBuf<uint32_t> geo;     // LDS row -> cell / neighbour table of the cell orders (net_c4.hip)
    spai::DevBuf<uint32_t> lane_geo;   // per-lane conv geometry of every (group size, plan, wave, tile) (net_c4.hip)
};

// Device training step of the C4 net (learner.hip).
struct spai_learner {
    spai_engine *eng = nullptr;
    int blocks = 0, hidden = 0;
    spai_adam_config cfg{};
    uint64_t step = 0;
    uint32_t max_batch = 0;
    uint32_t last_batch = 0;            // B of the latest train step (its activations stay in `a`)
    hipGraphExec_t graph = nullptr;     // SPAI_LEARNER_GRAPH=1: the step captured once per batch size
    uint32_t graph_batch = 0;
    size_t n_params = 0;
    struct Conv {
        int ci, co;
        size_t w, b, g, be, mu, var;   // offsets into the flat parameter array
        size_t wk, wkd;                // offsets of its packed forward / data-gradient matrices in wt
    };
    std::vector<Conv> convs;            // stem, 2*blocks residual, policy head, value head
    size_t pol_w = 0, pol_b = 0, val_w = 0, val_b = 0;
    spai::DevBuf<float> p, g, m, v;     // params, grads, Adam moments (flat)
    spai::DevBuf<float> bsum;           // data parallel: sum over ranks of the batch size
    spai::DevBuf<float> wt;             // packed conv matrices (forward and data gradient), once per step
    spai::DevBuf<uint32_t> pack_desc;   // their table (k_pack_all)
    int n_pack = 0;
    spai::DevBuf<float> batch_in;       // batch [x: B*126 | pi: B*7 | z: B]
    float *stage = nullptr;             // pinned host copy of it, then the loss terms [B*2]
    float *stage_b = nullptr;           // a second staging half (learner_train_batches alternates)
    hipEvent_t stage_ev[2] = {nullptr, nullptr};   // each half's upload done
    float *terms_host = nullptr;        // learner_train_batches: every step's loss terms (pinned)
    size_t terms_host_n = 0;
    std::vector<spai::DevBuf<float>> z, a, mean, invstd;   // per conv layer
    spai::DevBuf<float> d0, d1;         // backward scratch [B][64][42]
    spai::DevBuf<float> bn_part;        // SPAI_LEARNER_BN_FUSE=1: the convs' BN partials [layer][64][B] x 2
                                        // (forward: sum, centred sum of squares; backward: sum dy, sum dy xhat),
                                        // then the bias-gradient partials [64][B] and the hand-off counters
    spai::DevBuf<float> dzb, d2;        // fused BN backward: dz of the trunk convs [2 blocks][B][64][42]; a third
                                        // activation-gradient buffer
    spai::DevBuf<float> dlogits, dpre, loss_terms;
    spai::DevBuf<uint32_t> run_idx;     // BN running-stat offsets (for the cross-rank average)
    spai::DevBuf<float> run_buf;
    // backward: the weight gradients run on kWgStreams side streams (layers dealt
    // round-robin) beside the data-gradient chain (an event per conv layer: its dz
    // is ready), each with its own partials buffer, joined before the reduction.
    // One: two measured 163k against 167k samples/s (profiles/r02/learner/side_streams.txt)
    static constexpr int kWgStreams = 1;
    hipStream_t wg_stream[kWgStreams] = {};
    std::vector<hipEvent_t> ev_dz;
    hipEvent_t ev_wg_done[kWgStreams] = {};
    spai::DevBuf<float> wpart_side[kWgStreams];
    void *comm = nullptr;            // ncclComm_t (learner.hip)
    int rank = 0, world = 1;
    // host collective in place of RCCL (spai_learner_set_host_comm): every
    // all-reduce of the step is staged through `host_buf` (pinned) and summed by
    // the caller's function
    spai_host_allreduce host_ar = nullptr;
    void *host_ar_user = nullptr;
    float *host_buf = nullptr;
    size_t host_buf_n = 0;
};


struct spai_engine {
    int game = SPAI_GAME_CONNECT4;
    int device = 0;
    spai_config cfg{};
    hipStream_t stream = nullptr;
    spai::GameSlots games;
    spai::Trees trees;
    // The search runs its trees as kChains independent chains (select -> evaluate
    // -> expand), each with its own batch on its own stream, so one chain's
    // latency-bound tree kernels overlap the other's forward.  Chain 0 uses
    // `stream`.
    static constexpr int kChains = 4;    // capacity; the search uses chains_for(n) of them
    spai::Batch batch[kChains];
    hipStream_t chain_stream[kChains] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[kChains] = {nullptr, nullptr, nullptr, nullptr};
    double last_evals_per_iter = -1;   // previous search call's mean leaves per iteration (< 0: none yet)
    uint32_t last_tail_passes = 0;     // previous search call's tail-mode passes (0: not in tail mode)
    uint32_t last_max_tree_evals = ~0u;   // previous search call's most live leaves of one tree (~0: none yet)
    spai_net *net = nullptr;
    spai::DevBuf<uint32_t> active;   // active tree list
    spai::DevBuf<uint32_t> err;      // device error flags
    spai::DevBuf<uint32_t> stats;    // root stats [n][8]
    // self-play's move step on the device (search.hip k_advance): visits^T for every
    // visit count a game can reach (the host's std::pow), and the per-move records,
    // read back into one of two pinned buffers (move m's is read while m + 1 runs)
    spai::DevBuf<float> pow_tab;       // (visit count as f32).powf(T), host glibc powf
    float pow_tab_t = -1.0f;
    spai::DevBuf<uint32_t> move_out;
    uint32_t *h_move[2] = {nullptr, nullptr};
    size_t h_move_n = 0;
    spai::KernelTimer timer;
};

namespace spai {
// rules.hip
int rules_resize(spai_engine *e, uint32_t n);
int rules_reset(spai_engine *e, uint32_t first, uint32_t n);
int rules_write(spai_engine *e, uint32_t first, uint32_t n, const spai_c4_state *s);
int rules_read(spai_engine *e, uint32_t first, uint32_t n, spai_c4_state *s);
int rules_legal(spai_engine *e, uint32_t first, uint32_t n, uint32_t *mask);
int rules_apply(spai_engine *e, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc);
int rules_value_term(spai_engine *e, uint32_t first, uint32_t n, float *v, uint8_t *t);
int rules_encode(spai_engine *e, uint32_t first, uint32_t n, float *out);
int rules_mask(spai_engine *e, uint32_t first, uint32_t n, const float *p, uint32_t len, float *out);
int rules_bench(spai_engine *e, uint32_t n, uint32_t iters, double *ms);

// net_c4.hip
int net_create(spai_engine *e, int blocks, int hidden, const float *params, size_t nparams, int dtype,
               spai_net **out);
void net_destroy(spai_net *net);
int net_forward_x(spai_net *net, uint32_t n, const float *x, float *logits, float *value);
int net_predict(spai_net *net, uint32_t n, const spai_c4_state *states, float *priors, float *values);
size_t net_num_params(int game, int blocks, int hidden);
int net_phase_stamps(spai_net *net, uint32_t n, double *cycles);
int net_bench(spai_net *net, uint32_t n, uint32_t iters, double *ms, int conc = 1);
void net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params);
// evaluate `count` (device scalar) leaves of the batch; grid sized for max_n; conc:
// search chains whose forwards share the CUs (the group-size policy, net_c4.hip)
int net_eval_batch(spai_net *net, hipStream_t st, const uint32_t *d_count, uint32_t max_n,
                   const uint64_t *mine, const uint64_t *theirs, float *priors, float *value, uint32_t grid_cap = 0,
                   int conc = 1);

// net_c4_f32.hip
int net_create_f32(spai_net *n, const float *params);
int net_f32_launch(spai_net *n, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint64_t *mine,
                   const uint64_t *theirs, const float *x, float *priors, float *value, float *logits);

// learner.hip
int learner_create(spai_engine *e, int blocks, int hidden, const float *params, size_t n, const spai_adam_config *cfg,
                   spai_learner **out);
void learner_destroy(spai_learner *l);
int learner_train_batch(spai_learner *l, uint32_t n, const float *states, const float *policies, const float *values,
                        float *loss3);
int learner_train_batches(spai_learner *l, uint32_t k, uint32_t n, const float *states, const float *policies,
                          const float *values, float *losses);
int learner_activation(spai_learner *L, int layer, float *out, size_t n);
int learner_params(spai_learner *l, float *params, size_t n, bool grads);
int learner_train_epochs(spai_learner *l, uint32_t n, const float *states, const float *policies, const float *values,
                         uint32_t epochs, uint32_t batch, uint64_t seed, float *loss3);
int learner_set_comm(spai_learner *l, int rank, int world, const uint8_t *id);
int learner_broadcast(spai_learner *l, int root);
int learner_set_host_comm(spai_learner *l, int rank, int world, spai_host_allreduce fn, void *user);
int comm_unique_id(uint8_t *id);

// interop.cpp
int params_save_safetensors(int game, int blocks, int hidden, const float *params, size_t n, const char *path);
int params_load_safetensors(int game, int blocks, int hidden, const char *path, float *params, size_t n);

// pipeline.cpp
int replay_create(uint32_t capacity, spai_replay **out);
void replay_destroy(spai_replay *r);
struct Observer {   // pipeline event hook (spai_pipeline_config::observer) and the event's fixed fields
    spai_pipeline_observer fn;
    void *user;
    spai_pipeline_event ev;
};
int replay_push(spai_replay *r, uint32_t n, const float *s, const float *p, const float *v,
                const Observer *obs = nullptr);
int replay_pop_now(spai_replay *r, uint32_t n, float *s, float *p, float *v);
int replay_size(spai_replay *r, uint32_t *n);
void choose_multiple(uint32_t n, uint32_t k, uint64_t seed, uint64_t stream, std::vector<uint32_t> &out);
int pipeline_run(const spai_pipeline_config *cfg, const float *init_params, size_t n_params, spai_pipeline_stats *st);

// search.hip
int trees_create(spai_engine *e, uint32_t n);
int tree_reset(spai_engine *e, uint32_t t, const spai_c4_state *root);
int search(spai_engine *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
           uint32_t *child_ids, float *child_visits, uint32_t *n_children, double *evals_out);
int tree_use_subtree(spai_engine *e, uint32_t t, uint32_t child);
int tree_node(spai_engine *e, uint32_t t, uint32_t node, spai_c4_state *st, uint32_t *visits, float *w);
int tree_size(spai_engine *e, uint32_t t, uint32_t *nodes);
int selfplay_run(spai_engine *e, uint32_t n_games, uint64_t gid_base, spai_sample_sink sink, void *user,
                 spai_selfplay_stats *stats, uint32_t window = 0);

inline c4::State from_abi(const spai_c4_state &s) { return c4::State{s.x, s.o, s.num_actions_played, s.status}; }
inline spai_c4_state to_abi(const c4::State &s) {
    spai_c4_state r{};
    r.x = s.x;
    r.o = s.o;
    r.num_actions_played = s.n;
    r.status = s.status;
    return r;
}
}  // namespace spai

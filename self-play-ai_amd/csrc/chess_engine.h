// chess_engine.h — state of the chess engine (spai_chess) shared by its HIP
// translation units: rules slots, device MCTS trees, leaf batch, net.
#pragma once
#include <vector>

#include "chess.h"
#include "spai_internal.h"

namespace spai {
namespace chess {

constexpr int kMaxDepth = 160;          // deepest selection path (node ids per tree)
constexpr uint32_t kNone = 0xFFFFFFFFu;

// Node record, 16 B: x = visit_count, y = value_sum (f32 bits), z = prior (f32
// bits), w = move code (16 bits) | n_children << 16 (0 = not expanded; a
// non-terminal leaf always has >= 1 legal move).  Children are contiguous in
// MoveGen order; first[] holds the first child, nhash[] the node's legal-move
// list hash (for the repetition rule of its descendants).
struct Trees {
    uint32_t n = 0, cap = 0, max_hist = 0;
    DevBuf<uint4> nodes;        // [n][2*cap]: two halves, swapped by compaction
    DevBuf<uint32_t> first;     // [n][2*cap]
    DevBuf<uint64_t> nhash;     // [n][2*cap]
    DevBuf<uint32_t> root, fill, half;          // per tree: root id, arena fill, active half (0/1)
    DevBuf<Board> root_board;                   // per tree
    DevBuf<uint32_t> root_reps;                 // get_num_repetitions of the root
    DevBuf<uint64_t> hist;                      // [n][max_hist]: list hashes of the game's earlier positions
    DevBuf<uint32_t> hist_n;                    // [n] entries in hist
    DevBuf<uint32_t> path;                      // [n][kMaxDepth]
    DevBuf<uint32_t> depth;                     // [n]
    DevBuf<uint16_t> leaf_moves;                // [n][kMaxMoves]
    DevBuf<uint32_t> leaf_n;                    // [n]
    DevBuf<uint64_t> leaf_hash, leaf_key;       // [n]
    // root statistics after a search: [n] n_children, [n][kMaxMoves] visits / moves / child ids
    DevBuf<uint32_t> st_nch, st_visits, st_ids;
    DevBuf<uint16_t> st_moves;
    // advance: chosen child index per tree in, status/reps of the new root out
    DevBuf<uint32_t> adv_pick, adv_out;
    DevBuf<Board> adv_board;
    std::vector<uint32_t> h_nch, h_visits, h_ids, h_out;
    std::vector<uint16_t> h_moves;
    std::vector<Board> h_boards;
};

struct Batch {
    uint32_t cap = 0;
    DevBuf<uint32_t> counts;    // [num_searches] per-iteration leaf counters
    DevBuf<uint32_t> tree;      // slot -> tree
    DevBuf<uint16_t> x;         // [cap][64 cells][kInCh] bf16 net input
    DevBuf<float> logits;       // [cap][kPolicy]
    DevBuf<float> value;        // [cap]
};

// rules API game slots
struct Slots {
    uint32_t n = 0, max_hist = 0;
    DevBuf<Board> board;
    DevBuf<uint64_t> hist;      // [n][max_hist]
    DevBuf<uint32_t> n_hist;
    DevBuf<uint16_t> moves;     // [n][kMaxMoves] scratch
    DevBuf<uint32_t> u32;       // [n] scratch
    DevBuf<int32_t> i32;        // [n] scratch
    DevBuf<float> f32;          // [n][kPolicy] scratch
    DevBuf<float> f32b;         // [n][kPolicy] scratch
};

}  // namespace chess
}  // namespace spai

struct spai_chess_net;

struct spai_chess {
    int device = 0;
    spai_config cfg{};
    hipStream_t stream = nullptr;
    int n_cu = 256;
    spai::chess::Slots slots;
    spai::chess::Trees trees;
    spai::chess::Batch batch;
    spai::DevBuf<uint32_t> active;   // active tree list
    spai::DevBuf<uint32_t> err;      // device error flags
    spai_chess_net *net = nullptr;
    spai::KernelTimer timer;
};

struct spai_chess_net {
    spai_chess *eng = nullptr;
    int blocks = 0;
    // packed, BN-folded bf16 MFMA A-fragments and fp32 biases (chess_net.hip)
    spai::DevBuf<uint16_t> w_stem, w_res, w_p1, w_p2;
    spai::DevBuf<float> b_stem, b_res, b_p1, b_p2;
    spai::DevBuf<float> v_w, v_b, l1_w, l1_b, l2_w, l2_b;   // value head, fp32 (VALU)
    spai::DevBuf<uint16_t> io_x;
    spai::DevBuf<float> io_logits, io_value;
    spai::DevBuf<uint32_t> io_count;
    uint32_t io_cap = 0;
};

namespace spai {
namespace chess {
// chess_rules.hip
int slots_resize(spai_chess *e, uint32_t n, uint32_t max_hist);
int slots_write(spai_chess *e, uint32_t first, uint32_t n, const spai_chess_state *s);
int slots_read(spai_chess *e, uint32_t first, uint32_t n, spai_chess_state *s);
int slots_legal(spai_chess *e, uint32_t first, uint32_t n, uint16_t *moves, uint32_t *counts);
int slots_apply(spai_chess *e, uint32_t first, uint32_t n, const uint16_t *moves, int32_t *rc);
int slots_status(spai_chess *e, uint32_t first, uint32_t n, uint8_t *status, uint32_t *reps, float *value,
                 uint8_t *terminated);
int slots_encode(spai_chess *e, uint32_t first, uint32_t n, float *out);
int slots_mask(spai_chess *e, uint32_t first, uint32_t n, const float *policy, uint32_t len, float *out);
int slots_rules_bench(spai_chess *e, uint32_t first, uint32_t n, uint32_t iters, double *ms);
int perft(spai_chess *e, uint32_t slot, int depth, uint64_t *counts);
// device-pointer forms used by net_predict (chess_net.hip)
int slots_encode_device(spai_chess *e, uint32_t first, uint32_t n, float *d_out);   // f32 [n][19][64]
int slots_softmax_mask_device(spai_chess *e, uint32_t first, uint32_t n, const float *d_logits, float *d_out);
Board from_abi(const spai_chess_state &s);
spai_chess_state to_abi(const Board &b, uint32_t reps);
void encode_host(const Board &b, uint32_t reps, float *out);   // [19][8][8]
int get_action_host(int side, int index);

// chess_net.hip
size_t net_num_params(int blocks);
void net_init_params(int blocks, uint64_t seed, float *params);
int net_create(spai_chess *e, int blocks, const float *params, size_t n, spai_chess_net **out);
void net_destroy(spai_chess_net *net);
// evaluate `count` (device scalar) positions of x [max_n][64][kInCh] bf16
int net_eval(spai_chess_net *net, hipStream_t st, const uint32_t *d_count, uint32_t max_n, const uint16_t *x,
             float *logits, float *value);
int net_forward_host(spai_chess_net *net, uint32_t n, const float *x, float *logits, float *value);
int net_predict(spai_chess_net *net, uint32_t first, uint32_t n, float *priors, float *values);

// chess_search.hip
int trees_create(spai_chess *e, uint32_t n);
int search(spai_chess *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
           uint32_t *child_ids, float *child_visits, uint16_t *child_moves, uint32_t *n_children, double *evals);
int tree_use_subtree(spai_chess *e, uint32_t tree, uint32_t child_index);
int tree_reset_from_slot(spai_chess *e, uint32_t tree, uint32_t slot);
int tree_root(spai_chess *e, uint32_t tree, spai_chess_state *root, uint32_t *visits, float *value_sum);
int trees_advance(spai_chess *e, uint32_t n, const uint32_t *tree_idx, const uint32_t *child_index, uint8_t *status,
                  uint32_t *reps);
int selfplay_run(spai_chess *e, uint32_t n_games, uint64_t gid_base, spai_chess_sample_sink sink, void *user,
                 spai_selfplay_stats *stats, uint32_t window = 0);
}  // namespace chess
}  // namespace spai

/*
 * spai_oracle.h — CPU restatement of the reference self-play hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product (libspai.so) never links it.
 *
 * It restates, with the reference's own data layout (array-of-structs node
 * arena, a full State copy per node, sequential per-tree loops):
 *   game/connect_four.rs:128-283   Connect4 rules, encoding, masking
 *   game/tictactoe.rs:127-241      TicTacToe rules, encoding, masking
 *   mcts.rs:91-192,214-331         UCB, select, expand, backprop, use_subtree, search
 *   model/mod.rs:36-98,152-184     predict (encode -> forward -> softmax -> mask), ResNet
 *   model/{connect_four,tictactoe}.rs  heads
 *   learner_concurrent.rs:169-242  SelfPlayWorker::self_play
 * (paths relative to the reference root).
 *
 * Pinning: the reference has no tests, fixtures or golden vectors and cannot be
 * built here (Rust/tch, no cargo).  Rules and search are pinned by hand-derived
 * known-answer tests and by an independent pure-Python transliteration
 * (tests/golden/gen_golden.py); the net forward is pinned to libtorch (the
 * engine tch 0.13 wraps) through torch-CPU goldens.  Rules/search parity is
 * therefore "parity unpinned" against reference outputs; see DESIGN.md.
 */
#ifndef SPAI_ORACLE_H
#define SPAI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_ONGOING = 0, OR_TIED = 1, OR_WON = 2 };          /* game/mod.rs:9-15 */
enum { OR_GAME_TICTACTOE = 0, OR_GAME_CONNECT4 = 1 };
enum { OR_NONE = 0, OR_X = 1, OR_O = 2 };                  /* Piece(Option<Player>) */

/* Connect4 state, connect_four.rs:14-26.  board[row][col], row 0 = bottom. */
typedef struct {
    int8_t board[6][7];
    uint8_t current_player;       /* OR_X / OR_O */
    uint8_t num_actions_played;
    uint8_t status;               /* OR_ONGOING / OR_TIED / OR_WON */
} or_c4_state;

/* TicTacToe state, tictactoe.rs:14-26. */
typedef struct {
    int8_t board[3][3];
    uint8_t current_player;
    uint8_t num_actions_played;
    uint8_t status;
} or_ttt_state;

#define OR_MAX_STATE 64
#define OR_MAX_ACTIONS 9

/* ---- generic game table (the State trait, game/mod.rs:21-33) ---- */
typedef struct or_game {
    int kind;
    size_t state_size;
    int num_actions;              /* flat policy length */
    int enc_c, enc_h, enc_w;      /* get_encoding shape */
    void (*init)(void *s);
    int (*next_state)(const void *s, int action, void *out);   /* 0 ok, <0 Err */
    int (*valid_actions)(const void *s, int *actions);          /* ascending */
    int (*status)(const void *s);
    void (*value_terminated)(const void *s, float *v, int *term);
    void (*encoding)(const void *s, float *out);
    int (*mask_invalid)(const void *s, const float *policy, int len, float *out);
    int (*current_player)(const void *s);
} or_game;

const or_game *or_game_get(int kind);
/* get_encoding of n states into out [n][C*H*W] */
void or_encode_states(int game, int n, const void *const *states, float *out);

/* ndarray 0.15 `sum()` on a contiguous f32 slice (numeric_util::unrolled_fold). */
float or_nd_sum(const float *x, int n);

/* Connect4 rules (direct) */
void or_c4_init(or_c4_state *s);
int or_c4_next_state(const or_c4_state *s, int action, or_c4_state *out);
int or_c4_valid_actions(const or_c4_state *s, int *actions);
void or_c4_encoding(const or_c4_state *s, float *out);          /* [3][6][7] */
int or_c4_mask_invalid(const or_c4_state *s, const float *p, int len, float *out);
/* bitboards in the product's layout: bit (col*7+row) */
void or_c4_bitboards(const or_c4_state *s, uint64_t *x, uint64_t *o);

/* batch replay of action sequences [n][max_plies] (-1 = stop); per ply p in
 * [0, max_plies]: legal mask, status, bitboards, next_state rc */
long or_c4_replay(int n, int max_plies, const int32_t *actions, uint32_t *legal, uint8_t *status, uint64_t *xs,
                  uint64_t *os, int32_t *rc);

void or_ttt_init(or_ttt_state *s);
int or_ttt_next_state(const or_ttt_state *s, int action, or_ttt_state *out);

/* ---- Philox4x32-10 + sampling (deterministic restatement of the unseeded
 *      rand::thread_rng + WeightedIndex, learner_concurrent.rs:189-193) ---- */
void or_philox4x32(uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float or_u01_f32(uint64_t seed, uint64_t game_id, uint64_t move_no);
int or_weighted_index(const float *visits, int n, float temperature, float u01);
/* Policy::get_best_action / Policy::sample on a flat policy (game/mod.rs:42-43) */
int or_policy_best_action(const float *p, int n);
int or_policy_sample(const float *p, int n, float temperature, float u01);

/* ---- deterministic stub evaluators (shared definition with the device) ---- */
enum { OR_EVAL_NET = 0, OR_EVAL_UNIFORM = 1, OR_EVAL_HASH = 2 };
uint64_t or_splitmix64(uint64_t x);
/* raw (pre-mask) policy and value of the hash evaluator for a position */
void or_hash_eval_raw(uint64_t x, uint64_t o, int nmoves, int num_actions, float *policy, float *value);

/* ---- ResNet (model/mod.rs:152-184 + per-game heads) in fp32 ---- */
typedef struct or_net or_net;
size_t or_net_num_params(int game, int blocks, int hidden);
or_net *or_net_create(int game, int blocks, int hidden, const float *params, size_t nparams);
void or_net_destroy(or_net *net);
/* Net::forward(x, train=false): x [n][C][H][W] -> logits [n][A], value [n] */
void or_net_forward(const or_net *net, int n, const float *x, float *logits, float *value);
/* random init following tch 0.13 defaults (see DESIGN.md "Random init") */
void or_net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params);

/* Model::predict over game states (model/mod.rs:36-98): masked priors + values */
void or_predict(const or_net *net, int n, const void *const *states, float *priors, float *values);

/* ---- MCTS (mcts.rs) ---- */
typedef struct or_tree or_tree;
typedef void (*or_eval_fn)(void *user, int n, const void *const *states, float *priors, float *values);

or_tree *or_tree_create(int game);                        /* Tree::default() */
or_tree *or_tree_with_root(int game, const void *state);  /* Tree::with_root_state */
void or_tree_destroy(or_tree *t);
int or_tree_size(const or_tree *t);
void or_tree_use_subtree(or_tree *t, int new_root_id);
const void *or_tree_node_state(const or_tree *t, int id);
int or_tree_node_info(const or_tree *t, int id, int *parent, int *action, float *prior,
                      uint32_t *visits, float *value_sum, int *n_children, int *children);

/* Mcts::search; per tree writes policy[A], child_ids[A], child_visits[A], n_children.
 * Returns the number of leaves evaluated (>= 0) or -1 on a NaN UCB (reference panics). */
int or_search(or_tree **trees, int n, int num_searches, float c, int eval_kind, const or_net *net,
              or_eval_fn eval, void *eval_user, float *policy, int *child_ids, float *child_visits,
              int *n_children);

/* SelfPlayWorker::self_play (learner_concurrent.rs:169-242).
 * Emits every finished game's positions in the reference's order.  Returns the
 * number of samples written (<= cap), or <0 on error.  Arrays:
 *   enc [cap][C*H*W], pol [cap][A], val [cap], game [cap], ply [cap]
 * moves [n_games][max_plies] (-1 terminated), n_moves [n_games].
 * stats[0] = total simulations (trees x iterations), stats[1] = total NN evals. */
long or_self_play(int game, int n_games, int num_searches, float c, float temperature, uint64_t seed,
                  uint64_t game_id_base, int eval_kind, const or_net *net, or_eval_fn eval, void *eval_user,
                  long cap, float *enc, float *pol, float *val, int32_t *game_ids, int32_t *plies,
                  int max_plies, int32_t *moves, int32_t *n_moves, double *stats);

#ifdef __cplusplus
}
#endif
#endif

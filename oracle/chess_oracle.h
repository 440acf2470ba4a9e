/*
 * chess_oracle.h — CPU restatement of the reference's chess path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it, as the checker.  The product
 * (libspai.so) never links it.
 *
 * Restates, following the reference as text (paths relative to its root):
 *   game/chess.rs:26-299      State: transposition table of legal-move Vecs,
 *                             fifty-move counter, status (Won = +1, quirk Q7),
 *                             encoding [19][8][8], mask_invalid_actions
 *   game/chess.rs:311-493     Policy::get_channel / get_action (incl. the
 *                             knight-underpromotion get_action bug, :442)
 *   mcts.rs:91-192,214-331    search over chess trees (full State per node)
 *   learner_concurrent.rs:169-242  self-play
 * and the third-party `chess` crate 3.2.0 (un-vendored; restated from its
 * published source as recalled): Board::make_move, MoveGen::new_legal with its
 * enumeration order (piece type P,N,B,R,Q,K; unpinned sources then pinned
 * ones, ascending squares; en-passant entries after the pawns; destinations
 * ascending; promotions Q,N,R,B), Board::status, Game::make_move.
 *
 * Pinning: move-generation COUNTS are pinned by public perft known answers
 * (tests/test_chess_oracle.py).  The crate's enumeration ORDER (which the
 * reference's repetition rule compares, chess.rs:51-61) has no reference
 * fixture here: parity unpinned for order.
 */
#ifndef SPAI_CHESS_ORACLE_H
#define SPAI_CHESS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_PAWN = 0, ORC_KNIGHT, ORC_BISHOP, ORC_ROOK, ORC_QUEEN, ORC_KING };   /* chess::Piece order */
enum { ORC_WHITE = 0, ORC_BLACK = 1 };
#define ORC_NO_EP 64
#define ORC_MAX_MOVES 256
#define ORC_POLICY 4672               /* 73 * 8 * 8 */
#define ORC_ENC 1216                  /* 19 * 8 * 8 */

/* chess::Board: pieces[6], color_combined[2], side, castle rights per colour
 * (bit0 kingside, bit1 queenside), en_passant = square of the pawn that just
 * double-pushed (ORC_NO_EP if none). */
typedef struct {
    uint64_t pieces[6];
    uint64_t color[2];
    uint8_t side;
    uint8_t castle[2];
    uint8_t ep;
} orc_board;

/* chess.rs State: Game (board + MakeMove count), transposition_table
 * (legal-move Vec of every earlier position, a shared persistent list),
 * fifty_move_rule_halfmove_counter. */
typedef struct orc_hist orc_hist;
typedef struct {
    orc_board b;
    uint32_t made;          /* Action::MakeMove entries in Game::actions */
    uint32_t fifty;
    uint32_t n_tt;
    const orc_hist *tt;     /* newest entry */
} orc_state;

/* move code: src | dst << 6 | promo << 12 (promo = ORC_KNIGHT..ORC_QUEEN, 0 = none) */
static inline int orc_move(int src, int dst, int promo) { return src | (dst << 6) | (promo << 12); }

void orc_board_start(orc_board *b);
int orc_board_from_fen(const char *fen, orc_board *b);      /* 0 ok */
/* MoveGen::new_legal in enumeration order; returns the count */
int orc_legal_moves(const orc_board *b, uint16_t *moves);
int orc_in_check(const orc_board *b);
/* Board::make_move (legality not checked) */
void orc_board_make_move(const orc_board *b, int move, orc_board *out);
uint64_t orc_perft(const orc_board *b, int depth);

/* chess.rs State */
void orc_state_init(orc_state *s);                          /* State::default() */
void orc_state_from_board(orc_state *s, const orc_board *b, uint32_t made, uint32_t fifty);
int orc_next_state(const orc_state *s, int move, orc_state *out);   /* 0, -2 game over, -1 failed */
int orc_status(const orc_state *s);                         /* 0 Ongoing, 1 Tied, 2 Won */
int orc_num_repetitions(const orc_state *s);
void orc_value_terminated(const orc_state *s, float *v, int *term);
void orc_encoding(const orc_state *s, float *out);          /* [19][8][8] */
int orc_mask_invalid(const orc_state *s, const float *policy, int len, float *out);
int orc_get_channel(int side, int move);                    /* Policy::get_channel */
int orc_policy_index(int side, int move);                   /* get_prob / set_prob index */
int orc_get_action(int side, int index);                    /* Policy::get_action (bug kept) */
/* free every transposition-table entry allocated so far (states become invalid) */
void orc_arena_reset(void);

/* deterministic stub evaluator (shared definition with the device):
 * raw[i] = 1 + (splitmix64(key ^ i * K) & 15) as f32 (unnormalized, exact sums),
 * value = ((key >> 48) & 255) - 127) / 128 */
uint64_t orc_position_key(const orc_state *s);
void orc_hash_eval_raw(const orc_state *s, float *raw, float *value);

/* ---- MCTS over chess trees (mcts.rs), full State per node ---- */
typedef struct orc_tree orc_tree;
orc_tree *orc_tree_create(void);
orc_tree *orc_tree_with_root(const orc_state *s);   /* Tree::with_root_state */
void orc_tree_destroy(orc_tree *t);
void orc_tree_use_subtree(orc_tree *t, int new_root_id);
const orc_state *orc_tree_node_state(const orc_tree *t, int id);
int orc_tree_size(const orc_tree *t);
typedef void (*orc_eval_fn)(void *user, int n, const orc_state *const *states, float *priors, float *values);
/* Mcts::search.  eval NULL = hash stub.  Per tree: policy [4672] normalized
 * visits, child_ids / child_visits / child_moves [ORC_MAX_MOVES], n_children.
 * Returns leaves evaluated, or -1 on a NaN UCB. */
int orc_search(orc_tree **trees, int n, int num_searches, float c, orc_eval_fn eval, void *user, float *policy,
               int *child_ids, float *child_visits, int *child_moves, int *n_children);
/* SelfPlayWorker::self_play with the hash stub (eval NULL) or `eval`.
 * Per finished game, in emission order: samples (enc [19*64], pol [4672] or
 * NULL, val, game id, ply).  moves [n_games][max_plies], n_moves [n_games].
 * Returns samples written or < 0. */
long orc_self_play(int n_games, int num_searches, float c, float temperature, uint64_t seed, uint64_t game_id_base,
                   orc_eval_fn eval, void *user, long cap, float *enc, float *pol, float *val, int32_t *game_ids,
                   int32_t *plies, int max_plies, int32_t *moves, int32_t *n_moves, double *stats);

#ifdef __cplusplus
}
#endif
#endif

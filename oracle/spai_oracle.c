/*
 * spai_oracle.c — CPU restatement of the reference hot path.
 * TEST INFRASTRUCTURE ONLY (see spai_oracle.h for scope and pinning status).
 *
 * Written for fidelity, not speed: it keeps the reference's array board,
 * its array-of-structs node arena with a full State clone per node and its
 * sequential loops.  Every function names the reference lines it follows.
 */
#include "spai_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ========================================================================
 * ndarray 0.15 sum (numeric_util::unrolled_fold): eight partial sums over
 * full chunks of 8, combined as (p0+p4),(p1+p5),(p2+p6),(p3+p7) into acc,
 * then the tail added sequentially.  Used by Policy::normalize and
 * mask_invalid_actions (connect_four.rs:97,276; tictactoe.rs:380,516).
 * ====================================================================== */
float or_nd_sum(const float *x, int n) {
    float p[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int i = 0;
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

/* ========================================================================
 * Connect4 — game/connect_four.rs
 * ====================================================================== */
void or_c4_init(or_c4_state *s) {                  /* #[derive(Default)] :20-26 */
    memset(s, 0, sizeof(*s));
    s->current_player = OR_X;
    s->status = OR_ONGOING;
}

static int c4_next_row_idx(const or_c4_state *s, int col) {   /* :128-136 */
    for (int i = 0; i < 6; ++i)
        if (s->board[i][col] == OR_NONE) return i;
    return -1;
}

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

static int c4_get_winner(const or_c4_state *s, int latest_row, int latest_col) {  /* :140-179 */
    const int8_t *row = s->board[latest_row];
    for (int i = 0; i <= 7 - 4; ++i)
        if (row[i] != OR_NONE && row[i] == row[i + 1] && row[i] == row[i + 2] && row[i] == row[i + 3])
            return row[i];
    for (int i = 0; i <= 6 - 4; ++i) {
        int8_t v = s->board[i][latest_col];
        if (v != OR_NONE && v == s->board[i + 1][latest_col] && v == s->board[i + 2][latest_col] &&
            v == s->board[i + 3][latest_col])
            return v;
    }
    /* only the (+1 row, +1 col) diagonal is scanned (quirk Q1) */
    int start_offset = imax(-4, -imin(latest_col, latest_row));
    int end_offset = imin(0, imin(7 - (latest_col + 4), 6 - (latest_row + 4)));
    for (int i = start_offset; i <= end_offset; ++i) {
        int r = latest_row + i, c = latest_col + i;
        int8_t v = s->board[r][c];
        if (v != OR_NONE && v == s->board[r + 1][c + 1] && v == s->board[r + 2][c + 2] &&
            v == s->board[r + 3][c + 3])
            return v;
    }
    return OR_NONE;
}

int or_c4_next_state(const or_c4_state *s, int action, or_c4_state *out) {  /* :190-211 */
    if (s->status != OR_ONGOING) return -2;               /* "Game has already ended" */
    if (action < 0 || action >= 7) return -3;             /* index out of bounds -> panic */
    int r = c4_next_row_idx(s, action);
    if (r < 0) return -1;                                 /* "column already filled" */
    or_c4_state n = *s;
    n.board[r][action] = (int8_t)s->current_player;
    n.current_player = s->current_player == OR_X ? OR_O : OR_X;
    n.num_actions_played = (uint8_t)(s->num_actions_played + 1);
    if (c4_get_winner(&n, r, action) != OR_NONE)
        n.status = OR_WON;
    else if (n.num_actions_played == 6 * 7)
        n.status = OR_TIED;
    *out = n;
    return 0;
}

int or_c4_valid_actions(const or_c4_state *s, int *actions) {  /* :213-225 */
    int n = 0;
    if (s->status != OR_ONGOING) return 0;
    for (int col = 0; col < 7; ++col)
        if (s->board[5][col] == OR_NONE) actions[n++] = col;
    return n;
}

static void c4_value_terminated(const void *sv, float *v, int *term) {  /* :231-240 */
    const or_c4_state *s = (const or_c4_state *)sv;
    switch (s->status) {
    case OR_WON: *v = -1.0f; *term = 1; break;
    case OR_TIED: *v = 0.0f; *term = 1; break;
    default: *v = 0.0f; *term = 0; break;
    }
}

void or_c4_encoding(const or_c4_state *s, float *out) {  /* :242-259 */
    memset(out, 0, sizeof(float) * 3 * 6 * 7);
    for (int row = 0; row < 6; ++row)
        for (int col = 0; col < 7; ++col) {
            int8_t p = s->board[row][col];
            if (p != OR_NONE) {
                if (p == s->current_player) out[0 * 42 + row * 7 + col] = 1.0f;
                else out[1 * 42 + row * 7 + col] = 1.0f;
            } else {
                out[2 * 42 + row * 7 + col] = 1.0f;
            }
        }
}

int or_c4_mask_invalid(const or_c4_state *s, const float *p, int len, float *out) {  /* :261-279 */
    if (len != 7) return -1;
    float mask[7] = {0};
    int acts[7];
    int na = or_c4_valid_actions(s, acts);
    for (int i = 0; i < na; ++i) mask[acts[i]] = 1.0f;
    float m[7];
    for (int i = 0; i < 7; ++i) m[i] = p[i] * mask[i];
    float sum = or_nd_sum(m, 7);
    for (int i = 0; i < 7; ++i) out[i] = m[i] / sum;
    return 0;
}

void or_c4_bitboards(const or_c4_state *s, uint64_t *x, uint64_t *o) {
    uint64_t bx = 0, bo = 0;
    for (int row = 0; row < 6; ++row)
        for (int col = 0; col < 7; ++col) {
            uint64_t bit = 1ull << (col * 7 + row);
            if (s->board[row][col] == OR_X) bx |= bit;
            else if (s->board[row][col] == OR_O) bo |= bit;
        }
    *x = bx;
    *o = bo;
}

/* Batch replay for parity tests: game g plays actions[g][0..] until an action
 * is -1 or illegal.  Per ply p (state BEFORE the p-th action) writes the legal
 * mask, status and bitboards; returns total plies replayed. */
long or_c4_replay(int n, int max_plies, const int32_t *actions, uint32_t *legal, uint8_t *status, uint64_t *xs,
                  uint64_t *os, int32_t *rc) {
    long total = 0;
    for (int g = 0; g < n; ++g) {
        const size_t base = (size_t)g * (max_plies + 1);
        or_c4_state s;
        or_c4_init(&s);
        int p = 0;
        for (;; ++p) {
            const size_t k = base + p;
            int acts[7];
            int na = or_c4_valid_actions(&s, acts);
            uint32_t m = 0;
            for (int i = 0; i < na; ++i) m |= 1u << acts[i];
            legal[k] = m;
            status[k] = s.status;
            or_c4_bitboards(&s, &xs[k], &os[k]);
            rc[k] = 0;
            if (p == max_plies) break;
            int a = actions[(size_t)g * max_plies + p];
            if (a < 0) break;
            or_c4_state nx;
            rc[k] = or_c4_next_state(&s, a, &nx);
            if (rc[k] != 0) break;
            s = nx;
            ++total;
        }
        for (int q = p + 1; q <= max_plies; ++q) {   /* later plies keep the final state */
            const size_t k = base + q, l = base + p;
            legal[k] = legal[l];
            status[k] = status[l];
            xs[k] = xs[l];
            os[k] = os[l];
            rc[k] = 0;
        }
    }
    return total;
}

static void c4_init_v(void *s) { or_c4_init((or_c4_state *)s); }
static int c4_next_v(const void *s, int a, void *o) { return or_c4_next_state((const or_c4_state *)s, a, (or_c4_state *)o); }
static int c4_valid_v(const void *s, int *a) { return or_c4_valid_actions((const or_c4_state *)s, a); }
static int c4_status_v(const void *s) { return ((const or_c4_state *)s)->status; }
static void c4_enc_v(const void *s, float *o) { or_c4_encoding((const or_c4_state *)s, o); }
static int c4_mask_v(const void *s, const float *p, int len, float *o) { return or_c4_mask_invalid((const or_c4_state *)s, p, len, o); }
static int c4_cur_v(const void *s) { return ((const or_c4_state *)s)->current_player; }

/* ========================================================================
 * TicTacToe — game/tictactoe.rs.  Flat action index = row*3 + col
 * (Policy is a row-major 3x3 Array2, :100-102, :395).
 * ====================================================================== */
void or_ttt_init(or_ttt_state *s) {
    memset(s, 0, sizeof(*s));
    s->current_player = OR_X;
}

int or_ttt_next_state(const or_ttt_state *s, int action, or_ttt_state *out) {  /* :127-167 */
    if (s->status != OR_ONGOING) return -2;
    if (action < 0 || action >= 9) return -3;
    int r = action / 3, c = action % 3;
    if (s->board[r][c] != OR_NONE) return -1;
    or_ttt_state n = *s;
    n.board[r][c] = (int8_t)s->current_player;
    n.current_player = s->current_player == OR_X ? OR_O : OR_X;
    n.num_actions_played = (uint8_t)(s->num_actions_played + 1);
    const int8_t *row = n.board[r];
    int is_row_win = row[0] == row[1] && row[1] == row[2];
    int is_col_win = n.board[0][c] == n.board[1][c] && n.board[1][c] == n.board[2][c];
    int is_nw_se = r == c && n.board[0][0] == n.board[1][1] && n.board[1][1] == n.board[2][2];
    int adiff = r > c ? r - c : c - r;
    int is_ne_sw = ((r == 1 && c == 1) || adiff == 2) && n.board[0][2] == n.board[1][1] &&
                   n.board[1][1] == n.board[2][0];
    if (is_row_win || is_col_win || is_nw_se || is_ne_sw)
        n.status = OR_WON;
    else if (n.num_actions_played == 9)
        n.status = OR_TIED;
    *out = n;
    return 0;
}

static int ttt_valid(const or_ttt_state *s, int *actions) {  /* :169-182 */
    int n = 0;
    if (s->status != OR_ONGOING) return 0;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            if (s->board[r][c] == OR_NONE) actions[n++] = r * 3 + c;
    return n;
}

static void ttt_value_terminated(const void *sv, float *v, int *term) {  /* :188-197 */
    const or_ttt_state *s = (const or_ttt_state *)sv;
    switch (s->status) {
    case OR_WON: *v = -1.0f; *term = 1; break;
    case OR_TIED: *v = 0.0f; *term = 1; break;
    default: *v = 0.0f; *term = 0; break;
    }
}

static void ttt_encoding(const or_ttt_state *s, float *out) {  /* :199-216 */
    memset(out, 0, sizeof(float) * 27);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            int8_t p = s->board[r][c];
            if (p != OR_NONE) {
                if (p == s->current_player) out[0 * 9 + r * 3 + c] = 1.0f;
                else out[1 * 9 + r * 3 + c] = 1.0f;
            } else {
                out[2 * 9 + r * 3 + c] = 1.0f;
            }
        }
}

static int ttt_mask(const or_ttt_state *s, const float *p, int len, float *out) {  /* :218-236 */
    if (len != 9) return -1;
    float mask[9] = {0};
    int acts[9];
    int na = ttt_valid(s, acts);
    for (int i = 0; i < na; ++i) mask[acts[i]] = 1.0f;
    float m[9];
    for (int i = 0; i < 9; ++i) m[i] = p[i] * mask[i];
    float sum = or_nd_sum(m, 9);
    for (int i = 0; i < 9; ++i) out[i] = m[i] / sum;
    return 0;
}

static void ttt_init_v(void *s) { or_ttt_init((or_ttt_state *)s); }
static int ttt_next_v(const void *s, int a, void *o) { return or_ttt_next_state((const or_ttt_state *)s, a, (or_ttt_state *)o); }
static int ttt_valid_v(const void *s, int *a) { return ttt_valid((const or_ttt_state *)s, a); }
static int ttt_status_v(const void *s) { return ((const or_ttt_state *)s)->status; }
static void ttt_enc_v(const void *s, float *o) { ttt_encoding((const or_ttt_state *)s, o); }
static int ttt_mask_v(const void *s, const float *p, int len, float *o) { return ttt_mask((const or_ttt_state *)s, p, len, o); }
static int ttt_cur_v(const void *s) { return ((const or_ttt_state *)s)->current_player; }

static const or_game G_C4 = {OR_GAME_CONNECT4, sizeof(or_c4_state), 7, 3, 6, 7,
                             c4_init_v, c4_next_v, c4_valid_v, c4_status_v, c4_value_terminated,
                             c4_enc_v, c4_mask_v, c4_cur_v};
static const or_game G_TTT = {OR_GAME_TICTACTOE, sizeof(or_ttt_state), 9, 3, 3, 3,
                              ttt_init_v, ttt_next_v, ttt_valid_v, ttt_status_v, ttt_value_terminated,
                              ttt_enc_v, ttt_mask_v, ttt_cur_v};

const or_game *or_game_get(int kind) {
    if (kind == OR_GAME_CONNECT4) return &G_C4;
    if (kind == OR_GAME_TICTACTOE) return &G_TTT;
    return NULL;
}

void or_encode_states(int game, int n, const void *const *states, float *out) {
    const or_game *g = or_game_get(game);
    const int E = g->enc_c * g->enc_h * g->enc_w;
    for (int i = 0; i < n; ++i) g->encoding(states[i], out + (size_t)i * E);
}

/* ========================================================================
 * Philox4x32-10 and the self-play sampler.  The reference samples with the
 * unseeded thread_rng (learner_concurrent.rs:177,189-193); the restatement
 * keys a counter-based stream by (seed, game id, move number) so trajectories
 * are reproducible and independent of how games are sharded.
 * ====================================================================== */
void or_philox4x32(uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* rand 0.8's UniformFloat<f32> draw from the counter-based stream: the top 23
 * bits of the first Philox word as a float in [1, 2), minus 1 */
float or_u01_f32(uint64_t seed, uint64_t game_id, uint64_t move_no) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)move_no, (uint32_t)(move_no >> 32), (uint32_t)game_id, (uint32_t)(game_id >> 32)};
    uint32_t out[4];
    or_philox4x32(ctr, key, out);
    uint32_t b = (out[0] >> 9) | 0x3F800000u;
    float f;
    memcpy(&f, &b, 4);
    return f - 1.0f;
}

/* the self-play move draw (learner_concurrent.rs:189-193): WeightedIndex<f32> over
 * (visit_count as f32).powf(temperature), i.e. Policy::sample's arithmetic on the
 * child visit counts (or_policy_sample below); -1 when the reference panics */
int or_weighted_index(const float *visits, int n, float temperature, float u01) {
    return or_policy_sample(visits, n, temperature, u01);
}

/* Policy::get_best_action (connect_four.rs:116-124): Iterator::max_by with
 * f32::total_cmp returns the last of equal maxima.  total_cmp (Rust core,
 * f32.rs): left ^= ((left >> 31) as u32 >> 1) as i32 on the bit patterns, then
 * signed comparison. */
static int total_cmp_f32(float a, float b) {
    int32_t l, r;
    memcpy(&l, &a, 4);
    memcpy(&r, &b, 4);
    l ^= (int32_t)(((uint32_t)(l >> 31)) >> 1);
    r ^= (int32_t)(((uint32_t)(r >> 31)) >> 1);
    return (l > r) - (l < r);
}

int or_policy_best_action(const float *p, int n) {
    int best = -1;
    for (int i = 0; i < n; ++i)
        if (best < 0 || total_cmp_f32(p[best], p[i]) <= 0) best = i;   /* max_by: ties -> later */
    return best;
}

/* Policy::sample (connect_four.rs:104-114): rand 0.8.5 WeightedIndex<f32> over
 * mapv(powf(temperature)).  new(): total = w0; for each later w, push total,
 * total += w (f32).  UniformFloat<f32>::new(0, total) shrinks scale one ulp at a
 * time while scale * (1 - 2^-23) >= total; sample = u01 * scale + 0; the index
 * is the number of pushed totals <= that sample.  Returns -1 (NoItem /
 * InvalidWeight / AllWeightsZero / overflow, all panics in the reference). */
int or_policy_sample(const float *p, int n, float temperature, float u01) {
    if (n <= 0) return -1;
    float total = 0.0f;
    for (int i = 0; i < n; ++i) {
        float w = powf(p[i], temperature);
        if (!(w >= 0.0f)) return -1;
        total = i == 0 ? w : total + w;
    }
    if (total == 0.0f || isinf(total)) return -1;
    float scale = total;
    for (;;) {
        float top = scale * (1.0f - 1.1920929e-7f);
        if (!(top >= total)) break;
        uint32_t b;
        memcpy(&b, &scale, 4);
        b -= 1;
        memcpy(&scale, &b, 4);
    }
    float chosen = u01 * scale + 0.0f;
    int idx = 0;
    float run = 0.0f;
    for (int i = 0; i + 1 < n; ++i) {
        float w = powf(p[i], temperature);
        run = i == 0 ? w : run + w;
        if (run <= chosen) idx = i + 1;
    }
    return idx;
}

/* ========================================================================
 * Deterministic stub evaluators.  Not part of the reference: they replace the
 * net in search/self-play parity tests so visit counts are an exact function
 * of the inputs.  The device engine implements the same
 * definitions bit for bit (integer hashing, exact small-integer f32 sums).
 * ====================================================================== */
uint64_t or_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void or_hash_eval_raw(uint64_t x, uint64_t o, int nmoves, int num_actions, float *policy, float *value) {
    uint64_t h = or_splitmix64(x ^ (o * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)nmoves << 58));
    float w[OR_MAX_ACTIONS];
    float s = 0.0f;
    for (int a = 0; a < num_actions; ++a) {
        w[a] = (float)(1 + ((h >> (5 * a)) & 31));
        s = s + w[a];
    }
    for (int a = 0; a < num_actions; ++a) policy[a] = w[a] / s;
    *value = (float)((int)((h >> 48) & 255) - 127) / 128.0f;
}

static void state_bitboards(int game, const void *st, uint64_t *x, uint64_t *o, int *n) {
    if (game == OR_GAME_CONNECT4) {
        const or_c4_state *s = (const or_c4_state *)st;
        or_c4_bitboards(s, x, o);
        *n = s->num_actions_played;
    } else {
        const or_ttt_state *s = (const or_ttt_state *)st;
        uint64_t bx = 0, bo = 0;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                if (s->board[r][c] == OR_X) bx |= 1ull << (r * 3 + c);
                else if (s->board[r][c] == OR_O) bo |= 1ull << (r * 3 + c);
            }
        *x = bx;
        *o = bo;
        *n = s->num_actions_played;
    }
}

static void stub_eval(int game, int kind, int n, const void *const *states, float *priors, float *values) {
    const or_game *g = or_game_get(game);
    int A = g->num_actions;
    float raw[OR_MAX_ACTIONS];
    for (int i = 0; i < n; ++i) {
        if (kind == OR_EVAL_UNIFORM) {
            for (int a = 0; a < A; ++a) raw[a] = 1.0f / (float)A;
            values[i] = 0.0f;
        } else {
            uint64_t x, o;
            int nm;
            state_bitboards(game, states[i], &x, &o, &nm);
            or_hash_eval_raw(x, o, nm, A, raw, &values[i]);
        }
        g->mask_invalid(states[i], raw, A, priors + (size_t)i * A);
    }
}

/* ========================================================================
 * ResNet restatement in fp32 (model/mod.rs:152-184, model/connect_four.rs:
 * 50-81, model/tictactoe.rs:50-81).  Parameter order = module construction
 * order: torso (stem conv, stem BN, blocks), policy head, value head; each
 * conv = weight[co][ci][3][3], bias[co]; each BN = weight, bias,
 * running_mean, running_var; each linear = weight[out][in], bias[out].
 * ====================================================================== */
struct or_net {
    int game, blocks, hidden, C, H, W, A;
    float *params;
    size_t nparams;
};

#define PCONV(ci, co) ((size_t)(co) * (ci) * 9 + (co))
#define PBN(c) ((size_t)4 * (c))

static void game_dims(int game, int *C, int *H, int *W, int *A) {
    const or_game *g = or_game_get(game);
    *C = g->enc_c; *H = g->enc_h; *W = g->enc_w; *A = g->num_actions;
}

size_t or_net_num_params(int game, int blocks, int hidden) {
    int C, H, W, A;
    game_dims(game, &C, &H, &W, &A);
    size_t n = PCONV(C, hidden) + PBN(hidden);
    n += (size_t)blocks * 2 * (PCONV(hidden, hidden) + PBN(hidden));
    n += PCONV(hidden, 32) + PBN(32) + (size_t)A * 32 * H * W + A;
    n += PCONV(hidden, 3) + PBN(3) + (size_t)3 * H * W + 1;
    return n;
}

or_net *or_net_create(int game, int blocks, int hidden, const float *params, size_t nparams) {
    if (!or_game_get(game)) return NULL;
    if (nparams != or_net_num_params(game, blocks, hidden)) return NULL;
    or_net *n = (or_net *)calloc(1, sizeof(or_net));
    n->game = game; n->blocks = blocks; n->hidden = hidden;
    game_dims(game, &n->C, &n->H, &n->W, &n->A);
    n->nparams = nparams;
    n->params = (float *)malloc(nparams * sizeof(float));
    memcpy(n->params, params, nparams * sizeof(float));
    return n;
}

void or_net_destroy(or_net *net) {
    if (!net) return;
    free(net->params);
    free(net);
}

/* conv3x3, padding 1, bias: in [ci][H][W] -> out [co][H][W] */
static void conv3x3(const float *in, int ci, int H, int W, const float *w, const float *b, int co, float *out) {
    for (int o = 0; o < co; ++o) {
        float *op = out + (size_t)o * H * W;
        for (int p = 0; p < H * W; ++p) op[p] = b[o];
        for (int i = 0; i < ci; ++i) {
            const float *ip = in + (size_t)i * H * W;
            const float *wp = w + ((size_t)o * ci + i) * 9;
            for (int kh = 0; kh < 3; ++kh)
                for (int kw = 0; kw < 3; ++kw) {
                    float wv = wp[kh * 3 + kw];
                    int dh = kh - 1, dw = kw - 1;
                    for (int h = 0; h < H; ++h) {
                        int hh = h + dh;
                        if (hh < 0 || hh >= H) continue;
                        for (int x = 0; x < W; ++x) {
                            int ww = x + dw;
                            if (ww < 0 || ww >= W) continue;
                            op[h * W + x] += wv * ip[hh * W + ww];
                        }
                    }
                }
        }
    }
}

/* batch_norm2d eval: (x - mean) / sqrt(var + eps) * gamma + beta, then optional relu */
static void bn_relu(float *x, int c, int hw, const float *bn, int relu) {
    const float *g = bn, *be = bn + c, *mu = bn + 2 * c, *var = bn + 3 * c;
    for (int i = 0; i < c; ++i) {
        float inv = 1.0f / sqrtf(var[i] + 1e-5f);
        for (int p = 0; p < hw; ++p) {
            float v = (x[(size_t)i * hw + p] - mu[i]) * inv * g[i] + be[i];
            if (relu && v < 0.0f) v = 0.0f;
            x[(size_t)i * hw + p] = v;
        }
    }
}

static void forward_one(const or_net *net, const float *x, float *logits, float *value, float *buf) {
    const int C = net->C, H = net->H, W = net->W, A = net->A, hid = net->hidden, HW = H * W;
    float *a = buf, *b = buf + (size_t)hid * HW, *c = buf + (size_t)2 * hid * HW;
    const float *p = net->params;
    /* stem: conv, BN, ReLU (mod.rs:167-177) */
    conv3x3(x, C, H, W, p, p + (size_t)hid * C * 9, hid, a);
    p += PCONV(C, hid);
    bn_relu(a, hid, HW, p, 1);
    p += PBN(hid);
    /* residual blocks (mod.rs:152-165): relu(x + BN(conv(relu(BN(conv(x)))))) */
    for (int blk = 0; blk < net->blocks; ++blk) {
        conv3x3(a, hid, H, W, p, p + (size_t)hid * hid * 9, hid, b);
        p += PCONV(hid, hid);
        bn_relu(b, hid, HW, p, 1);
        p += PBN(hid);
        conv3x3(b, hid, H, W, p, p + (size_t)hid * hid * 9, hid, c);
        p += PCONV(hid, hid);
        bn_relu(c, hid, HW, p, 0);
        p += PBN(hid);
        for (size_t i = 0; i < (size_t)hid * HW; ++i) {
            float v = a[i] + c[i];
            a[i] = v < 0.0f ? 0.0f : v;
        }
    }
    /* policy head (connect_four.rs:59-64): conv 3x3 -> 32, BN, ReLU, flatten, linear */
    conv3x3(a, hid, H, W, p, p + (size_t)32 * hid * 9, 32, b);
    p += PCONV(hid, 32);
    bn_relu(b, 32, HW, p, 1);
    p += PBN(32);
    const float *lw = p, *lb = p + (size_t)A * 32 * HW;
    for (int o = 0; o < A; ++o) {
        float s = 0.0f;
        for (int i = 0; i < 32 * HW; ++i) s += b[i] * lw[(size_t)o * 32 * HW + i];
        logits[o] = s + lb[o];
    }
    p += (size_t)A * 32 * HW + A;
    /* value head (connect_four.rs:65-71): conv 3x3 -> 3, BN, ReLU, flatten, linear, tanh */
    conv3x3(a, hid, H, W, p, p + (size_t)3 * hid * 9, 3, b);
    p += PCONV(hid, 3);
    bn_relu(b, 3, HW, p, 1);
    p += PBN(3);
    float s = 0.0f;
    for (int i = 0; i < 3 * HW; ++i) s += b[i] * p[i];
    *value = tanhf(s + p[3 * HW]);
}

void or_net_forward(const or_net *net, int n, const float *x, float *logits, float *value) {
    const int HW = net->H * net->W;
    float *buf = (float *)malloc(sizeof(float) * 3 * (size_t)net->hidden * HW);
    for (int i = 0; i < n; ++i)
        forward_one(net, x + (size_t)i * net->C * HW, logits + (size_t)i * net->A, value + i, buf);
    free(buf);
}

/* softmax(-1) then mask_invalid_actions per state, values as-is (mod.rs:62-95) */
void or_predict(const or_net *net, int n, const void *const *states, float *priors, float *values) {
    const or_game *g = or_game_get(net->game);
    const int A = net->A, in = net->C * net->H * net->W;
    float *x = (float *)malloc(sizeof(float) * (size_t)in * (n > 0 ? n : 1));
    float *lg = (float *)malloc(sizeof(float) * (size_t)A * (n > 0 ? n : 1));
    for (int i = 0; i < n; ++i) g->encoding(states[i], x + (size_t)i * in);
    or_net_forward(net, n, x, lg, values);
    for (int i = 0; i < n; ++i) {
        float *l = lg + (size_t)i * A, sm[OR_MAX_ACTIONS];
        float mx = l[0];
        for (int a = 1; a < A; ++a) mx = l[a] > mx ? l[a] : mx;
        float s = 0.0f;
        for (int a = 0; a < A; ++a) { sm[a] = expf(l[a] - mx); s += sm[a]; }
        for (int a = 0; a < A; ++a) sm[a] = sm[a] / s;
        g->mask_invalid(states[i], sm, A, priors + (size_t)i * A);
    }
    free(x);
    free(lg);
}

/* ---- random init (tch 0.13 defaults as restated in DESIGN.md) ---- */
static float philox_unit(uint64_t seed, uint32_t tensor, uint64_t idx) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), tensor, 0x5EEDu};
    uint32_t out[4];
    or_philox4x32(ctr, key, out);
    return (float)(out[0] >> 8) * (1.0f / 16777216.0f);
}

static float *fill_uniform(float *p, size_t n, float lo, float hi, uint64_t seed, uint32_t *tensor) {
    for (size_t i = 0; i < n; ++i) p[i] = lo + (hi - lo) * philox_unit(seed, *tensor, i);
    ++*tensor;
    return p + n;
}
static float *fill_const(float *p, size_t n, float v, uint32_t *tensor) {
    for (size_t i = 0; i < n; ++i) p[i] = v;
    ++*tensor;
    return p + n;
}
static float *init_conv(float *p, int ci, int co, uint64_t seed, uint32_t *t) {
    float bound = (float)sqrt(6.0 / (double)(ci * 9));          /* Kaiming uniform, ReLU gain, fan_in */
    p = fill_uniform(p, (size_t)co * ci * 9, -bound, bound, seed, t);
    return fill_const(p, co, 0.0f, t);                           /* bs_init Const(0) */
}
static float *init_bn(float *p, int c, uint64_t seed, uint32_t *t) {
    p = fill_uniform(p, c, 0.0f, 1.0f, seed, t);                 /* ws_init Uniform(0,1) */
    p = fill_const(p, c, 0.0f, t);
    p = fill_const(p, c, 0.0f, t);                               /* running_mean */
    return fill_const(p, c, 1.0f, t);                            /* running_var */
}
static float *init_linear(float *p, int in, int out, uint64_t seed, uint32_t *t) {
    float bound = (float)sqrt(6.0 / (double)in);
    p = fill_uniform(p, (size_t)out * in, -bound, bound, seed, t);
    float bb = (float)(1.0 / sqrt((double)in));                 /* bias U(+-1/sqrt(fan_in)) */
    return fill_uniform(p, out, -bb, bb, seed, t);
}

void or_net_init_params(int game, int blocks, int hidden, uint64_t seed, float *params) {
    int C, H, W, A;
    game_dims(game, &C, &H, &W, &A);
    uint32_t t = 0;
    float *p = params;
    p = init_conv(p, C, hidden, seed, &t);
    p = init_bn(p, hidden, seed, &t);
    for (int b = 0; b < blocks; ++b) {
        p = init_conv(p, hidden, hidden, seed, &t);
        p = init_bn(p, hidden, seed, &t);
        p = init_conv(p, hidden, hidden, seed, &t);
        p = init_bn(p, hidden, seed, &t);
    }
    p = init_conv(p, hidden, 32, seed, &t);
    p = init_bn(p, 32, seed, &t);
    p = init_linear(p, 32 * H * W, A, seed, &t);
    p = init_conv(p, hidden, 3, seed, &t);
    p = init_bn(p, 3, seed, &t);
    p = init_linear(p, 3 * H * W, 1, seed, &t);
}

/* ========================================================================
 * MCTS — mcts.rs.  Node = full State + id + parent + action + prior +
 * children Vec + visit_count + value_sum (:20-30).
 * ====================================================================== */
typedef struct {
    unsigned char state[OR_MAX_STATE];
    int id, parent, action;
    float prior;           /* Option<f32>; NaN for None (root) */
    int *children;
    int n_children, cap_children;
    uint32_t visit_count;
    float value_sum;
} or_node;

struct or_tree {
    int game;
    or_node *arena;
    int size, cap;
    int node_id_to_expand;  /* Option<usize>; -1 = None */
};

static void node_push_child(or_node *n, int id) {
    if (n->n_children == n->cap_children) {
        n->cap_children = n->cap_children ? n->cap_children * 2 : 8;
        n->children = (int *)realloc(n->children, sizeof(int) * n->cap_children);
    }
    n->children[n->n_children++] = id;
}

static int arena_push(or_tree *t, const or_node *n) {
    if (t->size == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->arena = (or_node *)realloc(t->arena, sizeof(or_node) * t->cap);
    }
    t->arena[t->size] = *n;
    return t->size++;
}

or_tree *or_tree_with_root(int game, const void *state) {  /* :79-89 */
    const or_game *g = or_game_get(game);
    if (!g) return NULL;
    or_tree *t = (or_tree *)calloc(1, sizeof(or_tree));
    t->game = game;
    t->node_id_to_expand = -1;
    or_node root;
    memset(&root, 0, sizeof(root));
    memcpy(root.state, state, g->state_size);
    root.parent = -1;
    root.action = -1;
    root.prior = NAN;
    arena_push(t, &root);
    return t;
}

or_tree *or_tree_create(int game) {  /* Tree::default(), :67-77 */
    unsigned char st[OR_MAX_STATE];
    const or_game *g = or_game_get(game);
    if (!g) return NULL;
    g->init(st);
    return or_tree_with_root(game, st);
}

void or_tree_destroy(or_tree *t) {
    if (!t) return;
    for (int i = 0; i < t->size; ++i) free(t->arena[i].children);
    free(t->arena);
    free(t);
}

int or_tree_size(const or_tree *t) { return t->size; }
const void *or_tree_node_state(const or_tree *t, int id) { return t->arena[id].state; }

int or_tree_node_info(const or_tree *t, int id, int *parent, int *action, float *prior, uint32_t *visits,
                      float *value_sum, int *n_children, int *children) {
    if (id < 0 || id >= t->size) return -1;
    const or_node *n = &t->arena[id];
    if (parent) *parent = n->parent;
    if (action) *action = n->action;
    if (prior) *prior = n->prior;
    if (visits) *visits = n->visit_count;
    if (value_sum) *value_sum = n->value_sum;
    if (n_children) *n_children = n->n_children;
    if (children)
        for (int i = 0; i < n->n_children; ++i) children[i] = n->children[i];
    return 0;
}

/* get_ucb, :91-100.  c is Tree.args.c = Args::default().c (quirk Q6). */
static float get_ucb(const or_tree *t, int parent_id, int child_id, float c) {
    const or_node *p = &t->arena[parent_id], *ch = &t->arena[child_id];
    float q;
    if (ch->visit_count == 0) q = 0.0f;
    else q = ((-ch->value_sum / (float)ch->visit_count) + 1.0f) / 2.0f;
    float u = c * ch->prior;
    u = u * sqrtf((float)p->visit_count);
    u = u / (1.0f + (float)ch->visit_count);
    return q + u;
}

/* select, :102-114: Iterator::max_by returns the LAST maximum (quirk Q2). */
static int tree_select(const or_tree *t, int parent_id, float c, int *err) {
    const or_node *p = &t->arena[parent_id];
    int best = p->children[0];
    float bu = get_ucb(t, parent_id, best, c);
    if (isnan(bu)) *err = 1;
    for (int i = 1; i < p->n_children; ++i) {
        int id = p->children[i];
        float u = get_ucb(t, parent_id, id, c);
        if (isnan(u)) *err = 1;                 /* partial_cmp().unwrap() panics */
        if (!(u < bu)) { best = id; bu = u; }   /* ties -> later element */
    }
    return best;
}

/* expand, :116-143 */
static void tree_expand(or_tree *t, int parent_id, const float *policy) {
    const or_game *g = or_game_get(t->game);
    int acts[OR_MAX_ACTIONS];
    unsigned char parent_state[OR_MAX_STATE];
    memcpy(parent_state, t->arena[parent_id].state, g->state_size);
    int na = g->valid_actions(parent_state, acts);
    int first = t->size;
    for (int i = 0; i < na; ++i) node_push_child(&t->arena[parent_id], first + i);
    for (int i = 0; i < na; ++i) {
        or_node ch;
        memset(&ch, 0, sizeof(ch));
        g->next_state(parent_state, acts[i], ch.state);
        ch.id = first + i;
        ch.parent = parent_id;
        ch.action = acts[i];
        ch.prior = policy[acts[i]];
        arena_push(t, &ch);
    }
}

/* backprop, :145-159 */
static void tree_backprop(or_tree *t, int node_id, float value) {
    float sign = 1.0f;
    or_node *n = &t->arena[node_id];
    n->visit_count += 1;
    n->value_sum += sign * value;
    sign *= -1.0f;
    while (n->parent >= 0) {
        n = &t->arena[n->parent];
        n->visit_count += 1;
        n->value_sum += sign * value;
        sign *= -1.0f;
    }
}

/* use_subtree, :161-192: BFS copy into a new arena; the new root keeps N and W. */
void or_tree_use_subtree(or_tree *t, int new_root_id) {
    or_node *old = t->arena;
    int old_size = t->size;
    or_node *queue = (or_node *)malloc(sizeof(or_node) * (old_size + 1));
    int qh = 0, qt = 0;
    or_tree nt = {t->game, NULL, 0, 0, t->node_id_to_expand};
    or_node root = old[new_root_id];
    root.parent = -1;
    queue[qt++] = root;
    int next_id = 0;
    while (qh < qt) {
        or_node node = queue[qh++];
        node.id = next_id;
        for (int i = 0; i < node.n_children; ++i) {
            or_node ch = old[node.children[i]];
            ch.parent = node.id;
            queue[qt++] = ch;
        }
        node.children = NULL;            /* children.clear(); fresh Vec */
        node.n_children = node.cap_children = 0;
        if (node.parent >= 0) node_push_child(&nt.arena[node.parent], node.id);
        arena_push(&nt, &node);
        ++next_id;
    }
    free(queue);
    for (int i = 0; i < old_size; ++i) free(old[i].children);
    free(old);
    t->arena = nt.arena;
    t->size = nt.size;
    t->cap = nt.cap;
}

/* Mcts::search, :196-332 */
int or_search(or_tree **trees, int n, int num_searches, float c, int eval_kind, const or_net *net,
              or_eval_fn eval, void *eval_user, float *policy, int *child_ids, float *child_visits,
              int *n_children) {
    if (n <= 0) return 0;
    const int game = trees[0]->game;
    const or_game *g = or_game_get(game);
    const int A = g->num_actions;
    int *batch = (int *)malloc(sizeof(int) * n);
    const void **states = (const void **)malloc(sizeof(void *) * n);
    float *pri = (float *)malloc(sizeof(float) * (size_t)n * A);
    float *val = (float *)malloc(sizeof(float) * n);
    int err = 0;
    long evals = 0;
    for (int it = 0; it < num_searches; ++it) {
        int nb = 0;
        for (int ti = 0; ti < n; ++ti) {                          /* :235-252 */
            or_tree *t = trees[ti];
            int node = 0;
            while (t->arena[node].n_children > 0) node = tree_select(t, node, c, &err);
            float v;
            int term;
            g->value_terminated(t->arena[node].state, &v, &term);
            if (term) {
                tree_backprop(t, node, v);
                t->node_id_to_expand = -1;
            } else {
                t->node_id_to_expand = node;
                batch[nb++] = ti;
            }
        }
        evals += nb;
        if (nb > 0) {                                             /* :254-285 */
            for (int k = 0; k < nb; ++k) {
                or_tree *t = trees[batch[k]];
                states[k] = t->arena[t->node_id_to_expand].state;
            }
            if (eval) eval(eval_user, nb, states, pri, val);
            else if (eval_kind == OR_EVAL_NET) or_predict(net, nb, states, pri, val);
            else stub_eval(game, eval_kind, nb, states, pri, val);
            for (int k = 0; k < nb; ++k) {
                or_tree *t = trees[batch[k]];
                int id = t->node_id_to_expand;
                tree_expand(t, id, pri + (size_t)k * A);
                tree_backprop(t, id, val[k]);
            }
        }
    }
    for (int ti = 0; ti < n; ++ti) {                              /* :310-331 */
        const or_tree *t = trees[ti];
        const or_node *root = &t->arena[0];
        float *pol = policy + (size_t)ti * A;
        for (int a = 0; a < A; ++a) pol[a] = 0.0f;
        for (int k = 0; k < root->n_children; ++k) {
            const or_node *ch = &t->arena[root->children[k]];
            float cv = (float)ch->visit_count;
            pol[ch->action] = cv;
            if (child_ids) child_ids[(size_t)ti * A + k] = root->children[k];
            if (child_visits) child_visits[(size_t)ti * A + k] = cv;
        }
        if (n_children) n_children[ti] = root->n_children;
        float s = or_nd_sum(pol, A);
        for (int a = 0; a < A; ++a) pol[a] = pol[a] / s;
    }
    free(batch);
    free(states);
    free(pri);
    free(val);
    return err ? -1 : (int)(evals > 0x7fffffff ? 0x7fffffff : evals);
}

/* ========================================================================
 * SelfPlayWorker::self_play, learner_concurrent.rs:169-242.
 * ====================================================================== */
typedef struct {
    or_tree *tree;
    int game_index;
    int n_hist, cap_hist;
    unsigned char *states;  /* history of root states */
    float *policies;        /* history of visit policies */
} sp_game;

long or_self_play(int game, int n_games, int num_searches, float c, float temperature, uint64_t seed,
                  uint64_t game_id_base, int eval_kind, const or_net *net, or_eval_fn eval, void *eval_user,
                  long cap, float *enc, float *pol, float *val, int32_t *game_ids, int32_t *plies,
                  int max_plies, int32_t *moves, int32_t *n_moves, double *stats) {
    const or_game *g = or_game_get(game);
    if (!g) return -1;
    const int A = g->num_actions, E = g->enc_c * g->enc_h * g->enc_w;
    const size_t SS = g->state_size;
    sp_game *games = (sp_game *)calloc(n_games, sizeof(sp_game));
    or_tree **act = (or_tree **)malloc(sizeof(or_tree *) * (n_games > 0 ? n_games : 1));
    int *act_idx = (int *)malloc(sizeof(int) * (n_games > 0 ? n_games : 1));
    float *rpol = (float *)malloc(sizeof(float) * (size_t)A * (n_games > 0 ? n_games : 1));
    int *rids = (int *)malloc(sizeof(int) * (size_t)A * (n_games > 0 ? n_games : 1));
    float *rvis = (float *)malloc(sizeof(float) * (size_t)A * (n_games > 0 ? n_games : 1));
    int *rnc = (int *)malloc(sizeof(int) * (n_games > 0 ? n_games : 1));
    long out = 0;
    int n_act = n_games;
    int move_no = 0;
    double sims = 0, evals = 0;
    int rc = 0;
    for (int i = 0; i < n_games; ++i) {
        games[i].tree = or_tree_create(game);
        games[i].game_index = i;
        act_idx[i] = i;
        if (n_moves) n_moves[i] = 0;
    }
    while (n_act > 0) {
        for (int k = 0; k < n_act; ++k) act[k] = games[act_idx[k]].tree;
        int ne = or_search(act, n_act, num_searches, c, eval_kind, net, eval, eval_user, rpol, rids, rvis, rnc);
        if (ne < 0) {
            rc = -3;
            break;
        }
        evals += ne;
        sims += (double)n_act * num_searches;
        for (int k = n_act - 1; k >= 0; --k) {                    /* :182 rev(0..n) */
            sp_game *sg = &games[act_idx[k]];
            or_tree *t = sg->tree;
            int nc = rnc[k];
            float u = or_u01_f32(seed, game_id_base + (uint64_t)sg->game_index, (uint64_t)move_no);
            int idx = or_weighted_index(rvis + (size_t)k * A, nc, temperature, u);
            if (idx < 0) { rc = -4; goto done; }
            int selected = rids[(size_t)k * A + idx];
            if (sg->n_hist == sg->cap_hist) {
                sg->cap_hist = sg->cap_hist ? 2 * sg->cap_hist : 16;
                sg->states = (unsigned char *)realloc(sg->states, SS * sg->cap_hist);
                sg->policies = (float *)realloc(sg->policies, sizeof(float) * A * sg->cap_hist);
            }
            memcpy(sg->states + SS * sg->n_hist, t->arena[0].state, SS);
            memcpy(sg->policies + (size_t)A * sg->n_hist, rpol + (size_t)k * A, sizeof(float) * A);
            sg->n_hist++;
            if (moves && sg->n_hist <= max_plies)
                moves[(size_t)sg->game_index * max_plies + sg->n_hist - 1] = t->arena[selected].action;
            if (n_moves) n_moves[sg->game_index] = sg->n_hist;
            const void *st = t->arena[selected].state;
            float v;
            int term;
            g->value_terminated(st, &v, &term);
            if (term) {                                           /* :200-230 */
                int cur = g->current_player(st);
                for (int h = 0; h < sg->n_hist; ++h) {
                    if (out < cap) {
                        const void *hs = sg->states + SS * h;
                        if (enc) g->encoding(hs, enc + (size_t)out * E);
                        if (pol) memcpy(pol + (size_t)out * A, sg->policies + (size_t)A * h, sizeof(float) * A);
                        if (val) val[out] = g->current_player(hs) == cur ? v : -v;
                        if (game_ids) game_ids[out] = sg->game_index;
                        if (plies) plies[out] = h;
                    }
                    ++out;
                }
                for (int j = k; j < n_act - 1; ++j) act_idx[j] = act_idx[j + 1];   /* trees_vec.remove(i) */
                --n_act;
            } else {
                t->node_id_to_expand = -1;
                or_tree_use_subtree(t, selected);
            }
        }
        ++move_no;
    }
done:
    for (int i = 0; i < n_games; ++i) {
        or_tree_destroy(games[i].tree);
        free(games[i].states);
        free(games[i].policies);
    }
    if (stats) { stats[0] = sims; stats[1] = evals; }
    free(games); free(act); free(act_idx); free(rpol); free(rids); free(rvis); free(rnc);
    return rc < 0 ? rc : out;
}

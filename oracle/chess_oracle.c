/*
 * chess_oracle.c — CPU restatement of the reference chess path.
 * TEST INFRASTRUCTURE ONLY (scope and pinning: chess_oracle.h).
 *
 * Written for fidelity: slider attacks by plain ray walks, the crate's
 * enumeration order, the adapter's Vec<ChessMove> transposition table kept as
 * full move lists and compared element by element (chess.rs:51-61), and a
 * node arena holding a full State per node (mcts.rs:20-30).
 */
#include "chess_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "spai_oracle.h"

typedef uint64_t bb;
#define SQ(r, f) ((r) * 8 + (f))
#define BIT(s) (1ull << (s))

static int popcnt(bb x) { return __builtin_popcountll(x); }
static int lsb(bb x) { return __builtin_ctzll(x); }

/* ---- attack tables (chess crate: get_knight_moves, get_king_moves, rays,
 *      between, line, PAWN_MOVES / PAWN_ATTACKS) ---- */
static bb KNIGHT[64], KING[64], BRAYS[64], RRAYS[64], BETWEEN[64][64], LINE[64][64];
static bb PMOVES[2][64], PATT[2][64];
static int tables_ready = 0;
static const int DR[8] = {1, -1, 0, 0, 1, 1, -1, -1}, DF[8] = {0, 0, 1, -1, 1, -1, 1, -1};

static void init_tables(void) {
    if (tables_ready) return;
    for (int s = 0; s < 64; ++s) {
        int r = s >> 3, f = s & 7;
        static const int kr[8] = {2, 2, 1, 1, -1, -1, -2, -2}, kf[8] = {1, -1, 2, -2, 2, -2, 1, -1};
        for (int i = 0; i < 8; ++i) {
            int rr = r + kr[i], ff = f + kf[i];
            if (rr >= 0 && rr < 8 && ff >= 0 && ff < 8) KNIGHT[s] |= BIT(SQ(rr, ff));
        }
        for (int dr = -1; dr <= 1; ++dr)
            for (int df = -1; df <= 1; ++df) {
                if (!dr && !df) continue;
                int rr = r + dr, ff = f + df;
                if (rr >= 0 && rr < 8 && ff >= 0 && ff < 8) KING[s] |= BIT(SQ(rr, ff));
            }
        for (int d = 0; d < 8; ++d)
            for (int k = 1; k < 8; ++k) {
                int rr = r + DR[d] * k, ff = f + DF[d] * k;
                if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
                if (d < 4) RRAYS[s] |= BIT(SQ(rr, ff));
                else BRAYS[s] |= BIT(SQ(rr, ff));
            }
        for (int c = 0; c < 2; ++c) {
            int fw = c == ORC_WHITE ? 1 : -1, r1 = r + fw;
            if (r1 >= 0 && r1 < 8) {
                PMOVES[c][s] |= BIT(SQ(r1, f));
                if (f > 0) PATT[c][s] |= BIT(SQ(r1, f - 1));
                if (f < 7) PATT[c][s] |= BIT(SQ(r1, f + 1));
                if ((c == ORC_WHITE && r == 1) || (c == ORC_BLACK && r == 6)) PMOVES[c][s] |= BIT(SQ(r + 2 * fw, f));
            }
        }
    }
    for (int a = 0; a < 64; ++a)
        for (int d = 0; d < 8; ++d) {
            int r = a >> 3, f = a & 7;
            bb acc = 0;
            for (int k = 1; k < 8; ++k) {
                int rr = r + DR[d] * k, ff = f + DF[d] * k;
                if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
                int b = SQ(rr, ff);
                BETWEEN[a][b] = acc;
                acc |= BIT(b);
            }
            /* full line through a in direction d (both ways) */
            bb ln = BIT(a);
            for (int k = 1; k < 8; ++k) {
                int rr = r + DR[d] * k, ff = f + DF[d] * k;
                if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
                ln |= BIT(SQ(rr, ff));
            }
            for (int k = 1; k < 8; ++k) {
                int rr = r - DR[d] * k, ff = f - DF[d] * k;
                if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
                ln |= BIT(SQ(rr, ff));
            }
            for (int k = 1; k < 8; ++k) {
                int rr = r + DR[d] * k, ff = f + DF[d] * k;
                if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
                LINE[a][SQ(rr, ff)] = ln;
            }
        }
    tables_ready = 1;
}

static bb ray_attacks(int s, bb occ, int d0, int d1) {
    bb a = 0;
    int r = s >> 3, f = s & 7;
    for (int d = d0; d < d1; ++d)
        for (int k = 1; k < 8; ++k) {
            int rr = r + DR[d] * k, ff = f + DF[d] * k;
            if (rr < 0 || rr > 7 || ff < 0 || ff > 7) break;
            a |= BIT(SQ(rr, ff));
            if (occ & BIT(SQ(rr, ff))) break;
        }
    return a;
}
static bb rook_moves(int s, bb occ) { return ray_attacks(s, occ, 0, 4); }
static bb bishop_moves(int s, bb occ) { return ray_attacks(s, occ, 4, 8); }

static bb pawn_quiets(int s, int c, bb occ) {               /* get_pawn_quiets */
    int fwd = c == ORC_WHITE ? s + 8 : s - 8;
    if (fwd < 0 || fwd > 63 || (BIT(fwd) & occ)) return 0;
    return PMOVES[c][s] & ~occ;
}

/* ---- Board ---- */
static bb occ_all(const orc_board *b) { return b->color[0] | b->color[1]; }
static int piece_on(const orc_board *b, int s) {
    for (int p = 0; p < 6; ++p)
        if (b->pieces[p] & BIT(s)) return p;
    return -1;
}
static int king_sq(const orc_board *b, int c) { return lsb(b->pieces[ORC_KING] & b->color[c]); }

void orc_board_start(orc_board *b) {
    init_tables();
    memset(b, 0, sizeof(*b));
    static const int back[8] = {ORC_ROOK, ORC_KNIGHT, ORC_BISHOP, ORC_QUEEN, ORC_KING, ORC_BISHOP, ORC_KNIGHT, ORC_ROOK};
    for (int f = 0; f < 8; ++f) {
        b->pieces[back[f]] |= BIT(SQ(0, f)) | BIT(SQ(7, f));
        b->pieces[ORC_PAWN] |= BIT(SQ(1, f)) | BIT(SQ(6, f));
        b->color[ORC_WHITE] |= BIT(SQ(0, f)) | BIT(SQ(1, f));
        b->color[ORC_BLACK] |= BIT(SQ(6, f)) | BIT(SQ(7, f));
    }
    b->castle[0] = b->castle[1] = 3;
    b->ep = ORC_NO_EP;
}

int orc_board_from_fen(const char *fen, orc_board *b) {
    init_tables();
    memset(b, 0, sizeof(*b));
    b->ep = ORC_NO_EP;
    int r = 7, f = 0;
    const char *p = fen;
    for (; *p && *p != ' '; ++p) {
        char ch = *p;
        if (ch == '/') { --r; f = 0; continue; }
        if (ch >= '1' && ch <= '8') { f += ch - '0'; continue; }
        int c = (ch >= 'a') ? ORC_BLACK : ORC_WHITE;
        char l = (char)(ch | 0x20);
        int pc = l == 'p' ? ORC_PAWN : l == 'n' ? ORC_KNIGHT : l == 'b' ? ORC_BISHOP : l == 'r' ? ORC_ROOK
               : l == 'q' ? ORC_QUEEN : l == 'k' ? ORC_KING : -1;
        if (pc < 0 || r < 0 || f > 7) return -1;
        b->pieces[pc] |= BIT(SQ(r, f));
        b->color[c] |= BIT(SQ(r, f));
        ++f;
    }
    if (*p != ' ') return -1;
    ++p;
    b->side = (*p == 'b') ? ORC_BLACK : ORC_WHITE;
    p += 2;
    for (; *p && *p != ' '; ++p) {
        if (*p == 'K') b->castle[0] |= 1;
        if (*p == 'Q') b->castle[0] |= 2;
        if (*p == 'k') b->castle[1] |= 1;
        if (*p == 'q') b->castle[1] |= 2;
    }
    if (*p == ' ') ++p;
    if (*p && *p != '-') {
        int ef = p[0] - 'a', er = p[1] - '1';
        /* FEN gives the target square; the crate stores the pawn's square, and
         * only when an enemy pawn can capture it (Board::set_ep) */
        int pawn = b->side == ORC_WHITE ? SQ(er - 1, ef) : SQ(er + 1, ef);
        bb adj = 0;
        if (ef > 0) adj |= BIT(pawn - 1);
        if (ef < 7) adj |= BIT(pawn + 1);
        if (adj & b->pieces[ORC_PAWN] & b->color[b->side]) b->ep = (uint8_t)pawn;
    }
    return 0;
}

/* checkers of the side to move's king; pinned pieces (of either colour that
 * sit alone between the king and an enemy slider — only the mover's matter) */
static void checkers_pinned(const orc_board *b, bb *checkers, bb *pinned) {
    int c = b->side, o = c ^ 1, k = king_sq(b, c);
    bb occ = occ_all(b), them = b->color[o];
    bb ch = 0, pin = 0;
    ch |= KNIGHT[k] & b->pieces[ORC_KNIGHT] & them;
    ch |= PATT[c][k] & b->pieces[ORC_PAWN] & them;
    bb sl = them & ((BRAYS[k] & (b->pieces[ORC_BISHOP] | b->pieces[ORC_QUEEN])) |
                    (RRAYS[k] & (b->pieces[ORC_ROOK] | b->pieces[ORC_QUEEN])));
    for (bb s = sl; s; s &= s - 1) {
        int q = lsb(s);
        bb btw = BETWEEN[q][k] & occ;
        if (!btw) ch |= BIT(q);
        else if (popcnt(btw) == 1) pin |= btw;
    }
    *checkers = ch;
    *pinned = pin;
}

int orc_in_check(const orc_board *b) {
    bb ch, pin;
    checkers_pinned(b, &ch, &pin);
    return ch != 0;
}

static int legal_king_move(const orc_board *b, int dest) {   /* KingType::legal_king_move */
    int c = b->side, o = c ^ 1;
    bb occ = (occ_all(b) ^ (b->pieces[ORC_KING] & b->color[c])) | BIT(dest);
    bb them = b->color[o], att = 0;
    att |= rook_moves(dest, occ) & (b->pieces[ORC_ROOK] | b->pieces[ORC_QUEEN]) & them;
    att |= bishop_moves(dest, occ) & (b->pieces[ORC_BISHOP] | b->pieces[ORC_QUEEN]) & them;
    att |= KNIGHT[dest] & b->pieces[ORC_KNIGHT] & them;
    att |= KING[dest] & b->pieces[ORC_KING] & them;
    att |= PATT[c][dest] & b->pieces[ORC_PAWN] & them;
    return att == 0;
}

static int legal_ep_move(const orc_board *b, int src, int dest) {   /* PawnType::legal_ep_move */
    int c = b->side, o = c ^ 1;
    bb occ = occ_all(b) ^ BIT(b->ep) ^ BIT(src) ^ BIT(dest);
    int k = king_sq(b, c);
    bb rooks = (b->pieces[ORC_ROOK] | b->pieces[ORC_QUEEN]) & b->color[o];
    if ((RRAYS[k] & rooks) && (rook_moves(k, occ) & rooks)) return 0;
    bb bish = (b->pieces[ORC_BISHOP] | b->pieces[ORC_QUEEN]) & b->color[o];
    if ((BRAYS[k] & bish) && (bishop_moves(k, occ) & bish)) return 0;
    return 1;
}

static bb pseudo(const orc_board *b, int piece, int s, bb mask) {
    bb occ = occ_all(b);
    int c = b->side;
    switch (piece) {
        case ORC_PAWN: return ((PATT[c][s] & occ) ^ pawn_quiets(s, c, occ)) & mask;
        case ORC_KNIGHT: return KNIGHT[s] & mask;
        case ORC_BISHOP: return bishop_moves(s, occ) & mask;
        case ORC_ROOK: return rook_moves(s, occ) & mask;
        case ORC_QUEEN: return (bishop_moves(s, occ) | rook_moves(s, occ)) & mask;
        default: return KING[s] & mask;
    }
}

/* SquareAndBitBoard list entry expansion (MoveGen::next): destinations
 * ascending, promotions in PROMOTION_PIECES order Queen, Knight, Rook, Bishop */
static int emit(uint16_t *out, int n, int src, bb dests, int promo) {
    static const int PROMO[4] = {ORC_QUEEN, ORC_KNIGHT, ORC_ROOK, ORC_BISHOP};
    for (bb d = dests; d; d &= d - 1) {
        int dst = lsb(d);
        if (promo)
            for (int i = 0; i < 4; ++i) out[n++] = (uint16_t)orc_move(src, dst, PROMO[i]);
        else
            out[n++] = (uint16_t)orc_move(src, dst, 0);
    }
    return n;
}

/* MoveGen::enumerate_moves (chess 3.2.0 movegen.rs) + iteration */
int orc_legal_moves(const orc_board *b, uint16_t *out) {
    init_tables();
    int c = b->side, k = king_sq(b, c);
    bb mine = b->color[c], mask = ~mine;
    bb checkers, pinned;
    checkers_pinned(b, &checkers, &pinned);
    int n = 0;
    int nchk = popcnt(checkers);
    if (nchk <= 1) {
        int in_check = nchk == 1;
        bb check_mask = in_check ? (BETWEEN[lsb(checkers)][k] ^ checkers) : ~0ull;
        for (int piece = ORC_PAWN; piece <= ORC_QUEEN; ++piece) {
            bb pcs = b->pieces[piece] & mine;
            for (bb s = pcs & ~pinned; s; s &= s - 1) {
                int src = lsb(s);
                bb m = pseudo(b, piece, src, mask) & check_mask;
                int promo = piece == ORC_PAWN && (src >> 3) == (c == ORC_WHITE ? 6 : 1);
                if (m) n = emit(out, n, src, m, promo);
            }
            if (!in_check)
                for (bb s = pcs & pinned; s; s &= s - 1) {
                    int src = lsb(s);
                    bb m = pseudo(b, piece, src, mask) & LINE[k][src];
                    int promo = piece == ORC_PAWN && (src >> 3) == (c == ORC_WHITE ? 6 : 1);
                    if (m) n = emit(out, n, src, m, promo);
                }
            if (piece == ORC_PAWN && b->ep != ORC_NO_EP) {
                int ep = b->ep, er = ep >> 3, ef = ep & 7;
                bb rank = 0xFFull << (8 * er), files = 0;
                if (ef > 0) files |= 0x0101010101010101ull << (ef - 1);
                if (ef < 7) files |= 0x0101010101010101ull << (ef + 1);
                int dest = c == ORC_WHITE ? ep + 8 : ep - 8;
                for (bb s = rank & files & pcs; s; s &= s - 1) {
                    int src = lsb(s);
                    if (legal_ep_move(b, src, dest)) n = emit(out, n, src, BIT(dest), 0);
                }
            }
        }
    }
    /* KingType::legals */
    bb occ = occ_all(b);
    bb m = KING[k] & mask, copy = m;
    for (bb d = copy; d; d &= d - 1)
        if (!legal_king_move(b, lsb(d))) m ^= BIT(lsb(d));
    if (!checkers) {
        int rank0 = c == ORC_WHITE ? 0 : 56;
        bb ks = BIT(rank0 + 5) | BIT(rank0 + 6), qs = BIT(rank0 + 1) | BIT(rank0 + 2) | BIT(rank0 + 3);
        if ((b->castle[c] & 1) && !(occ & ks) && legal_king_move(b, k + 1) && legal_king_move(b, k + 2))
            m ^= BIT(k + 2);
        if ((b->castle[c] & 2) && !(occ & qs) && legal_king_move(b, k - 1) && legal_king_move(b, k - 2))
            m ^= BIT(k - 2);
    }
    if (m) n = emit(out, n, k, m, 0);
    return n;
}

/* CastleRights::square_to_castle_rights */
static int sq_castle(int c, int s) {
    int r0 = c == ORC_WHITE ? 0 : 56;
    if (s == r0) return 2;
    if (s == r0 + 4) return 3;
    if (s == r0 + 7) return 1;
    return 0;
}

static void xorp(orc_board *b, int piece, bb m, int c) {
    b->pieces[piece] ^= m;
    b->color[c] ^= m;
}

/* Board::make_move (chess 3.2.0 board.rs) */
void orc_board_make_move(const orc_board *b, int move, orc_board *r) {
    int src = move & 63, dst = (move >> 6) & 63, promo = (move >> 12) & 7;
    int c = b->side, o = c ^ 1;
    *r = *b;
    r->ep = ORC_NO_EP;
    bb sb = BIT(src), db = BIT(dst);
    int moved = piece_on(b, src);
    xorp(r, moved, sb, c);
    xorp(r, moved, db, c);
    int cap = piece_on(b, dst);
    if (cap >= 0) xorp(r, cap, db, o);
    r->castle[o] &= (uint8_t)~sq_castle(o, dst);
    r->castle[c] &= (uint8_t)~sq_castle(c, src);
    const bb castle_moves = BIT(2) | BIT(4) | BIT(6) | BIT(58) | BIT(60) | BIT(62);
    int castles = moved == ORC_KING && ((sb ^ db) & castle_moves) == (sb ^ db);
    if (moved == ORC_PAWN) {
        if (promo) {
            xorp(r, ORC_PAWN, db, c);
            xorp(r, promo, db, c);
        } else if ((sb & 0x00FF00000000FF00ull) && (db & 0x000000FFFF000000ull)) {
            /* set_ep: only when an enemy pawn stands beside the destination */
            int f = dst & 7;
            bb adj = 0;
            if (f > 0) adj |= BIT(dst - 1);
            if (f < 7) adj |= BIT(dst + 1);
            if (adj & r->pieces[ORC_PAWN] & r->color[o]) r->ep = (uint8_t)dst;
        } else if (b->ep != ORC_NO_EP && (c == ORC_WHITE ? dst - 8 : dst + 8) == b->ep) {
            xorp(r, ORC_PAWN, BIT(b->ep), o);
        }
    } else if (castles) {
        int r0 = c == ORC_WHITE ? 0 : 56, file = dst & 7;
        int rs = file == 2 ? r0 : r0 + 7, re = file == 2 ? r0 + 3 : r0 + 5;
        xorp(r, ORC_ROOK, BIT(rs), c);
        xorp(r, ORC_ROOK, BIT(re), c);
    }
    r->side = (uint8_t)o;
}

uint64_t orc_perft(const orc_board *b, int depth) {
    uint16_t mv[ORC_MAX_MOVES];
    int n = orc_legal_moves(b, mv);
    if (depth <= 1) return depth == 1 ? (uint64_t)n : 1;
    uint64_t t = 0;
    for (int i = 0; i < n; ++i) {
        orc_board nb;
        orc_board_make_move(b, mv[i], &nb);
        t += orc_perft(&nb, depth - 1);
    }
    return t;
}

/* ========================================================================
 * game/chess.rs State
 * ====================================================================== */
struct orc_hist {
    const orc_hist *prev;
    int n;
    uint16_t moves[];
};

/* transposition-table entries live in chunks freed by orc_arena_reset */
typedef struct chunk { struct chunk *next; size_t used, cap; } chunk;
static chunk *g_chunks = NULL;

static void *arena_alloc(size_t sz) {
    sz = (sz + 15) & ~(size_t)15;
    if (!g_chunks || g_chunks->used + sz > g_chunks->cap) {
        size_t cap = sz > (1u << 22) ? sz : (1u << 22);
        chunk *c = (chunk *)malloc(sizeof(chunk) + cap);
        c->next = g_chunks;
        c->used = 0;
        c->cap = cap;
        g_chunks = c;
    }
    void *p = (char *)(g_chunks + 1) + g_chunks->used;
    g_chunks->used += sz;
    return p;
}

void orc_arena_reset(void) {
    while (g_chunks) {
        chunk *n = g_chunks->next;
        free(g_chunks);
        g_chunks = n;
    }
}

void orc_state_init(orc_state *s) {
    memset(s, 0, sizeof(*s));
    orc_board_start(&s->b);
}

void orc_state_from_board(orc_state *s, const orc_board *b, uint32_t made, uint32_t fifty) {
    init_tables();
    memset(s, 0, sizeof(*s));
    s->b = *b;
    s->made = made;
    s->fifty = fifty;
}

int orc_num_repetitions(const orc_state *s) {               /* chess.rs:51-61 */
    uint16_t cur[ORC_MAX_MOVES];
    int n = orc_legal_moves(&s->b, cur);
    int count = 0;
    for (const orc_hist *h = s->tt; h; h = h->prev)
        if (h->n == n && memcmp(h->moves, cur, sizeof(uint16_t) * n) == 0) ++count;
    return count + 1;
}

int orc_status(const orc_state *s) {                        /* chess.rs:150-166 */
    uint16_t mv[ORC_MAX_MOVES];
    int n = orc_legal_moves(&s->b, mv);
    if (n == 0) return orc_in_check(&s->b) ? 2 : 1;         /* Checkmate -> Won, Stalemate -> Tied */
    if (orc_num_repetitions(s) >= 3 || s->fifty >= 100) return 1;
    return 0;
}

void orc_value_terminated(const orc_state *s, float *v, int *term) {   /* chess.rs:168-174, Won -> +1 (Q7) */
    int st = orc_status(s);
    *term = st != 0;
    *v = st == 2 ? 1.0f : 0.0f;
}

int orc_next_state(const orc_state *s, int move, orc_state *out) {     /* chess.rs:108-146 */
    if (orc_status(s) != 0) return -2;                      /* "Game is already over" */
    uint16_t mv[ORC_MAX_MOVES];
    int n = orc_legal_moves(&s->b, mv), ok = 0;
    for (int i = 0; i < n; ++i) ok |= mv[i] == (uint16_t)move;
    if (!ok) return -1;                                     /* Game::make_move false: "Failed to make move" */
    orc_hist *h = (orc_hist *)arena_alloc(sizeof(orc_hist) + sizeof(uint16_t) * (n > 0 ? n : 1));
    h->prev = s->tt;
    h->n = n;
    memcpy(h->moves, mv, sizeof(uint16_t) * n);
    orc_state r = *s;
    orc_board_make_move(&s->b, move, &r.b);
    r.made = s->made + 1;
    r.tt = h;
    r.n_tt = s->n_tt + 1;
    int src = move & 63, dst = (move >> 6) & 63;
    int reversible = !(s->b.pieces[ORC_PAWN] & BIT(src)) && !(occ_all(&s->b) & BIT(dst)) &&
                     r.b.castle[0] == s->b.castle[0] && r.b.castle[1] == s->b.castle[1];
    r.fifty = reversible ? s->fifty + 1 : 0;
    *out = r;
    return 0;
}

void orc_encoding(const orc_state *s, float *e) {           /* chess.rs:176-249 */
    const orc_board *b = &s->b;
    int me = b->side;
    memset(e, 0, sizeof(float) * ORC_ENC);
    for (int row = 0; row < 8; ++row) {
        int rank = me == ORC_WHITE ? row : 7 - row;
        for (int col = 0; col < 8; ++col) {
            int sq = SQ(rank, col);
            int owner = (b->color[0] & BIT(sq)) ? 0 : (b->color[1] & BIT(sq)) ? 1 : -1;
            if (owner < 0) continue;
            int off = owner == me ? 0 : 6;
            int p = piece_on(b, sq);
            e[(off + p) * 64 + row * 8 + col] = 1.0f;
        }
    }
    float fills[7];
    fills[0] = (b->castle[me] & 1) ? 1.0f : 0.0f;
    fills[1] = (b->castle[me] & 2) ? 1.0f : 0.0f;
    fills[2] = (b->castle[me ^ 1] & 1) ? 1.0f : 0.0f;
    fills[3] = (b->castle[me ^ 1] & 2) ? 1.0f : 0.0f;
    fills[4] = (float)orc_num_repetitions(s);
    fills[5] = (float)s->fifty / 100.0f;
    fills[6] = (float)(s->made / 2) / 50.0f;
    for (int k = 0; k < 7; ++k)
        for (int i = 0; i < 64; ++i) e[(12 + k) * 64 + i] = fills[k];
}

/* Policy::get_channel, chess.rs:311-393 */
int orc_get_channel(int side, int move) {
    int src = move & 63, dst = (move >> 6) & 63, promo = (move >> 12) & 7;
    int rd = (dst >> 3) - (src >> 3), fd = (dst & 7) - (src & 7);
    int ard = rd < 0 ? -rd : rd, afd = fd < 0 ? -fd : fd;
    if (side == ORC_BLACK) rd = -rd;
    int sub = fd + 1;
    if (promo == ORC_ROOK) return 0 + sub;
    if (promo == ORC_BISHOP) return 3 + sub;
    if (promo == ORC_KNIGHT) return 6 + sub;
    if (rd == 0) return fd < 0 ? 9 + (-fd) - 1 : 9 + 7 + fd - 1;
    if (fd == 0) return rd < 0 ? 23 + (-rd) - 1 : 23 + 7 + rd - 1;
    if (ard == afd) {
        if (fd < 0) return rd > 0 ? 37 + rd - 1 : 37 + 7 + (-rd) - 1;
        return rd > 0 ? 37 + 14 + rd - 1 : 37 + 21 + (-rd) - 1;
    }
    if (fd < 0) {
        if (rd > 0) return ard > afd ? 65 : 66;
        return ard > afd ? 67 : 68;
    }
    if (rd > 0) return ard > afd ? 69 : 70;
    return ard > afd ? 71 : 72;
}

int orc_policy_index(int side, int move) {                  /* get_prob / set_prob, chess.rs:497-516 */
    int src = move & 63;
    int row = src >> 3;
    if (side == ORC_BLACK) row = 7 - row;
    return orc_get_channel(side, move) * 64 + row * 8 + (src & 7);
}

/* Policy::get_action, chess.rs:395-493: the knight-underpromotion file
 * difference uses the bishop formula (:442 compares with KNIGHT_MOVE_START_IDX) */
int orc_get_action(int side, int index) {
    int ch = index / 64, row = (index % 64) / 8, col = index % 8;
    int promo = ch < 3 ? ORC_ROOK : ch < 6 ? ORC_BISHOP : ch < 9 ? ORC_KNIGHT : 0;
    int rd, fd;
    if (ch < 9) rd = 1;
    else if (ch < 23) rd = 0;
    else if (ch < 37) rd = (ch - 23 < 7) ? -(ch + 1 - 23) : (ch + 1 - 23 - 7);
    else if (ch < 65) {
        int o = ch - 37;
        rd = o < 7 ? (ch + 1 - 37) : o < 14 ? -(ch + 1 - 37 - 7) : o < 21 ? (ch + 1 - 37 - 14) : -(ch + 1 - 37 - 21);
    } else {
        static const int kr[8] = {2, 1, -2, -1, 2, 1, -2, -1};
        rd = kr[ch - 65];
    }
    if (ch < 9) fd = ch < 3 ? ch - 1 : ch < 65 ? ch - 3 - 1 : ch - 6 - 1;   /* bug: knight promos take ch-4 */
    else if (ch < 23) fd = (ch - 9 < 7) ? -(ch + 1 - 9) : (ch + 1 - 9 - 7);
    else if (ch < 37) fd = 0;
    else if (ch < 65) {
        int o = ch - 37;
        fd = o < 7 ? -(ch + 1 - 37) : o < 14 ? -(ch + 1 - 37 - 7) : o < 21 ? (ch + 1 - 37 - 14) : (ch + 1 - 37 - 21);
    } else {
        static const int kf[8] = {-1, -2, -1, -2, 1, 2, 1, 2};
        fd = kf[ch - 65];
    }
    if (side == ORC_BLACK) {
        rd = -rd;
        row = 7 - row;
    }
    int src = SQ(row, col);
    int dst = SQ((row + rd) & 7, (col + fd) & 7);   /* Rank/File::from_index mask with 7 */
    return orc_move(src, dst, promo);
}

int orc_mask_invalid(const orc_state *s, const float *policy, int len, float *out) {   /* chess.rs:252-275 */
    if (len != ORC_POLICY) return -1;
    float *mask = (float *)calloc(ORC_POLICY, sizeof(float));
    uint16_t mv[ORC_MAX_MOVES];
    int n = orc_legal_moves(&s->b, mv);
    for (int i = 0; i < n; ++i) mask[orc_policy_index(s->b.side, mv[i])] = 1.0f;
    for (int i = 0; i < ORC_POLICY; ++i) out[i] = policy[i] * mask[i];
    float sum = or_nd_sum(out, ORC_POLICY);
    for (int i = 0; i < ORC_POLICY; ++i) out[i] = out[i] / sum;
    free(mask);
    return 0;
}

uint64_t orc_position_key(const orc_state *s) {
    const orc_board *b = &s->b;
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int p = 0; p < 6; ++p) h = or_splitmix64(h ^ b->pieces[p]);
    h = or_splitmix64(h ^ b->color[0]);
    h = or_splitmix64(h ^ ((uint64_t)b->side | (uint64_t)b->castle[0] << 8 | (uint64_t)b->castle[1] << 16 |
                           (uint64_t)b->ep << 24 | (uint64_t)s->fifty << 32 | (uint64_t)(s->made & 0xFFFF) << 48));
    return h;
}

void orc_hash_eval_raw(const orc_state *s, float *raw, float *value) {
    uint64_t key = orc_position_key(s);
    for (int i = 0; i < ORC_POLICY; ++i)
        raw[i] = (float)(1 + (or_splitmix64(key ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull)) & 15));
    *value = (float)((int)((key >> 48) & 255) - 127) / 128.0f;
}

/* ========================================================================
 * MCTS over chess trees, mcts.rs (same structure as spai_oracle.c's)
 * ====================================================================== */
typedef struct {
    orc_state state;
    int parent, action;
    float prior;
    int *children;
    int n_children, cap_children;
    uint32_t visit_count;
    float value_sum;
} orc_node;

struct orc_tree {
    orc_node *arena;
    int size, cap;
    int node_id_to_expand;
};

static int arena_push(orc_tree *t, const orc_node *n) {
    if (t->size == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 256;
        t->arena = (orc_node *)realloc(t->arena, sizeof(orc_node) * t->cap);
    }
    t->arena[t->size] = *n;
    return t->size++;
}

orc_tree *orc_tree_create(void) {
    orc_tree *t = (orc_tree *)calloc(1, sizeof(orc_tree));
    orc_node root;
    memset(&root, 0, sizeof(root));
    orc_state_init(&root.state);
    root.parent = -1;
    root.action = -1;
    root.prior = NAN;
    t->node_id_to_expand = -1;
    arena_push(t, &root);
    return t;
}

/* Tree::with_root_state (mcts.rs:86-89): one root node holding a copy of s
 * (the transposition table is a persistent list, so the copy shares it) */
orc_tree *orc_tree_with_root(const orc_state *s) {
    orc_tree *t = orc_tree_create();
    t->arena[0].state = *s;
    return t;
}

void orc_tree_destroy(orc_tree *t) {
    if (!t) return;
    for (int i = 0; i < t->size; ++i) free(t->arena[i].children);
    free(t->arena);
    free(t);
}

const orc_state *orc_tree_node_state(const orc_tree *t, int id) { return &t->arena[id].state; }
int orc_tree_size(const orc_tree *t) { return t->size; }

static float get_ucb(const orc_tree *t, int pid, int cid, float c) {   /* mcts.rs:91-100 */
    const orc_node *p = &t->arena[pid], *ch = &t->arena[cid];
    float q = ch->visit_count == 0 ? 0.0f : ((-ch->value_sum / (float)ch->visit_count) + 1.0f) / 2.0f;
    float u = c * ch->prior;
    u = u * sqrtf((float)p->visit_count);
    u = u / (1.0f + (float)ch->visit_count);
    return q + u;
}

static int tree_select(const orc_tree *t, int pid, float c, int *err) {   /* :102-114, last max */
    const orc_node *p = &t->arena[pid];
    int best = p->children[0];
    float bu = get_ucb(t, pid, best, c);
    if (isnan(bu)) *err = 1;
    for (int i = 1; i < p->n_children; ++i) {
        float u = get_ucb(t, pid, p->children[i], c);
        if (isnan(u)) *err = 1;
        if (!(u < bu)) { best = p->children[i]; bu = u; }
    }
    return best;
}

static void tree_expand(orc_tree *t, int pid, const float *policy) {   /* :116-143 */
    orc_state ps = t->arena[pid].state;
    uint16_t mv[ORC_MAX_MOVES];
    int n = orc_legal_moves(&ps.b, mv);
    int first = t->size;
    orc_node *p = &t->arena[pid];
    p->children = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    p->cap_children = n;
    p->n_children = n;
    for (int i = 0; i < n; ++i) p->children[i] = first + i;
    for (int i = 0; i < n; ++i) {
        orc_node ch;
        memset(&ch, 0, sizeof(ch));
        orc_next_state(&ps, mv[i], &ch.state);
        ch.parent = pid;
        ch.action = mv[i];
        ch.prior = policy[orc_policy_index(ps.b.side, mv[i])];
        arena_push(t, &ch);
    }
}

static void tree_backprop(orc_tree *t, int id, float value) {   /* :145-159 */
    float sign = 1.0f;
    orc_node *n = &t->arena[id];
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

void orc_tree_use_subtree(orc_tree *t, int new_root_id) {   /* :161-192 */
    orc_node *old = t->arena;
    int old_size = t->size;
    orc_node *queue = (orc_node *)malloc(sizeof(orc_node) * (old_size + 1));
    int qh = 0, qt = 0;
    orc_tree nt = {NULL, 0, 0, t->node_id_to_expand};
    orc_node root = old[new_root_id];
    root.parent = -1;
    queue[qt++] = root;
    int next_id = 0;
    while (qh < qt) {
        orc_node node = queue[qh++];
        for (int i = 0; i < node.n_children; ++i) {
            orc_node ch = old[node.children[i]];
            ch.parent = next_id;
            queue[qt++] = ch;
        }
        node.children = NULL;
        node.n_children = node.cap_children = 0;
        if (node.parent >= 0) {
            orc_node *pp = &nt.arena[node.parent];
            if (pp->n_children == pp->cap_children) {
                pp->cap_children = pp->cap_children ? 2 * pp->cap_children : 8;
                pp->children = (int *)realloc(pp->children, sizeof(int) * pp->cap_children);
            }
            pp->children[pp->n_children++] = next_id;
        }
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

static void hash_eval(int n, const orc_state *const *states, float *priors, float *values) {
    float *raw = (float *)malloc(sizeof(float) * ORC_POLICY);
    for (int i = 0; i < n; ++i) {
        orc_hash_eval_raw(states[i], raw, &values[i]);
        orc_mask_invalid(states[i], raw, ORC_POLICY, priors + (size_t)i * ORC_POLICY);
    }
    free(raw);
}

int orc_search(orc_tree **trees, int n, int num_searches, float c, orc_eval_fn eval, void *user, float *policy,
               int *child_ids, float *child_visits, int *child_moves, int *n_children) {
    if (n <= 0) return 0;
    int *batch = (int *)malloc(sizeof(int) * n);
    const orc_state **states = (const orc_state **)malloc(sizeof(void *) * n);
    float *pri = (float *)malloc(sizeof(float) * (size_t)n * ORC_POLICY);
    float *val = (float *)malloc(sizeof(float) * n);
    int err = 0;
    long evals = 0;
    for (int it = 0; it < num_searches; ++it) {
        int nb = 0;
        for (int ti = 0; ti < n; ++ti) {
            orc_tree *t = trees[ti];
            int node = 0;
            while (t->arena[node].n_children > 0) node = tree_select(t, node, c, &err);
            float v;
            int term;
            orc_value_terminated(&t->arena[node].state, &v, &term);
            if (term) {
                tree_backprop(t, node, v);
                t->node_id_to_expand = -1;
            } else {
                t->node_id_to_expand = node;
                batch[nb++] = ti;
            }
        }
        evals += nb;
        if (nb > 0) {
            for (int k = 0; k < nb; ++k) states[k] = &trees[batch[k]]->arena[trees[batch[k]]->node_id_to_expand].state;
            if (eval) eval(user, nb, states, pri, val);
            else hash_eval(nb, states, pri, val);
            for (int k = 0; k < nb; ++k) {
                orc_tree *t = trees[batch[k]];
                int id = t->node_id_to_expand;
                tree_expand(t, id, pri + (size_t)k * ORC_POLICY);
                tree_backprop(t, id, val[k]);
            }
        }
    }
    for (int ti = 0; ti < n; ++ti) {
        const orc_tree *t = trees[ti];
        const orc_node *root = &t->arena[0];
        float *pol = policy ? policy + (size_t)ti * ORC_POLICY : NULL;
        float *tmp = (float *)calloc(ORC_POLICY, sizeof(float));
        for (int k = 0; k < root->n_children; ++k) {
            const orc_node *ch = &t->arena[root->children[k]];
            float cv = (float)ch->visit_count;
            tmp[orc_policy_index(root->state.b.side, ch->action)] = cv;
            if (child_ids) child_ids[(size_t)ti * ORC_MAX_MOVES + k] = root->children[k];
            if (child_visits) child_visits[(size_t)ti * ORC_MAX_MOVES + k] = cv;
            if (child_moves) child_moves[(size_t)ti * ORC_MAX_MOVES + k] = ch->action;
        }
        if (n_children) n_children[ti] = root->n_children;
        float s = or_nd_sum(tmp, ORC_POLICY);
        if (pol)
            for (int a = 0; a < ORC_POLICY; ++a) pol[a] = tmp[a] / s;
        free(tmp);
    }
    free(batch);
    free(states);
    free(pri);
    free(val);
    return err ? -1 : (int)(evals > 0x7fffffff ? 0x7fffffff : evals);
}

/* SelfPlayWorker::self_play, learner_concurrent.rs:169-242 */
typedef struct {
    orc_tree *tree;
    int index;
    int n_hist, cap_hist;
    orc_state *states;
    float *policies;
} orc_game;

long orc_self_play(int n_games, int num_searches, float c, float temperature, uint64_t seed, uint64_t game_id_base,
                   orc_eval_fn eval, void *user, long cap, float *enc, float *pol, float *val, int32_t *game_ids,
                   int32_t *plies, int max_plies, int32_t *moves, int32_t *n_moves, double *stats) {
    int ng = n_games > 0 ? n_games : 1;
    orc_game *g = (orc_game *)calloc(ng, sizeof(orc_game));
    orc_tree **act = (orc_tree **)malloc(sizeof(void *) * ng);
    int *idx = (int *)malloc(sizeof(int) * ng);
    float *rpol = (float *)malloc(sizeof(float) * (size_t)ORC_POLICY * ng);
    int *rids = (int *)malloc(sizeof(int) * (size_t)ORC_MAX_MOVES * ng);
    float *rvis = (float *)malloc(sizeof(float) * (size_t)ORC_MAX_MOVES * ng);
    int *rnc = (int *)malloc(sizeof(int) * ng);
    long out = 0;
    int n_act = n_games, move_no = 0, rc = 0;
    double sims = 0, evals = 0;
    for (int i = 0; i < n_games; ++i) {
        g[i].tree = orc_tree_create();
        g[i].index = i;
        idx[i] = i;
        if (n_moves) n_moves[i] = 0;
    }
    while (n_act > 0) {
        for (int k = 0; k < n_act; ++k) act[k] = g[idx[k]].tree;
        int ne = orc_search(act, n_act, num_searches, c, eval, user, rpol, rids, rvis, NULL, rnc);
        if (ne < 0) { rc = -3; break; }
        evals += ne;
        sims += (double)n_act * num_searches;
        for (int k = n_act - 1; k >= 0; --k) {
            orc_game *sg = &g[idx[k]];
            orc_tree *t = sg->tree;
            float u = or_u01_f32(seed, game_id_base + (uint64_t)sg->index, (uint64_t)move_no);
            int pick = or_weighted_index(rvis + (size_t)k * ORC_MAX_MOVES, rnc[k], temperature, u);
            if (pick < 0) { rc = -4; goto done; }
            int sel = rids[(size_t)k * ORC_MAX_MOVES + pick];
            if (sg->n_hist == sg->cap_hist) {
                sg->cap_hist = sg->cap_hist ? 2 * sg->cap_hist : 64;
                sg->states = (orc_state *)realloc(sg->states, sizeof(orc_state) * sg->cap_hist);
                sg->policies = (float *)realloc(sg->policies, sizeof(float) * ORC_POLICY * sg->cap_hist);
            }
            sg->states[sg->n_hist] = t->arena[0].state;
            memcpy(sg->policies + (size_t)ORC_POLICY * sg->n_hist, rpol + (size_t)k * ORC_POLICY,
                   sizeof(float) * ORC_POLICY);
            sg->n_hist++;
            if (moves && sg->n_hist <= max_plies)
                moves[(size_t)sg->index * max_plies + sg->n_hist - 1] = t->arena[sel].action;
            if (n_moves) n_moves[sg->index] = sg->n_hist;
            const orc_state *st = &t->arena[sel].state;
            float v;
            int term;
            orc_value_terminated(st, &v, &term);
            if (term) {
                int cur = st->b.side;
                for (int h = 0; h < sg->n_hist; ++h) {
                    if (out < cap) {
                        if (enc) orc_encoding(&sg->states[h], enc + (size_t)out * ORC_ENC);
                        if (pol) memcpy(pol + (size_t)out * ORC_POLICY, sg->policies + (size_t)ORC_POLICY * h,
                                        sizeof(float) * ORC_POLICY);
                        if (val) val[out] = sg->states[h].b.side == cur ? v : -v;
                        if (game_ids) game_ids[out] = sg->index;
                        if (plies) plies[out] = h;
                    }
                    ++out;
                }
                for (int j = k; j < n_act - 1; ++j) idx[j] = idx[j + 1];
                --n_act;
            } else {
                t->node_id_to_expand = -1;
                orc_tree_use_subtree(t, sel);
            }
        }
        ++move_no;
    }
done:
    for (int i = 0; i < n_games; ++i) {
        orc_tree_destroy(g[i].tree);
        free(g[i].states);
        free(g[i].policies);
    }
    if (stats) { stats[0] = sims; stats[1] = evals; }
    free(g); free(act); free(idx); free(rpol); free(rids); free(rvis); free(rnc);
    return rc < 0 ? rc : out;
}

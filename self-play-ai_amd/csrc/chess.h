// chess.h — chess rules for the device engine (and its host helpers).
//
// Reference: game/chess.rs (the adapter over the `chess` crate 3.2.0, which is
// not vendored; its Board::make_move / MoveGen::new_legal semantics are
// restated here) — paths relative to the reference root.
//
// Layout: a position is a 72-byte Board of bitboards (square = rank*8 + file,
// a1 = 0), piece sets in chess::Piece order.  Attacks are computed set-wise with
// Kogge-Stone occluded fills (no lookup tables, so nothing to stage in LDS or
// constant memory): one code path serves a single slider, all sliders of a
// colour at once (the king-danger map) and the x-ray pin probe.
//
// Move generation is wave-parallel (wave_movegen): lane s owns square s, computes
// the legal destinations of the piece standing there, and the move list is laid
// out in the crate's enumeration order (piece type P,N,B,R,Q,K; unpinned sources
// then pinned; en-passant entries after the pawns; destinations ascending;
// promotions Q,N,R,B) by one packed wave prefix sum over the 12 entry groups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SPAI_HD __host__ __device__ __forceinline__

namespace spai {
namespace chess {

typedef uint64_t bb;
enum { PAWN = 0, KNIGHT, BISHOP, ROOK, QUEEN, KING };
enum { WHITE = 0, BLACK = 1 };
constexpr int kNoEp = 64;
constexpr int kMaxMoves = 256;     // >= 218, the most legal moves of any position
constexpr int kPolicy = 4672;      // 73 x 8 x 8 (chess.rs:252-257)
constexpr int kPlanes = 19;        // chess.rs:176-249
constexpr int kInCh = 32;          // device input channels (19 planes, zero padded)

// castle bits: 1 white kingside, 2 white queenside, 4 black kingside, 8 black queenside
struct Board {
    bb pc[6];
    bb col[2];
    uint8_t side, castle, ep, status;   // ep: square of the pawn that just double-pushed (chess::Board::en_passant)
    uint16_t fifty;                     // fifty_move_rule_halfmove_counter (chess.rs:29)
    uint16_t made;                      // Action::MakeMove entries of the Game (chess.rs:243-246)
};
static_assert(sizeof(Board) == 72, "Board is 72 bytes");

constexpr bb kFileA = 0x0101010101010101ull;
constexpr bb kFileH = kFileA << 7;
constexpr bb kRank1 = 0xFFull;

SPAI_HD int lsb(bb x) { return __builtin_ctzll(x); }
SPAI_HD int popc(bb x) { return __builtin_popcountll(x); }
SPAI_HD bb bit(int s) { return 1ull << s; }

// direction d: 0 N, 1 S, 2 E, 3 W, 4 NE, 5 NW, 6 SE, 7 SW (0..3 rook, 4..7 bishop)
SPAI_HD bb shift_dir(bb x, int d) {
    switch (d) {
        case 0: return x << 8;
        case 1: return x >> 8;
        case 2: return (x << 1) & ~kFileA;
        case 3: return (x >> 1) & ~kFileH;
        case 4: return (x << 9) & ~kFileA;
        case 5: return (x << 7) & ~kFileH;
        case 6: return (x >> 7) & ~kFileA;
        default: return (x >> 9) & ~kFileH;
    }
}
SPAI_HD bb wrap_mask(int d) {
    return (d == 2 || d == 4 || d == 6) ? ~kFileA : (d == 3 || d == 5 || d == 7) ? ~kFileH : ~0ull;
}
SPAI_HD bb shift_n(bb x, int d, int n) {   // n steps in direction d, no wrap masking
    const int s = (d == 0) ? 8 : (d == 1) ? -8 : (d == 2) ? 1 : (d == 3) ? -1 : (d == 4) ? 9 : (d == 5) ? 7
                : (d == 6) ? -7 : -9;
    const int k = s * n;
    return k > 0 ? x << k : x >> (-k);
}
// Kogge-Stone occluded fill of `gen` through `empty` in direction d, then one
// more step: the squares the generators attack along d.
SPAI_HD bb ray_attacks(bb gen, bb empty, int d) {
    const bb m = wrap_mask(d);
    bb pro = empty & m;
    gen |= pro & shift_n(gen, d, 1);
    pro &= shift_n(pro, d, 1);
    gen |= pro & shift_n(gen, d, 2);
    pro &= shift_n(pro, d, 2);
    gen |= pro & shift_n(gen, d, 4);
    return shift_dir(gen, d);
}
SPAI_HD bb rook_att(bb gen, bb occ) {
    bb a = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) a |= ray_attacks(gen, ~occ, d);
    return a;
}
SPAI_HD bb bishop_att(bb gen, bb occ) {
    bb a = 0;
#pragma unroll
    for (int d = 4; d < 8; ++d) a |= ray_attacks(gen, ~occ, d);
    return a;
}
SPAI_HD bb knight_att(bb b) {
    const bb l1 = (b >> 1) & ~kFileH, l2 = (b >> 2) & ~(kFileH | (kFileH >> 1));
    const bb r1 = (b << 1) & ~kFileA, r2 = (b << 2) & ~(kFileA | (kFileA << 1));
    const bb h1 = l1 | r1, h2 = l2 | r2;
    return (h1 << 16) | (h1 >> 16) | (h2 << 8) | (h2 >> 8);
}
SPAI_HD bb king_att(bb b) {
    const bb lr = ((b << 1) & ~kFileA) | ((b >> 1) & ~kFileH);
    const bb row = b | lr;
    return lr | (row << 8) | (row >> 8);
}
// squares attacked by pawns of colour c standing on b
SPAI_HD bb pawn_att(bb b, int c) {
    return c == WHITE ? (((b << 7) & ~kFileH) | ((b << 9) & ~kFileA)) : (((b >> 9) & ~kFileH) | ((b >> 7) & ~kFileA));
}
// the whole line through a and b (chess crate `line`), 0 when not aligned
SPAI_HD bb line_through(int a, int b) {
    const int ra = a >> 3, fa = a & 7, rb = b >> 3, fb = b & 7;
    if (a == b) return 0;
    if (ra == rb) return kRank1 << (8 * ra);
    if (fa == fb) return kFileA << fa;
    if (ra - fa == rb - fb) {
        const int d = ra - fa;
        const bb D = 0x8040201008040201ull;
        return d >= 0 ? D << (8 * d) : D >> (-8 * d);
    }
    if (ra + fa == rb + fb) {
        const int d = ra + fa - 7;
        const bb A = 0x0102040810204080ull;
        return d >= 0 ? A << (8 * d) : A >> (-8 * d);
    }
    return 0;
}
// squares strictly between a and b on their line (chess crate `between`)
SPAI_HD bb between(int a, int b) {
    const int lo = a < b ? a : b, hi = a < b ? b : a;
    const bb range = ((1ull << hi) - 1) & ~((2ull << lo) - 1);
    return line_through(a, b) & range;
}
SPAI_HD int piece_on(const Board &b, int s) {
    const bb m = bit(s);
    int p = -1;
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if (b.pc[i] & m) p = i;
    return p;
}
// pc[p] ^= m without a dynamically indexed array (which would live in scratch on the device)
SPAI_HD void xor_piece(Board &b, int p, bb m) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if (i == p) b.pc[i] ^= m;
}
SPAI_HD uint8_t castle_bits(int c, int s) {   // CastleRights::square_to_castle_rights as our bits
    const int r0 = c == WHITE ? 0 : 56, sh = c == WHITE ? 0 : 2;
    if (s == r0) return (uint8_t)(2 << sh);
    if (s == r0 + 4) return (uint8_t)(3 << sh);
    if (s == r0 + 7) return (uint8_t)(1 << sh);
    return 0;
}

SPAI_HD void start_board(Board &b) {
    b.pc[PAWN] = 0x00FF00000000FF00ull;
    b.pc[KNIGHT] = 0x4200000000000042ull;
    b.pc[BISHOP] = 0x2400000000000024ull;
    b.pc[ROOK] = 0x8100000000000081ull;
    b.pc[QUEEN] = 0x0800000000000008ull;
    b.pc[KING] = 0x1000000000000010ull;
    b.col[WHITE] = 0xFFFFull;
    b.col[BLACK] = 0xFFFF000000000000ull;
    b.side = WHITE;
    b.castle = 15;
    b.ep = kNoEp;
    b.status = 0;
    b.fifty = 0;
    b.made = 0;
}

// State::get_next_state (chess.rs:108-146) for a legal move: Board::make_move of
// the crate, then the MakeMove count and the fifty-move counter (reset on a pawn
// move, a capture or any castle-rights change).
SPAI_HD void apply_move(Board &b, int mv) {
    const int src = mv & 63, dst = (mv >> 6) & 63, promo = (mv >> 12) & 7;
    const int c = b.side, o = c ^ 1;
    const bb sb = bit(src), db = bit(dst);
    const int moved = piece_on(b, src);
    const int cap = piece_on(b, dst);
    const uint8_t castle0 = b.castle;
    const int ep0 = b.ep;
    b.ep = kNoEp;
    xor_piece(b, moved, sb | db);
    if (c == WHITE) b.col[WHITE] ^= sb | db;
    else b.col[BLACK] ^= sb | db;
    if (cap >= 0) {
        xor_piece(b, cap, db);
        if (o == WHITE) b.col[WHITE] ^= db;
        else b.col[BLACK] ^= db;
    }
    b.castle &= (uint8_t)~(castle_bits(o, dst) | castle_bits(c, src));
    if (moved == PAWN) {
        if (promo) {
            b.pc[PAWN] ^= db;
            xor_piece(b, promo, db);
        } else if ((sb & 0x00FF00000000FF00ull) && (db & 0x000000FFFF000000ull)) {
            // Board::set_ep: only when an enemy pawn stands beside the destination
            const bb adj = ((db << 1) & ~kFileA) | ((db >> 1) & ~kFileH);
            if (adj & b.pc[PAWN] & (o == WHITE ? b.col[WHITE] : b.col[BLACK])) b.ep = (uint8_t)dst;
        } else if (ep0 != kNoEp && (c == WHITE ? dst - 8 : dst + 8) == ep0) {
            b.pc[PAWN] ^= bit(ep0);
            if (o == WHITE) b.col[WHITE] ^= bit(ep0);
            else b.col[BLACK] ^= bit(ep0);
        }
    } else if (moved == KING && (dst - src == 2 || src - dst == 2)) {
        const int r0 = c == WHITE ? 0 : 56;
        const bb rk = (dst & 7) == 2 ? (bit(r0) | bit(r0 + 3)) : (bit(r0 + 7) | bit(r0 + 5));
        b.pc[ROOK] ^= rk;
        if (c == WHITE) b.col[WHITE] ^= rk;
        else b.col[BLACK] ^= rk;
    }
    const bool reversible = moved != PAWN && cap < 0 && b.castle == castle0;
    b.fifty = reversible ? (uint16_t)(b.fifty + 1) : (uint16_t)0;
    b.made = (uint16_t)(b.made + 1);
    b.side = (uint8_t)o;
}

// Policy::get_channel (chess.rs:311-393); rank differences flipped for Black
SPAI_HD int get_channel(int side, int mv) {
    const int src = mv & 63, dst = (mv >> 6) & 63, promo = (mv >> 12) & 7;
    int rd = (dst >> 3) - (src >> 3);
    const int fd = (dst & 7) - (src & 7);
    const int ard = rd < 0 ? -rd : rd, afd = fd < 0 ? -fd : fd;
    if (side == BLACK) rd = -rd;
    if (promo == ROOK) return fd + 1;
    if (promo == BISHOP) return 3 + fd + 1;
    if (promo == KNIGHT) return 6 + fd + 1;
    if (rd == 0) return fd < 0 ? 8 - fd : 15 + fd;
    if (fd == 0) return rd < 0 ? 22 - rd : 29 + rd;
    if (ard == afd) {
        if (fd < 0) return rd > 0 ? 36 + rd : 43 - rd;
        return rd > 0 ? 50 + rd : 57 - rd;
    }
    if (fd < 0) return rd > 0 ? (ard > afd ? 65 : 66) : (ard > afd ? 67 : 68);
    return rd > 0 ? (ard > afd ? 69 : 70) : (ard > afd ? 71 : 72);
}
// Policy::get_prob / set_prob flat index: channel*64 + row*8 + file, row = rank (7-rank for Black)
SPAI_HD int policy_index(int side, int mv) {
    const int src = mv & 63;
    const int row = side == BLACK ? 7 - (src >> 3) : (src >> 3);
    return get_channel(side, mv) * 64 + row * 8 + (src & 7);
}

// deterministic stub evaluator (oracle/chess_oracle.c orc_position_key / orc_hash_eval_raw)
SPAI_HD uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
SPAI_HD uint64_t position_key(const Board &b) {
    uint64_t h = 0x243F6A8885A308D3ull;
#pragma unroll
    for (int p = 0; p < 6; ++p) h = splitmix(h ^ b.pc[p]);
    h = splitmix(h ^ b.col[WHITE]);
    // the oracle keeps castle rights per colour (bit0 kingside, bit1 queenside)
    const uint64_t cw = b.castle & 3, cb = (b.castle >> 2) & 3;
    return splitmix(h ^ ((uint64_t)b.side | cw << 8 | cb << 16 | (uint64_t)b.ep << 24 | (uint64_t)b.fifty << 32 |
                         (uint64_t)b.made << 48));
}
SPAI_HD float hash_raw(uint64_t key, int index) {
    return (float)(1 + (splitmix(key ^ ((uint64_t)index * 0x9E3779B97F4A7C15ull)) & 15));
}
SPAI_HD float hash_value(uint64_t key) { return (float)((int)((key >> 48) & 255) - 127) / 128.0f; }

// move-list hash: the repetition rule compares whole ordered Vec<ChessMove>
// (chess.rs:51-61); the device compares 64-bit hashes of (index, move) pairs.
SPAI_HD uint64_t move_mix(int index, int mv) { return splitmix(((uint64_t)index << 16) ^ (uint64_t)mv ^ 0x6A09E667F3BCC909ull); }
SPAI_HD uint64_t list_hash(uint64_t sum, int n) { return splitmix(sum ^ ((uint64_t)n << 40) ^ 0xB7E151628AED2A6Bull); }

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ uint64_t wave_or_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
    return x;
}
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(x, o, 64);
        if (lane >= o) x += t;
    }
    return x;
}

struct GenOut {
    int n;            // legal moves
    uint64_t hash;    // list_hash of the ordered list
    bool in_check;
};

// MoveGen::new_legal over one position by one wave (all 64 lanes call it with
// the same board).  Calls visit(index, move) in the lane that generates each
// move (index = its position in the enumeration order, move = src | dst<<6 |
// promo<<12), so callers consume the list without a memory round trip.
template <class F>
__device__ inline GenOut wave_movegen(const Board &b, int lane, F &&visit) {
    const int c = b.side, o = c ^ 1;
    const bb mine = c == WHITE ? b.col[WHITE] : b.col[BLACK], them = c == WHITE ? b.col[BLACK] : b.col[WHITE];
    const bb occ = mine | them;
    const bb kbb = b.pc[KING] & mine;
    const int k = lsb(kbb);
    const bb e_rq = (b.pc[ROOK] | b.pc[QUEEN]) & them, e_bq = (b.pc[BISHOP] | b.pc[QUEEN]) & them;
    // checkers and pinned pieces by rays from the king (uniform across the wave)
    bb checkers = (knight_att(kbb) & b.pc[KNIGHT] & them) | (pawn_att(kbb, c) & b.pc[PAWN] & them);
    bb pinned = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        const bb sl = d < 4 ? e_rq : e_bq;
        const bb first = ray_attacks(kbb, ~occ, d) & occ;
        if (first & sl) checkers |= first;
        else if (first & mine) {
            const bb second = ray_attacks(kbb, ~(occ ^ first), d) & occ & ~first;
            if (second & sl) pinned |= first;
        }
    }
    const int nchk = popc(checkers);
    // king danger: squares the enemy attacks with our king lifted off the board
    const bb occ_nk = occ ^ kbb;
    const bb danger = rook_att(e_rq, occ_nk) | bishop_att(e_bq, occ_nk) | knight_att(b.pc[KNIGHT] & them) |
                      king_att(b.pc[KING] & them) | pawn_att(b.pc[PAWN] & them, o);

    // ---- this lane's square
    const int s = lane;
    const bb sbit = bit(s);
    int group = -1, cnt = 0, epcnt = 0;
    bb dests = 0;
    bool promo = false;
    int ep_dest = -1;
    if (sbit & mine) {
        const int p = piece_on(b, s);
        if (p == KING) {
            dests = king_att(sbit) & ~mine & ~danger;
            if (!checkers) {
                const int r0 = c == WHITE ? 0 : 56;
                const uint8_t kbit = c == WHITE ? 1 : 4, qbit = c == WHITE ? 2 : 8;
                if ((b.castle & kbit) && !(occ & (bit(r0 + 5) | bit(r0 + 6))) && !(danger & (bit(k + 1) | bit(k + 2))))
                    dests |= bit(k + 2);
                if ((b.castle & qbit) && !(occ & (bit(r0 + 1) | bit(r0 + 2) | bit(r0 + 3))) &&
                    !(danger & (bit(k - 1) | bit(k - 2))))
                    dests |= bit(k - 2);
            }
            group = 11;
        } else if (nchk <= 1) {
            const bool pin = (pinned & sbit) != 0;
            bb m;
            if (p == PAWN) {
                const int fwd = c == WHITE ? s + 8 : s - 8;
                m = pawn_att(sbit, c) & them;
                if (!(occ & bit(fwd))) {
                    m |= bit(fwd);
                    const bool start = c == WHITE ? (s >> 3) == 1 : (s >> 3) == 6;
                    const int fwd2 = c == WHITE ? s + 16 : s - 16;
                    if (start && !(occ & bit(fwd2))) m |= bit(fwd2);
                }
                promo = (s >> 3) == (c == WHITE ? 6 : 1);
                // en passant (PawnType::legals, after the pawn entries)
                if (b.ep != kNoEp && (s >> 3) == (b.ep >> 3) && (s == b.ep - 1 || s == b.ep + 1)) {
                    const int dst = c == WHITE ? b.ep + 8 : b.ep - 8;
                    const bb occ2 = occ ^ bit(b.ep) ^ sbit ^ bit(dst);
                    const bool ok = !(rook_att(kbb, occ2) & e_rq) && !(bishop_att(kbb, occ2) & e_bq);
                    if (ok) {
                        epcnt = 1;
                        ep_dest = dst;
                    }
                }
            } else if (p == KNIGHT) {
                m = knight_att(sbit) & ~mine;
            } else if (p == BISHOP) {
                m = bishop_att(sbit, occ) & ~mine;
            } else if (p == ROOK) {
                m = rook_att(sbit, occ) & ~mine;
            } else {
                m = (rook_att(sbit, occ) | bishop_att(sbit, occ)) & ~mine;
            }
            if (nchk == 1) {
                const int cs = lsb(checkers);
                m &= between(cs, k) | checkers;
                if (pin) m = 0;   // the crate skips pinned pieces when in check
            } else if (pin) {
                m &= line_through(k, s);
            }
            dests = m;
            // groups: P 0/1, EP 2, N 3/4, B 5/6, R 7/8, Q 9/10, K 11
            group = p == PAWN ? (pin ? 1 : 0) : 1 + 2 * p + (pin ? 1 : 0);
        }
        cnt = popc(dests) * (promo ? 4 : 1);
        if (cnt == 0) group = -1;
    }
    // one packed exclusive scan over the 12 groups (8-bit fields; a group never
    // holds more than 218 moves): lo = groups 0..7, hi = groups 8..11
    uint64_t lo = 0, hi = 0;
    if (group >= 0) {
        if (group < 8) lo |= (uint64_t)cnt << (8 * group);
        else hi |= (uint64_t)cnt << (8 * (group - 8));
    }
    if (epcnt) lo |= 1ull << 16;   // group 2
    const uint64_t lo_inc = wave_incl_scan_u64(lo, lane), hi_inc = wave_incl_scan_u64(hi, lane);
    const uint64_t lo_tot = __shfl(lo_inc, 63, 64), hi_tot = __shfl(hi_inc, 63, 64);
    const uint64_t lo_exc = lo_inc - lo, hi_exc = hi_inc - hi;
    // group bases (uniform; no dynamically indexed arrays, which would spill to scratch)
    int my_base = 0, ep_base = 0, n = 0;
#pragma unroll
    for (int g = 0; g < 12; ++g) {
        const int tot = (int)((g < 8 ? (lo_tot >> (8 * g)) : (hi_tot >> (8 * (g - 8)))) & 255);
        if (g < group) my_base += tot;
        if (g < 2) ep_base += tot;
        n += tot;
    }
    uint64_t hsum = 0;
    if (group >= 0) {
        int off = my_base + (int)((group < 8 ? (lo_exc >> (8 * group)) : (hi_exc >> (8 * (group - 8)))) & 255);
        const int PROMO[4] = {QUEEN, KNIGHT, ROOK, BISHOP};
        for (bb d = dests; d; d &= d - 1) {
            const int dst = lsb(d);
            if (promo) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int mv = s | (dst << 6) | (PROMO[i] << 12);
                    visit(off, mv);
                    hsum += move_mix(off, mv);
                    ++off;
                }
            } else {
                const int mv = s | (dst << 6);
                visit(off, mv);
                hsum += move_mix(off, mv);
                ++off;
            }
        }
    }
    if (epcnt) {
        const int off = ep_base + (int)((lo_exc >> 16) & 255);
        const int mv = s | (ep_dest << 6);
        visit(off, mv);
        hsum += move_mix(off, mv);
    }
    GenOut r;
    r.n = n;
    r.hash = list_hash(wave_sum_u64(hsum), n);
    r.in_check = checkers != 0;
    return r;
}
// writes the ordered list to out[0..n) when out is non-null
__device__ inline GenOut wave_movegen(const Board &b, uint16_t *out, int lane) {
    return wave_movegen(b, lane, [&](int off, int mv) {
        if (out) out[off] = (uint16_t)mv;
    });
}

}  // namespace chess
}  // namespace spai

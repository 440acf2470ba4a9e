// chess_search.hip — Tree + Mcts::search (mcts.rs:32-332) and
// SelfPlayWorker::self_play (learner_concurrent.rs:169-242) over chess trees
// held in HBM.
//
// Per search iteration (all trees of the call, one wavefront per tree / leaf):
//   k_cleaf   PUCT descent (mcts.rs:235-243; ties -> last child, quirk Q2), the
//             leaf position replayed from the root along the chosen moves, its
//             legal moves (wave_movegen), repetition count against the game's
//             transposition table + the path's nodes, status (chess.rs:150-174).
//             Terminal -> backprop at once (value +1 on checkmate, quirk Q7);
//             else -> a batch slot with the leaf's net input planes.
//   forward   k_chess_forward over the slots (chess_net.hip), or a stub
//   k_cexpand softmax over the 4672 logits, mask to the legal moves, renormalize
//             (Model::predict, model/mod.rs:62-93), children in MoveGen order
//             (mcts.rs:116-143), backprop (mcts.rs:145-159).
// Node ids are per-tree handles into one half of a two-half arena; when the
// active half could overflow during the next search, k_ccompact copies the
// root's subtree depth-first into the other half (Tree::use_subtree's copy,
// mcts.rs:161-192, done only when needed; the root keeps N and W, quirk Q4).
#include <algorithm>
#include <chrono>
#include <memory>
#include <cmath>
#include <cstring>

#include "chess_engine.h"
#include "philox.h"

namespace spai {
namespace chess {
namespace {

constexpr int kWavesPerBlock = 4;
constexpr uint32_t kErrNan = 1, kErrDepth = 2, kErrCap = 4, kErrHist = 8;
constexpr int kMaxChildren = 218;   // most legal moves of any chess position

struct TV {
    uint4 *nodes;
    uint32_t *first;
    uint64_t *nhash;
    uint32_t *root, *fill, *half;
    Board *root_board;
    uint32_t *root_reps;
    uint64_t *hist;
    uint32_t *hist_n;
    uint32_t max_hist;
    uint32_t *path, *depth;
    uint16_t *leaf_moves;
    uint32_t *leaf_n;
    uint64_t *leaf_hash, *leaf_key;
    uint32_t cap;
};

struct BV {
    uint32_t *tree;
    uint16_t *x;
    float *logits, *value;
};

__device__ __forceinline__ size_t tbase(const TV &T, uint32_t t) {
    return (size_t)t * 2 * T.cap + (size_t)T.half[t] * T.cap;
}

// mcts.rs:91-100 in the reference's operation order (-ffp-contract=off)
__device__ __forceinline__ float ucb(float sq_parent, const uint4 &ch, float c) {
    const uint32_t n = ch.x;
    const float w = __uint_as_float(ch.y), prior = __uint_as_float(ch.z);
    const float q = n == 0 ? 0.0f : ((-w / (float)n) + 1.0f) / 2.0f;
    float u = c * prior;
    u = u * sq_parent;
    u = u / (1.0f + (float)n);
    return q + u;
}

__device__ __forceinline__ void backup(const TV &T, size_t base, const uint32_t *path, int d, float v, int lane) {
    for (int lvl = lane; lvl <= d; lvl += 64) {
        uint32_t *nd = (uint32_t *)(T.nodes + base + path[lvl]);
        const float sign = ((d - lvl) & 1) ? -1.0f : 1.0f;
        nd[0] = nd[0] + 1u;
        nd[1] = __float_as_uint(__uint_as_float(nd[1]) + sign * v);
    }
}

__global__ __launch_bounds__(64 * kWavesPerBlock) void k_cleaf(TV T, BV B, const uint32_t *__restrict__ active,
                                                              uint32_t n_active, float c, uint32_t *count,
                                                              uint32_t *err) {
    __shared__ uint32_t spath[kWavesPerBlock][kMaxDepth];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t gi = blockIdx.x * kWavesPerBlock + w;
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    const size_t base = tbase(T, t);
    uint32_t *path = spath[w];
    Board b = T.root_board[t];
    uint32_t node = T.root[t];
    int d = 0;
    if (lane == 0) path[0] = node;
    for (;;) {
        const uint4 rec = T.nodes[base + node];
        const uint32_t nch = rec.w >> 16;
        if (nch == 0) break;   // while node.is_fully_expanded()
        const uint32_t f = T.first[base + node];
        const float sq = sqrtf((float)rec.x);
        float bu = -INFINITY;
        int bi = -1;
        bool nan = false;
        for (uint32_t i = lane; i < nch; i += 64) {
            const float u = ucb(sq, T.nodes[base + f + i], c);
            nan |= u != u;
            if (!(u < bu)) {   // later children win ties (Iterator::max_by, mcts.rs:110-113)
                bu = u;
                bi = (int)i;
            }
        }
        // a NaN on any child panics in the reference (mcts.rs:106-109): stop the
        // whole wave before the argmax so its lanes never walk different children
        if (__ballot(nan)) {
            if (lane == 0) atomicOr(err, kErrNan);
            return;
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            const float ou = __shfl_xor(bu, m, 64);
            const int oi = __shfl_xor(bi, m, 64);
            if (oi >= 0 && (bi < 0 || ou > bu || (ou == bu && oi > bi))) {
                bu = ou;
                bi = oi;
            }
        }
        node = f + (uint32_t)bi;
        apply_move(b, (int)(T.nodes[base + node].w & 0xFFFFu));
        ++d;
        if (d >= kMaxDepth) {
            if (lane == 0) atomicOr(err, kErrDepth);
            return;
        }
        if (lane == 0) path[d] = node;
    }
    __builtin_amdgcn_wave_barrier();
    // the leaf: legal moves, repetition count, status (chess.rs:51-61,150-174)
    const GenOut g = wave_movegen(b, T.leaf_moves + (size_t)t * kMaxMoves, lane);
    uint32_t hits = 0;
    const uint64_t *hist = T.hist + (size_t)t * T.max_hist;
    const uint32_t hn = T.hist_n[t];
    for (uint32_t i = lane; i < hn; i += 64) hits += hist[i] == g.hash;
    for (int j = lane; j < d; j += 64) hits += T.nhash[base + path[j]] == g.hash;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hits += __shfl_xor(hits, o, 64);
    const uint32_t reps = 1 + hits;
    int status = SPAI_ONGOING;
    if (g.n == 0) status = g.in_check ? SPAI_WON : SPAI_TIED;
    else if (reps >= 3 || b.fifty >= 100) status = SPAI_TIED;
    if (status != SPAI_ONGOING) {
        backup(T, base, path, d, status == SPAI_WON ? 1.0f : 0.0f, lane);
        return;
    }
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(count, 1u);
    slot = __shfl(slot, 0, 64);
    if (lane == 0) {
        B.tree[slot] = t;
        T.depth[t] = (uint32_t)d;
        T.leaf_n[t] = (uint32_t)g.n;
        T.leaf_hash[t] = g.hash;
        T.leaf_key[t] = position_key(b);
    }
    for (int j = lane; j <= d; j += 64) T.path[(size_t)t * kMaxDepth + j] = path[j];
    // net input: lane = cell of the side to move's view, 19 planes (chess.rs:176-249) as bf16
    {
        const int me = b.side;
        const int row = lane >> 3, col = lane & 7;
        const int sq = (me == WHITE ? row : 7 - row) * 8 + col;
        const bb mine = me == WHITE ? b.col[WHITE] : b.col[BLACK];
        const bb theirs = me == WHITE ? b.col[BLACK] : b.col[WHITE];
        float v[kInCh];
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            v[p] = ((b.pc[p] & mine) >> sq) & 1 ? 1.0f : 0.0f;
            v[6 + p] = ((b.pc[p] & theirs) >> sq) & 1 ? 1.0f : 0.0f;
        }
        const int ck = me == WHITE ? 1 : 4, cq = me == WHITE ? 2 : 8, tk = me == WHITE ? 4 : 1,
                  tq = me == WHITE ? 8 : 2;
        v[12] = (b.castle & ck) ? 1.0f : 0.0f;
        v[13] = (b.castle & cq) ? 1.0f : 0.0f;
        v[14] = (b.castle & tk) ? 1.0f : 0.0f;
        v[15] = (b.castle & tq) ? 1.0f : 0.0f;
        v[16] = (float)reps;
        v[17] = (float)b.fifty / 100.0f;
        v[18] = (float)(b.made / 2) / 50.0f;
#pragma unroll
        for (int p = kPlanes; p < kInCh; ++p) v[p] = 0.0f;
        uint32_t pk[kInCh / 2];
#pragma unroll
        for (int p = 0; p < kInCh / 2; ++p)
            pk[p] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2 * p]) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v[2 * p + 1]) << 16);
        uint4 *dst = (uint4 *)(B.x + ((size_t)slot * 64 + lane) * kInCh);
#pragma unroll
        for (int k = 0; k < kInCh / 8; ++k) dst[k] = make_uint4(pk[4 * k], pk[4 * k + 1], pk[4 * k + 2], pk[4 * k + 3]);
    }
}

// expand + backprop of each evaluated leaf (mcts.rs:255-283), one wave per slot
__global__ __launch_bounds__(64 * kWavesPerBlock) void k_cexpand(TV T, BV B, uint32_t max_n,
                                                                const uint32_t *__restrict__ count, int eval_kind,
                                                                uint32_t *err) {
    const int lane = threadIdx.x & 63;
    const uint32_t s = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (s >= min(*count, max_n)) return;
    const uint32_t t = B.tree[s];
    const size_t base = tbase(T, t);
    const int d = (int)T.depth[t];
    const uint32_t *path = T.path + (size_t)t * kMaxDepth;
    const uint32_t leaf = path[d];
    const int n = (int)T.leaf_n[t];
    const uint16_t *mv = T.leaf_moves + (size_t)t * kMaxMoves;
    const int side = T.root_board[t].side ^ (d & 1);
    // per-lane legal moves j = lane + 64k (k < 4, n <= 218)
    float p[4];
    float msum = 0.0f;
    float v;
    if (eval_kind == SPAI_EVAL_NET) {
        // softmax over the whole policy (model/mod.rs:63), then mask + renormalize
        const float *lg = B.logits + (size_t)s * kPolicy;
        float mx = -INFINITY;
        for (int i = lane; i < kPolicy; i += 64) mx = fmaxf(mx, lg[i]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float se = 0.0f;
        for (int i = lane; i < kPolicy; i += 64) se += expf(lg[i] - mx);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = lane + 64 * k;
            p[k] = j < n ? expf(lg[policy_index(side, mv[j])] - mx) / se : 0.0f;
            msum += p[k];
        }
        v = B.value[s];
    } else {
        const uint64_t key = T.leaf_key[t];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int j = lane + 64 * k;
            p[k] = j < n ? (eval_kind == SPAI_EVAL_HASH ? hash_raw(key, policy_index(side, mv[j])) : 1.0f) : 0.0f;
            msum += p[k];   // small integers: exact in any order
        }
        v = eval_kind == SPAI_EVAL_HASH ? hash_value(key) : 0.0f;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) msum += __shfl_xor(msum, o, 64);
    const uint32_t first = T.fill[t];
    if (first + (uint32_t)n > T.cap) {
        if (lane == 0) atomicOr(err, kErrCap);
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = lane + 64 * k;
        if (j < n) {
            T.nodes[base + first + j] = make_uint4(0u, 0u, __float_as_uint(p[k] / msum), (uint32_t)mv[j]);
            T.first[base + first + j] = kNone;
        }
    }
    if (lane == 0) {
        T.fill[t] = first + (uint32_t)n;
        uint32_t *lr = (uint32_t *)(T.nodes + base + leaf);
        lr[3] = (lr[3] & 0xFFFFu) | ((uint32_t)n << 16);
        T.first[base + leaf] = first;
        T.nhash[base + leaf] = T.leaf_hash[t];
    }
    backup(T, base, path, d, v, lane);
}

// copy the root's subtree depth-first into the other half when the active half
// could overflow during a search adding up to `need` nodes
__global__ __launch_bounds__(64 * kWavesPerBlock) void k_ccompact(TV T, const uint32_t *__restrict__ active,
                                                                 uint32_t n_active, uint32_t need, uint32_t *err) {
    __shared__ uint4 stack[kWavesPerBlock][kMaxDepth];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t gi = blockIdx.x * kWavesPerBlock + w;
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    if (T.fill[t] + need <= T.cap) return;
    const uint32_t h = T.half[t];
    const size_t ob = (size_t)t * 2 * T.cap + (size_t)h * T.cap, nb = (size_t)t * 2 * T.cap + (size_t)(h ^ 1) * T.cap;
    const uint32_t r = T.root[t];
    const uint4 rr = T.nodes[ob + r];
    if (lane == 0) {
        T.nodes[nb] = rr;
        T.nhash[nb] = T.nhash[ob + r];
    }
    uint32_t tail = 1;
    uint32_t of = 0, nf = 0, nch = rr.w >> 16, i = 0;   // current frame
    int sp = 0;
    auto copy_block = [&](uint32_t from, uint32_t to, uint32_t cnt) {
        for (uint32_t k = lane; k < cnt; k += 64) {
            T.nodes[nb + to + k] = T.nodes[ob + from + k];
            T.nhash[nb + to + k] = T.nhash[ob + from + k];
            T.first[nb + to + k] = kNone;
        }
    };
    if (nch) {
        of = T.first[ob + r];
        nf = tail;
        copy_block(of, nf, nch);
        if (lane == 0) T.first[nb] = nf;
        tail += nch;
    } else if (lane == 0) {
        T.first[nb] = kNone;
    }
    while (nch) {
        if (i == nch) {   // frame done: pop
            if (sp == 0) break;
            --sp;
            __builtin_amdgcn_wave_barrier();
            const uint4 fr = stack[w][sp];
            of = fr.x;
            nf = fr.y;
            nch = fr.z;
            i = fr.w;
            continue;
        }
        const uint32_t oc = of + i, nc = nf + i;
        ++i;
        const uint4 cr = T.nodes[ob + oc];
        const uint32_t cn = cr.w >> 16;
        if (!cn) continue;
        if (tail + cn > T.cap || sp + 1 >= kMaxDepth) {
            if (lane == 0) atomicOr(err, kErrCap);
            return;
        }
        const uint32_t cf = T.first[ob + oc];
        copy_block(cf, tail, cn);
        if (lane == 0) {
            T.first[nb + nc] = tail;
            stack[w][sp] = make_uint4(of, nf, nch, i);
        }
        __builtin_amdgcn_wave_barrier();
        ++sp;
        of = cf;
        nf = tail;
        nch = cn;
        i = 0;
        tail += cn;
    }
    if (lane == 0) {
        T.root[t] = 0;
        T.fill[t] = tail;
        T.half[t] = h ^ 1;
    }
}

// every tree t < n (list null), or the n trees list[i], as a one-node tree at the start position
__global__ void k_ctrees_init(TV T, uint32_t n, const uint32_t *__restrict__ list) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = list ? list[i] : i;
    const size_t base = (size_t)t * 2 * T.cap;
    T.nodes[base] = make_uint4(0u, 0u, 0u, 0u);
    T.first[base] = kNone;
    T.nhash[base] = 0;
    T.root[t] = 0;
    T.fill[t] = 1;
    T.half[t] = 0;
    Board b;
    start_board(b);
    T.root_board[t] = b;
    T.root_reps[t] = 1;
    T.hist_n[t] = 0;
}

// Tree::with_root_state (mcts.rs:86-89) for the state held in game slot `slot`:
// a one-node tree whose root is that board, with the slot's history of earlier
// positions (their move-list hashes) as the tree's, and its repetition count and
// status.  One wave.
__global__ void k_ctree_from_slot(TV T, uint32_t t, const Board *__restrict__ boards,
                                  const uint64_t *__restrict__ shist, const uint32_t *__restrict__ sn_hist,
                                  uint32_t smax_hist, uint32_t slot, uint32_t *err) {
    const int lane = threadIdx.x;
    Board b = boards[slot];
    const uint32_t nh = sn_hist[slot];
    if (nh > T.max_hist) {
        if (lane == 0) atomicOr(err, kErrHist);
        return;
    }
    const uint64_t *src = shist + (size_t)slot * smax_hist;
    uint64_t *dst = T.hist + (size_t)t * T.max_hist;
    const GenOut g = wave_movegen(b, nullptr, lane);
    uint32_t hits = 0;
    for (uint32_t i = lane; i < nh; i += 64) {
        const uint64_t h = src[i];
        dst[i] = h;
        hits += h == g.hash;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hits += __shfl_xor(hits, o, 64);
    const uint32_t reps = 1 + hits;
    int status = SPAI_ONGOING;
    if (g.n == 0) status = g.in_check ? SPAI_WON : SPAI_TIED;
    else if (reps >= 3 || b.fifty >= 100) status = SPAI_TIED;
    b.status = (uint8_t)status;
    if (lane == 0) {
        const size_t base = (size_t)t * 2 * T.cap;
        T.nodes[base] = make_uint4(0u, 0u, 0u, 0u);
        T.first[base] = kNone;
        T.nhash[base] = 0;
        T.root[t] = 0;
        T.fill[t] = 1;
        T.half[t] = 0;
        T.root_board[t] = b;
        T.root_reps[t] = reps;
        T.hist_n[t] = nh;
    }
}

// root children after a search (mcts.rs:310-331): n_children, visits, moves, ids
__global__ void k_croot_stats(TV T, const uint32_t *__restrict__ active, uint32_t n_active, uint32_t *nch_out,
                              uint32_t *vis_out, uint16_t *mv_out, uint32_t *id_out) {
    const int lane = threadIdx.x & 63;
    const uint32_t gi = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    const size_t base = tbase(T, t);
    const uint32_t r = T.root[t];
    const uint32_t nch = T.nodes[base + r].w >> 16;
    const uint32_t f = nch ? T.first[base + r] : 0;
    if (lane == 0) nch_out[gi] = nch;
    for (uint32_t i = lane; i < kMaxMoves; i += 64) {
        const bool ok = i < nch;
        const uint4 cr = ok ? T.nodes[base + f + i] : make_uint4(0, 0, 0, 0);
        vis_out[(size_t)gi * kMaxMoves + i] = cr.x;
        mv_out[(size_t)gi * kMaxMoves + i] = (uint16_t)(cr.w & 0xFFFFu);
        id_out[(size_t)gi * kMaxMoves + i] = ok ? f + i : kNone;
    }
}

// Tree::use_subtree(child) + the sampled child's get_value_and_terminated
// (learner_concurrent.rs:194-197,234): the root's list hash joins the game's
// transposition table, the child becomes the root (keeping N and W).
// out[gi] = status | reps << 8; boards[gi] = the new root position.
__global__ void k_cadvance(TV T, const uint32_t *__restrict__ active, uint32_t n_active,
                           const uint32_t *__restrict__ pick, uint32_t *out, Board *boards, uint32_t *err) {
    const int lane = threadIdx.x & 63;
    const uint32_t gi = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    const size_t base = tbase(T, t);
    const uint32_t r = T.root[t];
    const uint32_t child = T.first[base + r] + pick[gi];
    Board b = T.root_board[t];
    const uint64_t rh = T.nhash[base + r];
    const uint32_t hn = T.hist_n[t];
    if (hn >= T.max_hist) {
        if (lane == 0) atomicOr(err, kErrHist);
        return;
    }
    apply_move(b, (int)(T.nodes[base + child].w & 0xFFFFu));
    const GenOut g = wave_movegen(b, nullptr, lane);
    const uint64_t *hist = T.hist + (size_t)t * T.max_hist;
    uint32_t hits = lane == 0 && rh == g.hash ? 1u : 0u;
    for (uint32_t i = lane; i < hn; i += 64) hits += hist[i] == g.hash;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) hits += __shfl_xor(hits, o, 64);
    const uint32_t reps = 1 + hits;
    int status = SPAI_ONGOING;
    if (g.n == 0) status = g.in_check ? SPAI_WON : SPAI_TIED;
    else if (reps >= 3 || b.fifty >= 100) status = SPAI_TIED;
    b.status = (uint8_t)status;
    if (lane == 0) {
        T.hist[(size_t)t * T.max_hist + hn] = rh;
        T.hist_n[t] = hn + 1;
        T.root[t] = child;
        T.root_board[t] = b;
        T.root_reps[t] = reps;
        out[gi] = (uint32_t)status | (reps << 8);
        boards[gi] = b;
    }
}

TV view(spai_chess *e) {
    Trees &Tr = e->trees;
    TV T;
    T.nodes = Tr.nodes.p;
    T.first = Tr.first.p;
    T.nhash = Tr.nhash.p;
    T.root = Tr.root.p;
    T.fill = Tr.fill.p;
    T.half = Tr.half.p;
    T.root_board = Tr.root_board.p;
    T.root_reps = Tr.root_reps.p;
    T.hist = Tr.hist.p;
    T.hist_n = Tr.hist_n.p;
    T.max_hist = Tr.max_hist;
    T.path = Tr.path.p;
    T.depth = Tr.depth.p;
    T.leaf_moves = Tr.leaf_moves.p;
    T.leaf_n = Tr.leaf_n.p;
    T.leaf_hash = Tr.leaf_hash.p;
    T.leaf_key = Tr.leaf_key.p;
    T.cap = Tr.cap;
    return T;
}

BV bview(spai_chess *e) {
    BV B;
    B.tree = e->batch.tree.p;
    B.x = e->batch.x.p;
    B.logits = e->batch.logits.p;
    B.value = e->batch.value.p;
    return B;
}

uint32_t blocks_for(uint32_t n) { return (n + kWavesPerBlock - 1) / kWavesPerBlock; }

int check_err(spai_chess *e) {
    uint32_t f = 0;
    SPAI_HIP(hipMemcpyAsync(&f, e->err.p, 4, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    if (!f) return SPAI_OK;
    SPAI_HIP(hipMemsetAsync(e->err.p, 0, 4, e->stream));
    if (f & kErrNan) {
        set_error("NaN UCB score (the reference panics in partial_cmp().unwrap(), mcts.rs:106-109)");
        return SPAI_ERR_NAN;
    }
    if (f & kErrDepth) {
        set_error("selection path deeper than %d", kMaxDepth);
        return SPAI_ERR_CAPACITY;
    }
    if (f & kErrHist) {
        set_error("game longer than cfg.max_moves (%u)", e->trees.max_hist);
        return SPAI_ERR_CAPACITY;
    }
    set_error("node arena full (%u nodes per half)", e->trees.cap);
    return SPAI_ERR_CAPACITY;
}

// timing: sampled launches bracketed by events on the engine stream
struct Timing {
    std::vector<hipEvent_t> ev;
    std::vector<int> which;
    size_t used = 0;
};

}  // namespace

int trees_create(spai_chess *e, uint32_t n) {
    Trees &T = e->trees;
    SPAI_CHECK(n >= 1 && n <= e->cfg.max_trees, SPAI_ERR_INVALID, "trees: n=%u (max_trees %u)", n, e->cfg.max_trees);
    const uint64_t cap = std::max<uint64_t>(4ull * e->cfg.num_searches * kMaxChildren, 1u << 14);
    SPAI_CHECK(cap < (1ull << 31), SPAI_ERR_CAPACITY, "arena too large");
    if (T.n != n || T.cap != cap) {
        T.cap = (uint32_t)cap;
        T.n = n;
        T.max_hist = e->cfg.max_moves;
        SPAI_TRY(T.nodes.alloc((size_t)n * 2 * cap));
        SPAI_TRY(T.first.alloc((size_t)n * 2 * cap));
        SPAI_TRY(T.nhash.alloc((size_t)n * 2 * cap));
        SPAI_TRY(T.root.alloc(n));
        SPAI_TRY(T.fill.alloc(n));
        SPAI_TRY(T.half.alloc(n));
        SPAI_TRY(T.root_board.alloc(n));
        SPAI_TRY(T.root_reps.alloc(n));
        SPAI_TRY(T.hist.alloc((size_t)n * T.max_hist));
        SPAI_TRY(T.hist_n.alloc(n));
        SPAI_TRY(T.path.alloc((size_t)n * kMaxDepth));
        SPAI_TRY(T.depth.alloc(n));
        SPAI_TRY(T.leaf_moves.alloc((size_t)n * kMaxMoves));
        SPAI_TRY(T.leaf_n.alloc(n));
        SPAI_TRY(T.leaf_hash.alloc(n));
        SPAI_TRY(T.leaf_key.alloc(n));
        SPAI_TRY(T.st_nch.alloc(n));
        SPAI_TRY(T.st_visits.alloc((size_t)n * kMaxMoves));
        SPAI_TRY(T.st_ids.alloc((size_t)n * kMaxMoves));
        SPAI_TRY(T.st_moves.alloc((size_t)n * kMaxMoves));
        SPAI_TRY(T.adv_pick.alloc(n));
        SPAI_TRY(T.adv_out.alloc(n));
        SPAI_TRY(T.adv_board.alloc(n));
        Batch &B = e->batch;
        B.cap = n;
        SPAI_TRY(B.tree.alloc(n));
        SPAI_TRY(B.x.alloc((size_t)n * 64 * kInCh));
        SPAI_TRY(B.logits.alloc((size_t)n * kPolicy));
        SPAI_TRY(B.value.alloc(n));
        SPAI_TRY(e->active.alloc(n));
    }
    k_ctrees_init<<<(n + 255) / 256, 256, 0, e->stream>>>(view(e), n, nullptr);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

namespace {
int run_search(spai_chess *e, uint32_t na, uint32_t sims, double *evals_out) {
    Trees &Tr = e->trees;
    Batch &B = e->batch;
    if (B.counts.n < sims) SPAI_TRY(B.counts.alloc(sims));
    SPAI_HIP(hipMemsetAsync(B.counts.p, 0, sizeof(uint32_t) * sims, e->stream));
    const TV T = view(e);
    const BV BVv = bview(e);
    const int kind = (int)e->cfg.eval;
    SPAI_CHECK(kind != SPAI_EVAL_NET || e->net, SPAI_ERR_INVALID, "cfg.eval = NET but no net set (spai_chess_set_net)");
    k_ccompact<<<blocks_for(na), 64 * kWavesPerBlock, 0, e->stream>>>(T, e->active.p, na, sims * kMaxChildren,
                                                                      e->err.p);
    SPAI_HIP(hipGetLastError());
    KernelTimer &tm = e->timer;
    auto stamp = [&](int which, bool begin) -> int {
        if (tm.used >= tm.ev.size()) {
            hipEvent_t ev;
            SPAI_HIP(hipEventCreate(&ev));
            tm.ev.push_back(ev);
        }
        SPAI_HIP(hipEventRecord(tm.ev[tm.used++], e->stream));
        if (begin) tm.which.push_back(which);
        return SPAI_OK;
    };
    for (uint32_t it = 0; it < sims; ++it) {
        const bool timed = tm.enabled && (it % 8 == 0);
        uint32_t *cnt = B.counts.p + it;
        if (timed) SPAI_TRY(stamp(0, true));
        k_cleaf<<<blocks_for(na), 64 * kWavesPerBlock, 0, e->stream>>>(T, BVv, e->active.p, na, e->cfg.c, cnt,
                                                                       e->err.p);
        SPAI_HIP(hipGetLastError());
        if (timed) SPAI_TRY(stamp(0, false));
        if (kind == SPAI_EVAL_NET) {
            if (timed) SPAI_TRY(stamp(1, true));
            SPAI_TRY(net_eval(e->net, e->stream, cnt, na, B.x.p, B.logits.p, B.value.p));
            if (timed) SPAI_TRY(stamp(1, false));
        }
        if (timed) SPAI_TRY(stamp(2, true));
        k_cexpand<<<blocks_for(na), 64 * kWavesPerBlock, 0, e->stream>>>(T, BVv, na, cnt, kind, e->err.p);
        SPAI_HIP(hipGetLastError());
        if (timed) SPAI_TRY(stamp(2, false));
    }
    std::vector<uint32_t> counts(sims);
    SPAI_HIP(hipMemcpyAsync(counts.data(), B.counts.p, 4 * sims, hipMemcpyDeviceToHost, e->stream));
    SPAI_TRY(check_err(e));
    double ev = 0;
    for (uint32_t c : counts) ev += c;
    if (evals_out) *evals_out = ev;
    // per-kernel sampled times (event pairs in launch order)
    if (tm.enabled) {
        for (size_t k = 0; k + 1 < tm.used; k += 2) {
            float ms = 0;
            SPAI_HIP(hipEventElapsedTime(&ms, tm.ev[k], tm.ev[k + 1]));
            const int which = tm.which[k / 2];
            tm.total_ms[which] += ms;
            tm.launches[which] += 1;
        }
        // items: trees for select/expand, leaves for the forward (exact per iteration)
        for (uint32_t it = 0; it < sims; it += 8) {
            tm.items[0] += na;
            tm.items[1] += counts[it];
            tm.items[2] += counts[it];
        }
        tm.used = 0;
        tm.which.clear();
    }
    (void)Tr;
    return SPAI_OK;
}

int root_stats(spai_chess *e, uint32_t na) {
    Trees &Tr = e->trees;
    k_croot_stats<<<blocks_for(na), 64 * kWavesPerBlock, 0, e->stream>>>(view(e), e->active.p, na, Tr.st_nch.p,
                                                                         Tr.st_visits.p, Tr.st_moves.p, Tr.st_ids.p);
    SPAI_HIP(hipGetLastError());
    Tr.h_nch.resize(na);
    Tr.h_visits.resize((size_t)na * kMaxMoves);
    Tr.h_moves.resize((size_t)na * kMaxMoves);
    Tr.h_ids.resize((size_t)na * kMaxMoves);
    SPAI_HIP(hipMemcpyAsync(Tr.h_nch.data(), Tr.st_nch.p, 4 * na, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(Tr.h_visits.data(), Tr.st_visits.p, 4ull * na * kMaxMoves, hipMemcpyDeviceToHost,
                            e->stream));
    SPAI_HIP(hipMemcpyAsync(Tr.h_moves.data(), Tr.st_moves.p, 2ull * na * kMaxMoves, hipMemcpyDeviceToHost,
                            e->stream));
    SPAI_HIP(hipMemcpyAsync(Tr.h_ids.data(), Tr.st_ids.p, 4ull * na * kMaxMoves, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

// visit-count policy of a root (mcts.rs:318-328): set_prob(action, N), normalize
void dense_policy(int side, uint32_t nch, const uint32_t *vis, const uint16_t *mv, float *pol) {
    std::fill(pol, pol + kPolicy, 0.0f);
    float tot = 0.0f;
    for (uint32_t k = 0; k < nch; ++k) tot += (float)vis[k];   // integers < 2^24: exact in any order
    for (uint32_t k = 0; k < nch; ++k) pol[policy_index(side, mv[k])] = (float)vis[k];
    for (int i = 0; i < kPolicy; ++i) pol[i] = pol[i] / tot;
}
}  // namespace

int search(spai_chess *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
           uint32_t *child_ids, float *child_visits, uint16_t *child_moves, uint32_t *n_children, double *evals) {
    Trees &Tr = e->trees;
    SPAI_CHECK(Tr.n > 0, SPAI_ERR_INVALID, "no trees (spai_chess_trees_create)");
    SPAI_CHECK(n >= 1 && n <= Tr.n, SPAI_ERR_INVALID, "search: n=%u trees (have %u)", n, Tr.n);
    SPAI_CHECK(num_searches <= e->cfg.num_searches, SPAI_ERR_INVALID,
               "num_searches %u > cfg.num_searches %u (sizes the arena)", num_searches, e->cfg.num_searches);
    for (uint32_t i = 0; i < n; ++i)
        SPAI_CHECK(tree_idx[i] < Tr.n, SPAI_ERR_INVALID, "tree index %u out of range", tree_idx[i]);
    SPAI_HIP(hipMemcpyAsync(e->active.p, tree_idx, 4 * n, hipMemcpyHostToDevice, e->stream));
    SPAI_TRY(run_search(e, n, num_searches, evals));
    SPAI_TRY(root_stats(e, n));
    std::vector<Board> rb(Tr.n);
    SPAI_HIP(hipMemcpy(rb.data(), Tr.root_board.p, sizeof(Board) * Tr.n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t nch = Tr.h_nch[i];
        const uint32_t *vis = Tr.h_visits.data() + (size_t)i * kMaxMoves;
        const uint16_t *mv = Tr.h_moves.data() + (size_t)i * kMaxMoves;
        if (n_children) n_children[i] = nch;
        for (uint32_t k = 0; k < (uint32_t)kMaxMoves; ++k) {
            if (child_ids) child_ids[(size_t)i * kMaxMoves + k] = Tr.h_ids[(size_t)i * kMaxMoves + k];
            if (child_visits) child_visits[(size_t)i * kMaxMoves + k] = (float)vis[k];
            if (child_moves) child_moves[(size_t)i * kMaxMoves + k] = mv[k];
        }
        if (policy) dense_policy(rb[tree_idx[i]].side, nch, vis, mv, policy + (size_t)i * kPolicy);
    }
    return SPAI_OK;
}

int tree_reset_from_slot(spai_chess *e, uint32_t tree, uint32_t slot) {
    Trees &Tr = e->trees;
    SPAI_CHECK(tree < Tr.n, SPAI_ERR_INVALID, "tree %u out of range (%u trees)", tree, Tr.n);
    SPAI_CHECK(slot < e->slots.n, SPAI_ERR_INVALID, "slot %u out of range (%u slots)", slot, e->slots.n);
    k_ctree_from_slot<<<1, 64, 0, e->stream>>>(view(e), tree, e->slots.board.p, e->slots.hist.p, e->slots.n_hist.p,
                                               e->slots.max_hist, slot, e->err.p);
    SPAI_HIP(hipGetLastError());
    return check_err(e);
}

int tree_use_subtree(spai_chess *e, uint32_t tree, uint32_t child_index) {
    Trees &Tr = e->trees;
    SPAI_CHECK(tree < Tr.n, SPAI_ERR_INVALID, "tree %u out of range", tree);
    SPAI_HIP(hipMemcpyAsync(e->active.p, &tree, 4, hipMemcpyHostToDevice, e->stream));
    SPAI_TRY(root_stats(e, 1));
    SPAI_CHECK(child_index < Tr.h_nch[0], SPAI_ERR_INVALID, "child index %u >= %u root children", child_index,
               Tr.h_nch[0]);
    SPAI_HIP(hipMemcpyAsync(Tr.adv_pick.p, &child_index, 4, hipMemcpyHostToDevice, e->stream));
    k_cadvance<<<1, 64 * kWavesPerBlock, 0, e->stream>>>(view(e), e->active.p, 1, Tr.adv_pick.p, Tr.adv_out.p,
                                                         Tr.adv_board.p, e->err.p);
    SPAI_HIP(hipGetLastError());
    return check_err(e);
}

int trees_advance(spai_chess *e, uint32_t n, const uint32_t *tree_idx, const uint32_t *child_index, uint8_t *status,
                  uint32_t *reps) {
    Trees &Tr = e->trees;
    SPAI_CHECK(n >= 1 && n <= Tr.n, SPAI_ERR_INVALID, "advance: n=%u trees (have %u)", n, Tr.n);
    for (uint32_t i = 0; i < n; ++i)
        SPAI_CHECK(tree_idx[i] < Tr.n, SPAI_ERR_INVALID, "tree index %u out of range", tree_idx[i]);
    SPAI_HIP(hipMemcpyAsync(e->active.p, tree_idx, 4 * n, hipMemcpyHostToDevice, e->stream));
    SPAI_TRY(root_stats(e, n));
    for (uint32_t i = 0; i < n; ++i)
        SPAI_CHECK(child_index[i] < Tr.h_nch[i], SPAI_ERR_INVALID, "tree %u: child index %u >= %u root children",
                   tree_idx[i], child_index[i], Tr.h_nch[i]);
    SPAI_HIP(hipMemcpyAsync(Tr.adv_pick.p, child_index, 4 * n, hipMemcpyHostToDevice, e->stream));
    k_cadvance<<<blocks_for(n), 64 * kWavesPerBlock, 0, e->stream>>>(view(e), e->active.p, n, Tr.adv_pick.p,
                                                                     Tr.adv_out.p, Tr.adv_board.p, e->err.p);
    SPAI_HIP(hipGetLastError());
    std::vector<uint32_t> out(n);
    SPAI_HIP(hipMemcpyAsync(out.data(), Tr.adv_out.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_TRY(check_err(e));
    for (uint32_t i = 0; i < n; ++i) {
        if (status) status[i] = (uint8_t)(out[i] & 0xFF);
        if (reps) reps[i] = out[i] >> 8;
    }
    return SPAI_OK;
}

int tree_root(spai_chess *e, uint32_t tree, spai_chess_state *root, uint32_t *visits, float *value_sum) {
    Trees &Tr = e->trees;
    SPAI_CHECK(tree < Tr.n, SPAI_ERR_INVALID, "tree %u out of range", tree);
    uint32_t r = 0, h = 0, reps = 0;
    Board b;
    SPAI_HIP(hipMemcpy(&r, Tr.root.p + tree, 4, hipMemcpyDeviceToHost));
    SPAI_HIP(hipMemcpy(&h, Tr.half.p + tree, 4, hipMemcpyDeviceToHost));
    SPAI_HIP(hipMemcpy(&reps, Tr.root_reps.p + tree, 4, hipMemcpyDeviceToHost));
    SPAI_HIP(hipMemcpy(&b, Tr.root_board.p + tree, sizeof(Board), hipMemcpyDeviceToHost));
    uint4 rec;
    SPAI_HIP(hipMemcpy(&rec, Tr.nodes.p + (size_t)tree * 2 * Tr.cap + (size_t)h * Tr.cap + r, 16,
                       hipMemcpyDeviceToHost));
    if (root) *root = to_abi(b, reps);
    if (visits) *visits = rec.x;
    if (value_sum) memcpy(value_sum, &rec.y, 4);
    return SPAI_OK;
}

// SelfPlayWorker::self_play (learner_concurrent.rs:169-242).  window < n_games
// (spai_chess_selfplay_stream): the games run through `window` tree slots, a slot
// whose game ended taking the next game (a fresh start-position tree) before the
// next search; each game's draws are keyed by its id and its own move number, so
// every game is the one the lockstep run plays.
int selfplay_run(spai_chess *e, uint32_t n_games, uint64_t gid_base, spai_chess_sample_sink sink, void *user,
                 spai_selfplay_stats *stats, uint32_t window) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t W = (window == 0 || window >= n_games) ? n_games : window;   // tree slots
    SPAI_CHECK(n_games >= 1 && W <= e->cfg.max_trees, SPAI_ERR_INVALID, "%u tree slots (max_trees %u)", W,
               e->cfg.max_trees);
    SPAI_TRY(trees_create(e, W));
    Trees &Tr = e->trees;
    const uint32_t sims = e->cfg.num_searches;
    std::vector<uint32_t> slot_game(W), slot_move(W, 0);   // each slot's game (index < n_games) and its move number
    for (uint32_t i = 0; i < W; ++i) slot_game[i] = i;
    uint32_t next_game = W;
    std::vector<uint32_t> refill;
    struct Rec {
        Board board;
        uint32_t reps;
        uint16_t move;
        std::vector<uint32_t> vis;
        std::vector<uint16_t> mv;
    };
    std::vector<std::vector<Rec>> hist(W);
    std::vector<uint32_t> act(W);
    for (uint32_t i = 0; i < W; ++i) act[i] = i;
    std::vector<Board> roots(W);
    std::vector<uint32_t> root_reps(W, 1);
    for (auto &b : roots) start_board(b);
    double sims_done = 0, evals = 0, games = 0, positions = 0, moves = 0;
    uint64_t move_no = 0;
    std::vector<uint32_t> pick;
    std::vector<uint32_t> out;
    std::vector<Board> nb;
    std::vector<float> enc, pol, val;
    std::vector<uint16_t> mvs;
    // optional per-move trace (diagnostics): SPAI_TRACE_MOVES=<csv path>, lines of
    // move, active games, leaves evaluated, seconds (search + root statistics)
    std::unique_ptr<FILE, int (*)(FILE *)> trace(nullptr, &std::fclose);
    if (const char *tp = std::getenv("SPAI_TRACE_MOVES")) trace.reset(std::fopen(tp, "a"));
    while (!act.empty()) {
        const uint32_t na = (uint32_t)act.size();
        const auto tm0 = std::chrono::steady_clock::now();
        SPAI_HIP(hipMemcpyAsync(e->active.p, act.data(), 4 * na, hipMemcpyHostToDevice, e->stream));
        double ev = 0;
        SPAI_TRY(run_search(e, na, sims, &ev));
        SPAI_TRY(root_stats(e, na));
        if (trace)
            std::fprintf(trace.get(), "%llu,%u,%.0f,%.6f\n", (unsigned long long)move_no, na, ev,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - tm0).count());
        evals += ev;
        sims_done += (double)na * sims;
        moves += 1;
        pick.assign(na, 0);
        for (int k = (int)na - 1; k >= 0; --k) {   // for i in (0..trees_vec.len()).rev()
            const uint32_t t = act[k];
            const uint32_t nch = Tr.h_nch[k];
            const uint32_t *vis = Tr.h_visits.data() + (size_t)k * kMaxMoves;
            float fv[kMaxMoves];
            for (uint32_t j = 0; j < nch; ++j) fv[j] = (float)vis[j];
            const float u = sample_u01_f32(e->cfg.seed, gid_base + slot_game[t], slot_move[t]++);
            const int idx = weighted_index(fv, (int)nch, e->cfg.temperature, u);
            SPAI_CHECK(idx >= 0, SPAI_ERR_NAN, "WeightedIndex over all-zero visits (the reference panics)");
            pick[k] = (uint32_t)idx;
            Rec r;
            r.board = roots[t];
            r.reps = root_reps[t];
            r.move = Tr.h_moves[(size_t)k * kMaxMoves + idx];
            r.vis.assign(vis, vis + nch);
            r.mv.assign(Tr.h_moves.data() + (size_t)k * kMaxMoves, Tr.h_moves.data() + (size_t)k * kMaxMoves + nch);
            hist[t].push_back(std::move(r));
        }
        SPAI_HIP(hipMemcpyAsync(Tr.adv_pick.p, pick.data(), 4 * na, hipMemcpyHostToDevice, e->stream));
        k_cadvance<<<blocks_for(na), 64 * kWavesPerBlock, 0, e->stream>>>(view(e), e->active.p, na, Tr.adv_pick.p,
                                                                          Tr.adv_out.p, Tr.adv_board.p, e->err.p);
        SPAI_HIP(hipGetLastError());
        out.resize(na);
        nb.resize(na);
        SPAI_HIP(hipMemcpyAsync(out.data(), Tr.adv_out.p, 4 * na, hipMemcpyDeviceToHost, e->stream));
        SPAI_HIP(hipMemcpyAsync(nb.data(), Tr.adv_board.p, sizeof(Board) * na, hipMemcpyDeviceToHost, e->stream));
        SPAI_TRY(check_err(e));
        std::vector<uint32_t> keep;
        keep.reserve(na);
        std::vector<char> done(na, 0);
        for (int k = (int)na - 1; k >= 0; --k) {
            const uint32_t t = act[k];
            const int status = (int)(out[k] & 0xFF);
            roots[t] = nb[k];
            root_reps[t] = out[k] >> 8;
            if (status == SPAI_ONGOING) continue;
            done[k] = 1;
            // emit (learner_concurrent.rs:200-230): value of the terminal child
            // signed by each recorded position's player to move
            const float v = status == SPAI_WON ? 1.0f : 0.0f;
            const int cur = nb[k].side;
            const std::vector<Rec> &H = hist[t];
            const size_t m = H.size();
            positions += (double)m;
            games += 1;
            if (sink) {
                enc.assign(m * kPlanes * 64, 0.f);
                pol.assign(m * kPolicy, 0.f);
                val.resize(m);
                mvs.resize(m);
                for (size_t h = 0; h < m; ++h) {
                    encode_host(H[h].board, H[h].reps, enc.data() + h * kPlanes * 64);
                    dense_policy(H[h].board.side, (uint32_t)H[h].vis.size(), H[h].vis.data(), H[h].mv.data(),
                                 pol.data() + h * kPolicy);
                    val[h] = H[h].board.side == cur ? v : -v;
                    mvs[h] = H[h].move;
                }
                sink(user, (uint32_t)(gid_base + slot_game[t]), (uint32_t)m, enc.data(), pol.data(), val.data(),
                     mvs.data());
            }
            hist[t].clear();
            hist[t].shrink_to_fit();
        }
        for (uint32_t k = 0; k < na; ++k)
            if (!done[k]) keep.push_back(act[k]);
        // streaming: the slots whose game ended take the next games (appended)
        refill.clear();
        for (uint32_t k = 0; k < na && next_game < n_games; ++k)
            if (done[k]) {
                const uint32_t t = act[k];
                refill.push_back(t);
                slot_game[t] = next_game++;
                slot_move[t] = 0;
                start_board(roots[t]);
                root_reps[t] = 1;
                keep.push_back(t);
            }
        if (!refill.empty()) {
            const uint32_t nr = (uint32_t)refill.size();
            SPAI_HIP(hipMemcpyAsync(e->active.p, refill.data(), 4 * nr, hipMemcpyHostToDevice, e->stream));
            k_ctrees_init<<<(nr + 255) / 256, 256, 0, e->stream>>>(view(e), nr, e->active.p);
            SPAI_HIP(hipGetLastError());
        }
        act.swap(keep);
        ++move_no;
    }
    if (stats) {
        stats->sims = sims_done;
        stats->evals = evals;
        stats->games = games;
        stats->positions = positions;
        stats->moves = moves;
        stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return SPAI_OK;
}

}  // namespace chess
}  // namespace spai

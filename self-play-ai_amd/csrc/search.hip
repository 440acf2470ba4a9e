// search.hip — device-resident MCTS (mcts.rs) + the self-play driver
// (learner_concurrent.rs:169-242).
//
// Trees live in HBM as per-tree arenas of 16-B node records (spai_internal.h).
// One search iteration (mcts.rs:214-285) is two launches per search chain:
//   evaluate        the fused ResNet forward (net_c4.hip) or a stub evaluator
//                   over this iteration's leaf batch;
//   k_expand_select per tree, 8 lanes (one per board column): expand the tree's
//                   leaf of this iteration if it had one (legal moves by
//                   ballot, children packed by a prefix count, priors written,
//                   value backed up along the recorded path, lanes splitting
//                   the levels), then the NEXT iteration's PUCT descent from
//                   the root (state replayed on bitboards, leaf terminal check;
//                   terminal leaves backed up in place, live leaves appended to
//                   the next batch).
// Trees are independent, so expanding tree t and selecting tree t again in one
// launch is the reference's per-tree order (expand+backprop of iteration i,
// then select of i+1) and the results are those of separate launches; the
// fusion removes one kernel boundary from every iteration's critical path.
// The first iteration starts with k_select alone, the last ends with k_expand.
// Leaf batches are double-buffered by iteration parity, and every iteration
// has its own slot counter (zeroed once per search call).
// The host only sees the trees between moves: root visit counts come back once
// per search call.  In self-play the move is sampled on the device too
// (k_advance), which writes the sampled child as the new root.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "philox.h"
#include "spai_internal.h"

namespace spai {
namespace {

constexpr int kLanesPerTree = 8;
#ifndef SPAI_TREE_BLOCK
#define SPAI_TREE_BLOCK 64
#endif
constexpr int kBlock = SPAI_TREE_BLOCK;   // threads per tree-kernel workgroup (kBlock / 8 trees)
constexpr int kTreesPerBlock = kBlock / kLanesPerTree;
constexpr uint32_t kErrNan = 1u, kErrCapacity = 2u, kErrDepth = 4u;

struct TreeView {
    uint4 *nodes;
    uint32_t cap;
    const uint32_t *root;
    uint32_t *next_free;
    const uint64_t *root_x, *root_o;
    const uint8_t *root_n, *root_status;
    uint32_t *path;
    uint8_t *depth;
    uint32_t *slot;   // the tree's leaf slot in the current batch, kNoSlot if terminal
    uint32_t *left;   // tail run-on mode: search iterations the tree still has to run
    uint32_t *evals;  // live leaves of this search call (the tail-mode policy's input)
};
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

struct BatchView {
    uint32_t *count;
    uint32_t *more;   // tail mode: set when a tree stopped at the run cap with iterations left (else null)
    uint32_t *tree;
    uint64_t *mine, *theirs;
    float *priors;
    float *value;
};

// PUCT score, mcts.rs:91-100, evaluated in the reference's operation order
// (no contraction: built with -ffp-contract=off; sqrt and / correctly rounded).
// sqrt_np = sqrtf(parent visits), computed while the children's records load.
// The quotient is computed for every child and selected (an unvisited child has
// q = 0): under a branch the compiler sank the load of the record's value sum
// into it, which put a second dependent memory round trip on every level.
__device__ __forceinline__ float ucb(float sqrt_np, const uint4 &ch, float c) {
    const uint32_t n = ch.x;
    const float w = __uint_as_float(ch.y), prior = __uint_as_float(ch.z);
    const float qv = ((-w / (float)(n == 0 ? 1u : n)) + 1.0f) / 2.0f;
    const float q = n == 0 ? 0.0f : qv;
    float u = c * prior;
    u = u * sqrt_np;
    u = u / (1.0f + (float)n);
    return q + u;
}

// backprop (mcts.rs:145-159) over path[0..d]: level d is the leaf (+v), signs
// alternate upward; lane l of the 8-lane group updates the levels == l (mod 8)
// (at most kMaxDepth / 8 = 6 per lane).  The nodes of a path are distinct, so a
// lane loads all of its levels' records first and then stores them: one memory
// round trip, where a load-add-store per level (the compiler cannot reorder a
// level's load above the previous level's store) paid one per level.
constexpr int kLevelsPerLane = kMaxDepth / kLanesPerTree;
// (The loads are unconditional -- levels past d read the path's root, whose node
// exists -- so that no branch separates them: hipcc waits vmcnt(0) at each one.)
__device__ __forceinline__ void backup_load(const uint4 *nodes, const uint32_t (&node)[kLevelsPerLane], int d,
                                            int lane8, uint2 (&r)[kLevelsPerLane]) {
#pragma unroll
    for (int j = 0; j < kLevelsPerLane; ++j) r[j] = *(const uint2 *)(nodes + (lane8 + 8 * j <= d ? node[j] : node[0]));
}
__device__ __forceinline__ void backup_store(uint4 *nodes, const uint32_t (&node)[kLevelsPerLane], int d, float v,
                                             int lane8, const uint2 (&r)[kLevelsPerLane]) {
#pragma unroll
    for (int j = 0; j < kLevelsPerLane; ++j) {
        const int lvl = lane8 + 8 * j;
        if (lvl <= d) {
            const float sign = ((d - lvl) & 1) ? -1.0f : 1.0f;
            *(uint2 *)(nodes + node[j]) = make_uint2(r[j].x + 1u, __float_as_uint(__uint_as_float(r[j].y) + sign * v));
        }
    }
}
__device__ __forceinline__ void backup_nodes(uint4 *nodes, const uint32_t (&node)[kLevelsPerLane], int d, float v,
                                             int lane8) {
    uint2 r[kLevelsPerLane];
    backup_load(nodes, node, d, lane8, r);
    backup_store(nodes, node, d, v, lane8, r);
}

// this lane's bit of its tree's 8-lane group in a wave-wide ballot
__device__ __forceinline__ uint32_t group_bits(uint64_t ball) {
    return (uint32_t)(ball >> (threadIdx.x & 63 & ~(kLanesPerTree - 1))) & 0xFFu;
}

// has_line without the early exits (no branch on the descent's chain)
__device__ __forceinline__ bool has_line_flat(uint64_t b) {
    const uint64_t h = b & (b >> 7), v = b & (b >> 1), g = b & (b >> 8);
    return ((h & (h >> 14)) | (v & (v >> 2)) | (g & (g >> 16))) != 0ull;
}

// A non-NaN score as an unsigned key in the same order, -0 and +0 equal (the
// reference compares f32 with partial_cmp, where they tie).
__device__ __forceinline__ uint32_t score_key(float u) {
    const uint32_t b = __float_as_uint(u + 0.0f);   // -0 + 0 = +0 (not folded: signed zeros are kept)
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// a tree's best child so far in the argmax over its 8 lanes: the 64-bit key
// (score, then column: ties go to the last child, i.e. the highest column) with
// the child index in the key's low bits, and the child record's visit count and
// children word (what the next level needs)
struct Cand {
    uint32_t hi, lo, n, w;
};
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// one butterfly step: take the partner lane's candidate if its key is larger
template <int CTRL>
__device__ __forceinline__ void cand_step(Cand &c) {
    const Cand o{dpp_mov<CTRL>(c.hi), dpp_mov<CTRL>(c.lo), dpp_mov<CTRL>(c.n), dpp_mov<CTRL>(c.w)};
    const bool take = (((uint64_t)o.hi << 32) | o.lo) > (((uint64_t)c.hi << 32) | c.lo);
    c.hi = take ? o.hi : c.hi;
    c.lo = take ? o.lo : c.lo;
    c.n = take ? o.n : c.n;
    c.w = take ? o.w : c.w;
}

// a tree's root for this search call: node id and position (constant while it
// runs), and its record's visit count and children word, kept current in
// registers (each iteration's backup adds one visit; an expansion of the root
// sets its children), so a descent starts without reloading it
struct RootInfo {
    uint32_t node;
    uint64_t x, o;
    uint8_t n, status;
    uint32_t rn, rw;
};
__device__ __forceinline__ RootInfo load_root(const TreeView &T, uint32_t t) {
    const uint32_t node = T.root[t];
    const uint4 r = T.nodes[(size_t)t * T.cap + node];
    return RootInfo{node, T.root_x[t], T.root_o[t], T.root_n[t], T.root_status[t], r.x, r.w};
}

// One PUCT descent of tree t (mcts.rs:235-250) by its 8 lanes.  A terminal leaf
// is backed up in place (mcts.rs:245-247) and kTerminal returned; a live leaf is
// returned as kLive with its position in (x, o, n) and its path recorded (T.path,
// T.depth); kError after a NaN UCB or an over-deep path (flag set in err).
//
// Lane c of the tree's 8 stands for board column c: a node's children are its
// position's open columns in ascending order (expand_leaf), so column c's child
// is number popcount(open columns below c).  Per level: one 16-B record load,
// the UCB, and the argmax with ties to the LAST child (Iterator::max_by,
// mcts.rs:110-113) as a butterfly of DPP moves over the 8 lanes on a 64-bit key
// (score, column), carrying the child index, visit count and children word --
// no lane shuffle through the LDS crossbar and no branch on the chain.
enum Descent { kTerminal = 0, kLive = 1, kError = 2 };
__device__ __forceinline__ Descent descend(const TreeView &T, uint32_t t, const RootInfo &root, int lane8, float c,
                                           uint32_t *err, uint64_t &x, uint64_t &o, uint8_t &n) {
    uint4 *nodes = T.nodes + (size_t)t * T.cap;
    uint32_t *path = T.path + (size_t)t * kMaxDepth;
    uint32_t node = root.node;
    x = root.x;
    o = root.o;
    n = root.n;
    uint8_t status = root.status;
    uint32_t rn = root.rn, rw = root.rw;   // the current node's visit count and children word
    // path levels == lane8 (mod 8) kept in this lane's registers (kMaxDepth = 6 x 8)
    uint32_t pr[kLevelsPerLane] = {node, 0u, 0u, 0u, 0u, 0u};
    const int top = 7 * lane8 + 5;   // this column's top cell (lane 7: none)
    int d = 0;
    if (lane8 == 0) path[0] = node;
    while (rw != kNoChildren) {                             // while node.is_fully_expanded()
        const uint32_t first = rw & 0xFFFFFFu;
        const uint64_t occ = x | o;
        const bool open = lane8 < c4::kActions && !((occ >> top) & 1ull);
        const uint32_t k = c4::popc32(group_bits(__ballot(open)) & ((1u << lane8) - 1u));
        const uint4 ch = nodes[first + (open ? k : 0u)];
        const float sq = sqrtf((float)rn);
        const float u = ucb(sq, ch, c);
        Cand w{open ? score_key(u) : 0u, ((uint32_t)lane8 << 3) | k, ch.x, ch.w};
        cand_step<0xB1>(w);    // quad_perm [1,0,3,2]: lane ^ 1
        cand_step<0x4E>(w);    // quad_perm [2,3,0,1]: lane ^ 2
        cand_step<0x141>(w);   // row_half_mirror: lane i <-> 7 - i of the 8, across the two quads
        // a NaN on ANY child panics in the reference (partial_cmp().unwrap(),
        // mcts.rs:106-109): OR over the tree's 8 lanes and stop the whole group,
        // so lanes never split onto different children.  Tested after the argmax
        // (whose result is then dropped): before it, the branch made the compiler
        // split the record load and sink the children word's half past it.
        if (group_bits(__ballot(open && u != u))) {
            if (lane8 == 0) atomicOr(err, kErrNan);
            return kError;
        }
        rn = w.n;
        rw = w.w;
        // replay the child's action on the bitboards
        const int a = (int)(w.lo >> 3);
        const uint64_t bit = c4::drop_bit(occ, a);
        const bool xm = c4::x_to_move(n);
        x = xm ? x | bit : x;
        o = xm ? o : o | bit;
        n = (uint8_t)(n + 1);
        status = has_line_flat(xm ? x : o) ? c4::kWon : (n == c4::kCells ? c4::kTied : c4::kOngoing);
        node = first + (w.lo & 7u);
        ++d;
        if (d >= kMaxDepth) {
            if (lane8 == 0) atomicOr(err, kErrDepth);
            return kError;
        }
        const bool mine = (d & 7) == lane8;
        if (mine) path[d] = node;
#pragma unroll
        for (int j = 0; j < kLevelsPerLane; ++j) pr[j] = mine && (d >> 3) == j ? node : pr[j];
    }
    if (lane8 == 0) T.depth[t] = (uint8_t)d;
    if (status != c4::kOngoing) {                           // terminal leaf: backprop(leaf, value), mcts.rs:245-247
        backup_nodes(nodes, pr, d, c4::terminal_value(status), lane8);
        return kTerminal;
    }
    return kLive;
}

// live leaf -> batch slot (mcts.rs:249-250)
__device__ __forceinline__ void slot_leaf(const TreeView &T, const BatchView &B, uint32_t t, int lane8, uint64_t x,
                                          uint64_t o, uint8_t n) {
    if (lane8 == 0) {
        const uint32_t slot = atomicAdd(B.count, 1u);
        __hip_atomic_fetch_add(T.evals + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // result unused: no wait
        const bool xm = c4::x_to_move(n);
        T.slot[t] = slot;
        B.tree[slot] = t;
        B.mine[slot] = xm ? x : o;
        B.theirs[slot] = xm ? o : x;
    }
}

// One search iteration's selection for tree t: a live leaf gets a slot in batch
// B (recorded in T.slot[t]), a terminal leaf is backed up in place.
//
// RUN_ON (tail mode, search()): the tree runs its remaining iterations (T.left)
// in this launch for as long as they end on terminal leaves -- each is backed
// up, then the next descent starts -- and stops at the first live leaf, which
// goes to the batch, or after run_cap descents (B.more set: the next pass goes
// on).  The tree's iterations keep the reference's order (select, backprop,
// select, ...), so the results equal one descent per launch.  The cap keeps a
// pass from lasting a solved tree's whole run while a tree that still evaluates
// waits for the next one.
template <bool RUN_ON>
__device__ __forceinline__ void select_tree(const TreeView &T, const BatchView &B, uint32_t t, RootInfo &root,
                                            int lane8, float c, uint32_t *err, uint32_t run_cap) {
    if (lane8 == 0) T.slot[t] = kNoSlot;
    uint64_t x, o;
    uint8_t n;
    if (!RUN_ON) {
        if (descend(T, t, root, lane8, c, err, x, o, n) == kLive) slot_leaf(T, B, t, lane8, x, o, n);
        return;
    }
    uint32_t left = T.left[t];
    for (uint32_t run = 0; left > 0; ++run) {
        if (run == run_cap) {
            if (lane8 == 0) atomicOr(B.more, 1u);
            break;
        }
        --left;
        const Descent r = descend(T, t, root, lane8, c, err, x, o, n);
        if (r == kLive) slot_leaf(T, B, t, lane8, x, o, n);
        if (r != kTerminal) break;
        root.rn += 1;   // the backup's visit of the root
        // the next descent reads records the other lanes of this tree just backed
        // up: one wave, so a wavefront-scope fence (as in k_expand_select)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane8 == 0) T.left[t] = left;
}

// What an expansion needs of the tree itself (not of its leaf): loaded with the
// tree's slot, before the slot is known to hold a leaf.
struct LeafPath {
    int d;                                 // the leaf's depth
    uint32_t lv[kLevelsPerLane];           // this lane's path levels (stale past the depth)
    uint32_t first;                        // the arena fill: the new children's first id
};
__device__ __forceinline__ LeafPath load_leaf_path(const TreeView &T, uint32_t t, int lane8) {
    LeafPath L;
    const uint32_t *path = T.path + (size_t)t * kMaxDepth;
    L.d = T.depth[t];
#pragma unroll
    for (int j = 0; j < kLevelsPerLane; ++j) L.lv[j] = path[lane8 + 8 * j];
    L.first = T.next_free[t];
    return L;
}

// expand leaf slot s of batch B (mcts.rs:116-143) and back its value up (:145-159).
// One memory round trip after the slot: the leaf's position, this lane's prior
// and the value, together with the records of the path levels this lane backs up
// (the new children are past the arena fill, never on the path); then only
// stores.  The leaf is path[d], which lane d & 7 holds.  The root's visit count
// and children word in `root` are brought up to date.
__device__ __forceinline__ void expand_leaf(const TreeView &T, const BatchView &B, uint32_t t, uint32_t s, int lane8,
                                            uint32_t *err, const LeafPath &L, RootInfo &root) {
    uint4 *nodes = T.nodes + (size_t)t * T.cap;
    const int d = L.d;
    uint32_t node[kLevelsPerLane];   // this lane's levels of the path; 0 (a valid dummy) past the depth
#pragma unroll
    for (int j = 0; j < kLevelsPerLane; ++j) node[j] = lane8 + 8 * j <= d ? L.lv[j] : 0u;
    const uint64_t occ = B.mine[s] | B.theirs[s];
    const float prior = B.priors[(size_t)s * kPriorStride + lane8];   // lane 7: the stride's padding
    const float value = B.value[s];
    uint2 r[kLevelsPerLane];
    backup_load(nodes, node, d, lane8, r);
    // legal actions of the (live) leaf; children in ascending action order (mcts.rs:116-143)
    const bool legal = lane8 < c4::kActions && !((occ >> (7 * lane8 + 5)) & 1ull);
    const uint32_t grp = group_bits(__ballot(legal));
    const uint32_t nch = c4::popc32(grp);
    const uint32_t idx = c4::popc32(grp & ((1u << lane8) - 1u));
    const uint32_t first = L.first;
    if (first + nch > T.cap) {
        if (lane8 == 0) atomicOr(err, kErrCapacity);
        return;
    }
    if (legal) nodes[first + idx] = make_uint4(0u, 0u, __float_as_uint(prior), kNoChildren);
    if (lane8 == 0) T.next_free[t] = first + nch;
    if (lane8 == (d & 7)) {
        uint32_t leaf = node[0];
#pragma unroll
        for (int j = 1; j < kLevelsPerLane; ++j) leaf = (d >> 3) == j ? node[j] : leaf;
        nodes[leaf].w = first | (nch << 24);
    }
    backup_store(nodes, node, d, value, lane8, r);
    root.rn += 1;
    if (d == 0) root.rw = first | (nch << 24);
}

template <bool RUN_ON>
__global__ __launch_bounds__(kBlock) void k_select(TreeView T, BatchView B, const uint32_t *__restrict__ active,
                                                   uint32_t n_active, float c, uint32_t *err, uint32_t run_cap) {
    const uint32_t gi = (blockIdx.x * blockDim.x + threadIdx.x) / kLanesPerTree;
#ifdef SPAI_TREE_PRIO
    __builtin_amdgcn_s_setprio(SPAI_TREE_PRIO);   // experiment: issue priority against the co-resident forward
#endif
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    RootInfo root = load_root(T, t);
    select_tree<RUN_ON>(T, B, t, root, threadIdx.x & (kLanesPerTree - 1), c, err, run_cap);
}

// expand this iteration's leaf of every tree (batch `cur`), then select the next
// iteration's leaf into batch `nxt`.  A tree's lanes are one group of 8 in one
// wave, so its expand stores are seen by its own select loads in program order:
// a wavefront-scope fence (no instruction; it keeps the compiler from moving the
// loads above the stores), not a workgroup-scope one (s_waitcnt vmcnt(0): a
// store round trip on every iteration's critical path).
template <bool RUN_ON>
__global__ __launch_bounds__(kBlock) void k_expand_select(TreeView T, BatchView cur, BatchView nxt,
                                                          const uint32_t *__restrict__ active, uint32_t n_active,
                                                          float c, uint32_t *err, uint32_t run_cap) {
    const uint32_t gi = (blockIdx.x * blockDim.x + threadIdx.x) / kLanesPerTree;
#ifdef SPAI_TREE_PRIO
    __builtin_amdgcn_s_setprio(SPAI_TREE_PRIO);
#endif
    if (gi >= n_active) return;
    const int lane8 = threadIdx.x & (kLanesPerTree - 1);
    const uint32_t t = active[gi];
    const uint32_t s = T.slot[t];
    RootInfo root = load_root(T, t);                      // loaded with the slot, off the chain
    const LeafPath L = load_leaf_path(T, t, lane8);       // likewise (unused when the tree has no leaf)
    // the root's and the path's loads retire here: used first (or, with no leaf,
    // never) after the expansion's branch, whose join would otherwise make the
    // compiler wait for the expansion's stores too (in-order vmcnt, merged
    // conservatively over both paths)
    asm volatile("" ::"v"(root.rn), "v"(root.rw), "v"((uint32_t)root.x), "v"((uint32_t)(root.x >> 32)),
                 "v"((uint32_t)root.o), "v"((uint32_t)(root.o >> 32)), "v"((uint32_t)root.n), "v"((uint32_t)root.status));
    asm volatile("" ::"v"(L.d), "v"(L.first), "v"(L.lv[0]), "v"(L.lv[1]), "v"(L.lv[2]), "v"(L.lv[3]), "v"(L.lv[4]),
                 "v"(L.lv[5]));
    if (s != kNoSlot) expand_leaf(T, cur, t, s, lane8, err, L, root);
    // the select reads records this tree's lanes just wrote: lanes of one wave,
    // whose memory operations are performed in order (no wait for the stores)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    select_tree<RUN_ON>(T, nxt, t, root, lane8, c, err, run_cap);
}

// tail mode: every active tree has all `iters` iterations of this search call ahead
__global__ void k_set_left(TreeView T, const uint32_t *__restrict__ active, uint32_t n, uint32_t iters) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) T.left[active[i]] = iters;
}

__global__ __launch_bounds__(kBlock) void k_eval_stub(BatchView B, uint32_t max_n, int kind) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= max_n || s >= *B.count) return;
    // hash evaluator keys on absolute X/O stones: recover them from the player-to-move view
    const uint32_t n = (uint32_t)c4::popc64(B.mine[s] | B.theirs[s]);
    const bool xm = (n & 1u) == 0;
    const uint64_t x = xm ? B.mine[s] : B.theirs[s], o = xm ? B.theirs[s] : B.mine[s];
    float pr[c4::kActions], v;
    c4::stub_eval(kind, x, o, (uint8_t)n, pr, &v);
    for (int a = 0; a < c4::kActions; ++a) B.priors[(size_t)s * kPriorStride + a] = pr[a];
    B.value[s] = v;
}

__global__ __launch_bounds__(kBlock) void k_expand(TreeView T, BatchView B, uint32_t max_n, uint32_t *err) {
    const uint32_t s = (blockIdx.x * blockDim.x + threadIdx.x) / kLanesPerTree;
    if (s >= max_n || s >= *B.count) return;
    const int lane8 = threadIdx.x & (kLanesPerTree - 1);
    const uint32_t t = B.tree[s];
    RootInfo root{};   // (the root's record is not needed after the last expansion)
    expand_leaf(T, B, t, s, lane8, err, load_leaf_path(T, t, lane8), root);
}

// per active tree: [0] = root first|nch<<24 (children word), [1..7] child visit counts;
// max_evals: the most live leaves one tree evaluated in this search call
__global__ void k_root_stats(TreeView T, const uint32_t *__restrict__ active, uint32_t n_active, uint32_t *out,
                             uint32_t *max_evals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_active) return;
    const uint32_t t = active[i];
    atomicMax(max_evals, T.evals[t]);
    const uint4 *nodes = T.nodes + (size_t)t * T.cap;
    const uint4 r = nodes[T.root[t]];
    out[i * 8] = r.w;
    const uint32_t nch = r.w == kNoChildren ? 0 : r.w >> 24, first = r.w & 0xFFFFFFu;
    for (uint32_t k = 0; k < 7; ++k) out[i * 8 + 1 + k] = k < nch ? nodes[first + k].x : 0u;
}

// Self-play's move after a search call (learner_concurrent.rs:177-203), per active
// tree: the root's visit counts, the sampled child (the Philox uniform of philox.h
// and rand's WeightedIndex<f32> over (visits as f32).powf(T), the weights from a
// table of the host's powf, so the pick is the host sampler's bit for bit), and for a game that goes on the
// child written as the tree's new root (use_subtree).  One record per tree goes
// back to the host: [0] the root's children word, [1..7] the child visit counts,
// [8] the pick (index | action << 8 | new status << 16; without one, bit 31 and
// the weighted_index code, or kPickNoTable for a visit count beyond the table),
// [9] the tree's live leaves of the call.  out[0] gets the error flags, and
// block 0 copies every chain's per-iteration leaf counts after the records, so
// one copy brings back everything the host needs.
constexpr int kMoveRec = 10;
constexpr uint32_t kPickNone = 0x80000000u, kPickNoTable = 3u;
struct RootsOut {
    uint32_t *root;
    uint64_t *x, *o;
    uint8_t *n, *status;
};
struct ChainCounts {
    const uint32_t *p[spai_engine::kChains];
};
__global__ void k_advance(TreeView T, RootsOut R, const uint32_t *__restrict__ active, uint32_t n_active,
                          const float *__restrict__ pow_tab, uint32_t pow_n, uint64_t seed,
                          const uint64_t *__restrict__ slot_gid, uint32_t *__restrict__ slot_move,
                          const uint32_t *err, ChainCounts cc, int nchain, uint32_t n_counts, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            out[0] = *err;
            out[1] = 0;
        }
        uint32_t *counts = out + 2 + (size_t)n_active * kMoveRec;
        for (int h = 0; h < nchain; ++h)
            for (uint32_t j = threadIdx.x; j < n_counts; j += blockDim.x) counts[(size_t)h * n_counts + j] = cc.p[h][j];
    }
    if (i >= n_active) return;
    const uint32_t t = active[i];
    const uint4 *nodes = T.nodes + (size_t)t * T.cap;
    const uint4 r = nodes[T.root[t]];
    const uint32_t nch = r.w == kNoChildren ? 0 : r.w >> 24, first = r.w & 0xFFFFFFu;
    uint32_t vis[c4::kActions];
#pragma unroll
    for (int k = 0; k < c4::kActions; ++k) vis[k] = (uint32_t)k < nch ? nodes[first + k].x : 0u;
    uint32_t *rec = out + 2 + (size_t)i * kMoveRec;
    rec[0] = r.w;
#pragma unroll
    for (int k = 0; k < c4::kActions; ++k) rec[1 + k] = vis[k];
    rec[9] = T.evals[t];
    bool beyond = false;
    int idx = -1;   // weighted_index_with: -1 without children
    if (nch > 0) {   // WeightedIndex<f32> over (visits as f32).powf(T) (learner_concurrent.rs:189-193)
        float w[c4::kActions];
        for (uint32_t k = 0; k < nch; ++k) {
            beyond |= vis[k] >= pow_n;
            w[k] = pow_tab[min(vis[k], pow_n - 1)];
        }
        idx = weighted_index_f32(w, (int)nch, sample_u01_f32(seed, slot_gid[t], slot_move[t]));
    }
    if (beyond || idx < 0) {
        rec[8] = kPickNone | (beyond ? kPickNoTable : (uint32_t)(-idx));
        return;
    }
    const c4::State rs{T.root_x[t], T.root_o[t], T.root_n[t], T.root_status[t]};
    const int a = c4::kth_bit(c4::legal_mask(rs.x, rs.o, rs.status), idx);
    c4::State cs = rs;
    (void)c4::next_state(rs, a, cs);
    rec[8] = (uint32_t)idx | (uint32_t)a << 8 | (uint32_t)cs.status << 16;
    slot_move[t] += 1;   // the game's next move number (its sampling counter)
    if (cs.status == c4::kOngoing) {
        R.root[t] = first + (uint32_t)idx;
        R.x[t] = cs.x;
        R.o[t] = cs.o;
        R.n[t] = cs.n;
        R.status[t] = cs.status;
    }
}
// self-play: tree slot list[i] starts game list[n + i] (refill) or game gid_base +
// slot (list == null, every slot in [0, n)): an empty board as its root, an empty
// arena, move number 0
__global__ void k_slots_start(TreeView T, RootsOut R, uint64_t *__restrict__ slot_gid,
                              uint32_t *__restrict__ slot_move, const uint32_t *__restrict__ list, uint32_t n,
                              uint64_t gid_base) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = list ? list[i] : i;
    T.nodes[(size_t)t * T.cap] = make_uint4(0u, 0u, 0u, kNoChildren);
    T.next_free[t] = 1;
    R.root[t] = 0;
    R.x[t] = 0;
    R.o[t] = 0;
    R.n[t] = 0;
    R.status[t] = c4::kOngoing;
    slot_gid[t] = gid_base + (list ? list[n + i] : i);
    slot_move[t] = 0;
}

__global__ void k_trees_init(TreeView T, uint32_t first_tree, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = first_tree + i;
    T.nodes[(size_t)t * T.cap] = make_uint4(0u, 0u, 0u, kNoChildren);
    T.next_free[t] = 1;
}

TreeView tree_view(spai_engine *e) {
    Trees &T = e->trees;
    return TreeView{T.nodes.p, T.cap, T.root.p, T.next_free.p, T.root_x.p, T.root_o.p, T.root_n.p, T.root_status.p,
                    T.path.p, T.depth.p, T.slot.p, T.left.p, T.evals.p};
}

// chain `chain`'s leaf batch of search iteration `it`: buffers by parity, counter per iteration
BatchView batch_view(spai_engine *e, int chain, uint32_t it) {
    Batch &B = e->batch[chain];
    const size_t h = (size_t)(it & 1u) * B.cap;
    return BatchView{B.iter_counts.p + it, B.iter_more.p ? B.iter_more.p + it : nullptr, B.tree.p + h, B.mine.p + h, B.theirs.p + h,
                     B.priors.p + h * kPriorStride, B.value.p + h};
}

// Number of search chains for n trees: two halves when each half still fills
// a useful batch.  Late in a game most trees are solved and an iteration
// evaluates almost nothing; then the second chain only doubles the launches,
// so one chain is used when the previous search call averaged fewer than
// kMinChainLeaves leaves per iteration.  (SPAI_CHAINS=k forces up to k chains,
// for A/B measurements.)  The split never changes results: trees are independent.
constexpr double kMinChainLeaves = 64;
// Tail mode (select_tree RUN_ON): a search call runs as passes, one per live leaf
// of its busiest tree (and at least iterations / kTailRun), each lasting as long
// as its longest terminal run, at most kTailRun descents (~2.5 us each); the host
// checks for the end every kTailChunk passes.  So it pays when every tree needs
// few evaluations: it is chosen when in the previous search call no tree
// evaluated kTailTreeEvals leaves or more, or the call averaged fewer than
// kTailLeaves leaves per iteration.  (By the average alone, at 34 and
// 6.6 leaves per iteration -- moves 36 and 37 of a bench step, where some trees
// still evaluate most iterations -- it took 114 and 49 ms against ~25 and ~18 ms
// for one launch pair per iteration: profiles/r04/tail.)
constexpr double kTailLeaves = 0.05;
constexpr uint32_t kTailChunk = 4;
constexpr uint32_t kTailTreeEvals = 160;
constexpr uint32_t kTailRun = 128;   // terminal descents per tree and pass
static int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}
// Mid-game policy (tuning knobs, off by default): when the previous search call
// averaged fewer than SPAI_MID_LEAVES leaves per iteration (but at least
// kMinChainLeaves), run SPAI_MID_CHAINS chains whose forwards are capped at
// SPAI_MID_GRID workgroups, so that small per-chain batches run as larger groups
// side by side on disjoint CUs instead of one after the other over all CUs.
struct ChainPolicy {
    int chains;
    uint32_t grid_cap;   // 0: no cap
};
ChainPolicy chains_for(uint32_t n, double last_evals_per_iter) {
    static const int forced = std::max(0, std::min(spai_engine::kChains, env_int("SPAI_CHAINS", 0)));
    static const int mid_leaves = env_int("SPAI_MID_LEAVES", 0);
    static const int mid_chains = std::max(1, std::min(spai_engine::kChains, env_int("SPAI_MID_CHAINS", 2)));
    static const uint32_t mid_grid = (uint32_t)std::max(0, env_int("SPAI_MID_GRID", 0));
    static const double min_chain_leaves = env_int("SPAI_MIN_CHAIN_LEAVES", (int)kMinChainLeaves);   // A/B knob
    // A/B knob: one chain at or above this many leaves per iteration (a fresh set
    // of trees counts as one leaf per tree)
    static const int hi_leaves = env_int("SPAI_HI_LEAVES", 0);
    if (forced) return {std::max(1, std::min<int>(forced, (int)(n / 64))), 0u};
    if (hi_leaves > 0 && (last_evals_per_iter < 0 ? (double)n : last_evals_per_iter) >= hi_leaves) return {1, 0u};
    if (last_evals_per_iter >= 0 && last_evals_per_iter < min_chain_leaves) return {1, 0u};
    if (last_evals_per_iter >= 0 && last_evals_per_iter < mid_leaves)
        return {std::max(1, std::min<int>(mid_chains, (int)(n / 64))), mid_grid};
    return {std::max(1, std::min<int>(2, (int)(n / 64))), 0u};
}

// upload host root bookkeeping for trees [t0, t0+n)
int upload_roots(spai_engine *e, uint32_t t0, uint32_t n) {
    Trees &T = e->trees;
    std::vector<uint64_t> x(n), o(n);
    std::vector<uint8_t> nn(n), st(n);
    for (uint32_t i = 0; i < n; ++i) {
        const c4::State &s = T.h_root_state[t0 + i];
        x[i] = s.x;
        o[i] = s.o;
        nn[i] = s.n;
        st[i] = s.status;
    }
    hipStream_t s = e->stream;
    SPAI_HIP(hipMemcpyAsync(T.root.p + t0, T.h_root.data() + t0, n * 4, hipMemcpyHostToDevice, s));
    SPAI_HIP(hipMemcpyAsync(T.root_x.p + t0, x.data(), n * 8, hipMemcpyHostToDevice, s));
    SPAI_HIP(hipMemcpyAsync(T.root_o.p + t0, o.data(), n * 8, hipMemcpyHostToDevice, s));
    SPAI_HIP(hipMemcpyAsync(T.root_n.p + t0, nn.data(), n, hipMemcpyHostToDevice, s));
    SPAI_HIP(hipMemcpyAsync(T.root_status.p + t0, st.data(), n, hipMemcpyHostToDevice, s));
    SPAI_HIP(hipStreamSynchronize(s));
    return SPAI_OK;
}

int timer_record(spai_engine *e, int which, uint32_t iter, bool begin, hipStream_t st, int chain) {
    KernelTimer &K = e->timer;
    if (!K.enabled) return SPAI_OK;
    if (begin) {
        if (K.used + 2 > K.ev.size()) {
            for (int i = 0; i < 64; ++i) {
                hipEvent_t ev;
                SPAI_HIP(hipEventCreate(&ev));
                K.ev.push_back(ev);
            }
        }
        K.which.push_back(which);
        K.iter.push_back(iter);
        K.chain.push_back(chain);
        SPAI_HIP(hipEventRecord(K.ev[K.used], st));
    } else {
        SPAI_HIP(hipEventRecord(K.ev[K.used + 1], st));
        K.used += 2;
    }
    return SPAI_OK;
}

// fold the sampled event pairs of one search call into the totals
// ch_counts [chain][num_searches] leaves per iteration; n_active[chain] trees
int timer_collect(spai_engine *e, const uint32_t *ch_counts, uint32_t num_searches,
                  const uint32_t *n_active) {
    KernelTimer &K = e->timer;
    if (!K.enabled) return SPAI_OK;
    for (size_t i = 0; i < K.which.size(); ++i) {
        float ms = 0;
        SPAI_HIP(hipEventElapsedTime(&ms, K.ev[2 * i], K.ev[2 * i + 1]));
        const int w = K.which[i], h = K.chain[i];
        K.total_ms[w] += ms;
        K.launches[w] += 1;
        K.items[w] += w == 0 ? n_active[h] : ch_counts[(size_t)h * num_searches + K.iter[i]];
    }
    K.used = 0;
    K.which.clear();
    K.iter.clear();
    K.chain.clear();
    return SPAI_OK;
}

}  // namespace

int trees_create(spai_engine *e, uint32_t n) {
    SPAI_CHECK(n > 0 && n <= e->cfg.max_trees, SPAI_ERR_INVALID, "trees_create: n=%u exceeds max_trees=%u", n,
               e->cfg.max_trees);
    Trees &T = e->trees;
    // worst case: one expansion of <= 7 children per search iteration for every ply of the game
    const uint64_t cap = 1ull + (uint64_t)c4::kActions * e->cfg.num_searches * std::max(1u, e->cfg.max_moves);
    SPAI_CHECK(cap < (1ull << 24), SPAI_ERR_CAPACITY, "node arena of %llu nodes per tree exceeds 2^24",
               (unsigned long long)cap);
    if (T.n_trees != n || T.cap != cap) {
        T.n_trees = 0;
        SPAI_TRY(T.nodes.alloc((size_t)n * cap));
        SPAI_TRY(T.root.alloc(n));
        SPAI_TRY(T.next_free.alloc(n));
        SPAI_TRY(T.root_x.alloc(n));
        SPAI_TRY(T.root_o.alloc(n));
        SPAI_TRY(T.root_n.alloc(n));
        SPAI_TRY(T.root_status.alloc(n));
        SPAI_TRY(T.path.alloc((size_t)n * kMaxDepth));
        SPAI_TRY(T.depth.alloc(n));
        SPAI_TRY(T.slot.alloc(n));
        SPAI_TRY(T.left.alloc(n));
        SPAI_TRY(T.evals.alloc(n + 1));   // [n]: the search call's max over trees (k_root_stats)
        SPAI_TRY(T.slot_gid.alloc(n));
        SPAI_TRY(T.slot_move.alloc(n));
        SPAI_TRY(T.refill.alloc(2 * (size_t)n));
        SPAI_TRY(e->active.alloc(n));
        SPAI_TRY(e->stats.alloc((size_t)n * 8));
        for (Batch &B : e->batch) {   // one double-buffered leaf batch per search chain
            SPAI_TRY(B.tree.alloc(2 * (size_t)n));
            SPAI_TRY(B.mine.alloc(2 * (size_t)n));
            SPAI_TRY(B.theirs.alloc(2 * (size_t)n));
            SPAI_TRY(B.priors.alloc(2 * (size_t)n * kPriorStride));
            SPAI_TRY(B.value.alloc(2 * (size_t)n));
            B.cap = n;
        }
        T.n_trees = n;
        T.cap = (uint32_t)cap;
    }
    e->last_evals_per_iter = -1;   // a fresh set of trees: no per-iteration statistics yet
    e->last_max_tree_evals = ~0u;
    T.h_root.assign(n, 0);
    T.h_root_state.assign(n, c4::State{0, 0, 0, c4::kOngoing});
    T.h_root_first.assign(n, 0);
    T.h_root_nch.assign(n, 0);
    k_trees_init<<<(n + 255) / 256, 256, 0, e->stream>>>(tree_view(e), 0, n);
    SPAI_HIP(hipGetLastError());
    return upload_roots(e, 0, n);
}

int tree_reset(spai_engine *e, uint32_t t, const spai_c4_state *root) {
    Trees &T = e->trees;
    SPAI_CHECK(t < T.n_trees, SPAI_ERR_INVALID, "tree %u out of range", t);
    c4::State s{0, 0, 0, c4::kOngoing};
    if (root) {
        SPAI_CHECK(!(root->x & root->o) && !((root->x | root->o) & ~c4::kBoard) && root->status <= c4::kWon,
                   SPAI_ERR_INVALID, "root is not a Connect4 bitboard");
        s = from_abi(*root);
    }
    T.h_root[t] = 0;
    T.h_root_state[t] = s;
    T.h_root_first[t] = 0;
    T.h_root_nch[t] = 0;
    k_trees_init<<<1, 64, 0, e->stream>>>(tree_view(e), t, 1);
    SPAI_HIP(hipGetLastError());
    return upload_roots(e, t, 1);
}

namespace {
// Policy::normalize: ndarray sum (sequential for 7) then divide
inline void normalize_policy(const float (&pol)[c4::kActions], float *out) {
    float s = 0.0f;
    for (int a = 0; a < c4::kActions; ++a) s = s + pol[a];
    for (int a = 0; a < c4::kActions; ++a) out[a] = pol[a] / s;
}

// one search call's launch layout, for search_finish
struct SearchRun {
    int nchain = 1;
    bool tail = false;
    uint32_t n_counts = 0;                                  // per-iteration leaf counters per chain
    uint32_t cnt[spai_engine::kChains] = {0, 0, 0, 0};      // trees per chain
};

// Enqueue one search call over n >= 1 validated trees (mcts.rs:214-285 per tree),
// up to the join of its chains on the engine stream.  Only tail mode waits (once
// per chunk of passes, for its stop condition).
int search_launch(spai_engine *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, SearchRun &R) {
    Trees &T = e->trees;
    const int kind = (int)e->cfg.eval;
    hipStream_t st = e->stream;
    // tail mode (select_tree RUN_ON, one chain): late in a game, when in the previous
    // search call of these trees no tree evaluated SPAI_TAIL_TREE_EVALS leaves or
    // more (a pass per live leaf of the busiest tree: few passes), or the call
    // averaged fewer than SPAI_TAIL_LEAVES leaves per iteration.  Both read per
    // call (tests set them per case); 0 turns a criterion off.
    const char *tl_env = std::getenv("SPAI_TAIL_LEAVES");
    const char *tt_env = std::getenv("SPAI_TAIL_TREE_EVALS");
    const double tail_leaves = tl_env ? std::atof(tl_env) : kTailLeaves;
    const uint32_t tail_tree = tt_env ? (uint32_t)std::max(0, std::atoi(tt_env)) : kTailTreeEvals;
    const bool tail = num_searches > 0 && e->last_evals_per_iter >= 0 &&
                      (e->last_evals_per_iter < tail_leaves || e->last_max_tree_evals < tail_tree);
    // the run cap; after a call that evaluated nothing (every tree solved: no tree
    // to keep waiting) none, and a check after every pass -- normally one
    const bool solved = e->last_evals_per_iter == 0.0;
    const char *tr_env = std::getenv("SPAI_TAIL_RUN");
    const uint32_t tail_run =
        tr_env ? (uint32_t)std::max(1, std::atoi(tr_env)) : (solved ? std::max(num_searches, 1u) : kTailRun);
    const uint32_t tail_chunk = solved ? 1u : kTailChunk;
    // chain h searches active[off[h] .. off[h] + cnt[h]) on chain_stream[h]
    const ChainPolicy pol = tail ? ChainPolicy{1, 0u} : chains_for(n, e->last_evals_per_iter);
    const int nchain = pol.chains;
    uint32_t off[spai_engine::kChains] = {0, 0, 0, 0};
    uint32_t *cnt = R.cnt;
    R.nchain = nchain;
    R.tail = tail;
    for (int h = 0; h < nchain; ++h) {
        off[h] = (uint32_t)((uint64_t)n * h / nchain);
        cnt[h] = (uint32_t)((uint64_t)n * (h + 1) / nchain) - off[h];
    }
    for (int h = 0; h < nchain; ++h) {   // per-iteration leaf counters (also the batch slot counters)
        Batch &B = e->batch[h];
        // at least one counter even for num_searches == 0, so the memset never sees a
        // null buffer on a fresh engine; tail mode runs up to num_searches + 1 passes
        // in chunks of kTailChunk
        const uint32_t nc = std::max<uint32_t>(num_searches, 1) + (tail ? kTailChunk + 1 : 0);
        if (B.iter_counts.n < nc) SPAI_TRY(B.iter_counts.alloc(nc));
        SPAI_HIP(hipMemsetAsync(B.iter_counts.p, 0, (size_t)nc * 4, st));
        if (tail) {
            if (B.iter_more.n < nc) SPAI_TRY(B.iter_more.alloc(nc));
            SPAI_HIP(hipMemsetAsync(B.iter_more.p, 0, (size_t)nc * 4, st));
        }
    }
    SPAI_HIP(hipMemcpyAsync(e->active.p, tree_idx, n * 4, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemsetAsync(e->err.p, 0, 4, st));
    SPAI_HIP(hipMemsetAsync(T.evals.p, 0, ((size_t)T.n_trees + 1) * 4, st));
    if (nchain > 1) {   // fork: chains 1.. start after the setup on the engine stream
        SPAI_HIP(hipEventRecord(e->ev_fork, st));
        for (int h = 1; h < nchain; ++h) SPAI_HIP(hipStreamWaitEvent(e->chain_stream[h], e->ev_fork, 0));
    }
    const TreeView tv = tree_view(e);
    const bool timed = e->timer.enabled && !tail;   // samples every chain's launches every stride-th iteration
    uint32_t &n_counts = R.n_counts;   // leaf counters to read back per chain
    n_counts = num_searches;
    if (tail) {
        // passes on the engine stream: select(0), then per pass p: evaluate(p),
        // expand(p) + select(p + 1), each select running its trees on through
        // terminal leaves (at most tail_run per pass).  A pass whose select slots
        // no leaf and caps no tree leaves no tree with iterations to run (a tree
        // stops a launch only at a live leaf or the cap), so the host checks every
        // tail_chunk passes and stops there.
        const uint32_t g8 = (n + kTreesPerBlock - 1) / kTreesPerBlock;
        const uint32_t *act = e->active.p;
        k_set_left<<<(n + 255) / 256, 256, 0, st>>>(tv, act, n, num_searches);
        k_select<true><<<g8, kBlock, 0, st>>>(tv, batch_view(e, 0, 0), act, n, e->cfg.c, e->err.p, tail_run);
        uint32_t p = 0, next = 1, more = 0;
        for (;;) {
            for (uint32_t q = 0; q < tail_chunk; ++q, ++p) {
                const BatchView bv = batch_view(e, 0, p);
                if (kind == SPAI_EVAL_NET) {
                    SPAI_TRY(net_eval_batch(e->net, st, bv.count, n, bv.mine, bv.theirs, bv.priors, bv.value, 0));
                } else {
                    k_eval_stub<<<(n + kBlock - 1) / kBlock, kBlock, 0, st>>>(bv, n, kind);
                }
                k_expand_select<true><<<g8, kBlock, 0, st>>>(tv, bv, batch_view(e, 0, p + 1), act, n, e->cfg.c,
                                                             e->err.p, tail_run);
            }
            SPAI_HIP(hipGetLastError());
            SPAI_HIP(hipMemcpyAsync(&next, e->batch[0].iter_counts.p + p, 4, hipMemcpyDeviceToHost, st));
            SPAI_HIP(hipMemcpyAsync(&more, e->batch[0].iter_more.p + p, 4, hipMemcpyDeviceToHost, st));
            SPAI_HIP(hipStreamSynchronize(st));
            if (next == 0 && more == 0) break;   // pass p has nothing to evaluate and no tree was capped: all done
            SPAI_CHECK(p <= num_searches + 1, SPAI_ERR_INVALID, "internal: tail passes exceed the iterations");
            // this chunk's counters are read back below; the next chunk's are fresh
        }
        n_counts = p;
    }
    e->last_tail_passes = tail ? n_counts : 0;
    // per chain: select(0); then per iteration: evaluate(it), expand(it)+select(it+1)
    // fused, and expand alone after the last evaluation.  Timer 0 samples the
    // select-bearing launch (k_select / k_expand_select), 2 the last k_expand.
    for (uint32_t it = 0; it < (tail ? 0u : num_searches); ++it) {
        for (int h = 0; h < nchain; ++h) {
            const hipStream_t sh = e->chain_stream[h];
            const BatchView bv = batch_view(e, h, it);
            const uint32_t nh = cnt[h], g8 = (nh + kTreesPerBlock - 1) / kTreesPerBlock;
            const uint32_t *act = e->active.p + off[h];
            const bool sample = timed && (it % e->timer.stride == 0);
            if (it == 0) {
                if (sample) SPAI_TRY(timer_record(e, 0, it, true, sh, h));
                k_select<false><<<g8, kBlock, 0, sh>>>(tv, bv, act, nh, e->cfg.c, e->err.p, 0u);
                if (sample) SPAI_TRY(timer_record(e, 0, it, false, sh, h));
            }
            if (sample) SPAI_TRY(timer_record(e, 1, it, true, sh, h));
            if (kind == SPAI_EVAL_NET) {
                SPAI_TRY(net_eval_batch(e->net, sh, bv.count, nh, bv.mine, bv.theirs, bv.priors, bv.value,
                                        pol.grid_cap, nchain));
            } else {
                k_eval_stub<<<(nh + kBlock - 1) / kBlock, kBlock, 0, sh>>>(bv, nh, kind);
            }
            if (sample) SPAI_TRY(timer_record(e, 1, it, false, sh, h));
            if (it + 1 < num_searches) {
                const bool s2 = timed && ((it + 1) % e->timer.stride == 0);
                if (s2) SPAI_TRY(timer_record(e, 0, it + 1, true, sh, h));
                k_expand_select<false><<<g8, kBlock, 0, sh>>>(tv, bv, batch_view(e, h, it + 1), act, nh,
                                                              e->cfg.c, e->err.p, 0u);
                if (s2) SPAI_TRY(timer_record(e, 0, it + 1, false, sh, h));
            } else {
                if (sample) SPAI_TRY(timer_record(e, 2, it, true, sh, h));
                k_expand<<<g8, kBlock, 0, sh>>>(tv, bv, nh, e->err.p);
                if (sample) SPAI_TRY(timer_record(e, 2, it, false, sh, h));
            }
        }
    }
    SPAI_HIP(hipGetLastError());
    for (int h = 1; h < nchain; ++h) {   // join
        SPAI_HIP(hipEventRecord(e->ev_join[h], e->chain_stream[h]));
        SPAI_HIP(hipStreamWaitEvent(st, e->ev_join[h], 0));
    }
    return SPAI_OK;
}

// The call's bookkeeping once its counters [chain][n_counts], error flags and
// largest per-tree leaf count are on the host: timers, the device errors, and the
// statistics the next call's chain and tail policies read.
int search_finish(spai_engine *e, const SearchRun &R, uint32_t num_searches, const uint32_t *ch_counts, uint32_t err,
                  uint32_t max_tree_evals, double *evals_out) {
    SPAI_TRY(timer_collect(e, ch_counts, R.n_counts, R.cnt));
    double s = 0;
    for (int h = 0; h < R.nchain; ++h)
        for (uint32_t i = 0; i < R.n_counts; ++i) s += ch_counts[(size_t)h * R.n_counts + i];
    SPAI_CHECK(!(err & kErrCapacity), SPAI_ERR_CAPACITY, "node arena full (cap %u per tree)", e->trees.cap);
    SPAI_CHECK(!(err & kErrDepth), SPAI_ERR_CAPACITY, "tree deeper than %d", kMaxDepth);
    SPAI_CHECK(!(err & kErrNan), SPAI_ERR_NAN, "NaN UCB in select (reference: partial_cmp().unwrap() panics)");
    if (evals_out) *evals_out = s;
    e->last_evals_per_iter = num_searches ? s / num_searches : -1;
    e->last_max_tree_evals = max_tree_evals;
    return SPAI_OK;
}
}  // namespace

int search(spai_engine *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
           uint32_t *child_ids, float *child_visits, uint32_t *n_children, double *evals_out) {
    Trees &T = e->trees;
    SPAI_CHECK(T.n_trees > 0, SPAI_ERR_INVALID, "no trees: call spai_trees_create first");
    SPAI_CHECK(n <= T.n_trees, SPAI_ERR_INVALID, "search over %u trees, %u exist", n, T.n_trees);
    for (uint32_t i = 0; i < n; ++i) SPAI_CHECK(tree_idx[i] < T.n_trees, SPAI_ERR_INVALID, "tree %u out of range", tree_idx[i]);
    const int kind = (int)e->cfg.eval;
    SPAI_CHECK(kind != SPAI_EVAL_NET || e->net, SPAI_ERR_INVALID, "eval = NET but no net set (spai_engine_set_net)");
    if (n == 0) return SPAI_OK;
    hipStream_t st = e->stream;
    SearchRun R;
    SPAI_TRY(search_launch(e, n, tree_idx, num_searches, R));
    const TreeView tv = tree_view(e);
    const int nchain = R.nchain;
    const uint32_t n_counts = R.n_counts;
    k_root_stats<<<(n + 255) / 256, 256, 0, st>>>(tv, e->active.p, n, e->stats.p, T.evals.p + T.n_trees);
    SPAI_HIP(hipGetLastError());
    std::vector<uint32_t> stats((size_t)n * 8), ch_counts((size_t)nchain * n_counts);
    uint32_t err = 0, max_tree_evals = 0;
    SPAI_HIP(hipMemcpyAsync(stats.data(), e->stats.p, stats.size() * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipMemcpyAsync(&max_tree_evals, T.evals.p + T.n_trees, 4, hipMemcpyDeviceToHost, st));
    if (n_counts)
        for (int h = 0; h < nchain; ++h)
            SPAI_HIP(hipMemcpyAsync(ch_counts.data() + (size_t)h * n_counts, e->batch[h].iter_counts.p,
                                    n_counts * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipMemcpyAsync(&err, e->err.p, 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    SPAI_TRY(search_finish(e, R, num_searches, ch_counts.data(), err, max_tree_evals, evals_out));
    // root visit policy (mcts.rs:310-331)
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t t = tree_idx[i];
        const uint32_t w = stats[i * 8];
        const uint32_t nch = w == kNoChildren ? 0 : w >> 24, first = w & 0xFFFFFFu;
        T.h_root_first[t] = first;
        T.h_root_nch[t] = (uint8_t)nch;
        const c4::State &rs = T.h_root_state[t];
        const uint32_t legal = c4::legal_mask(rs.x, rs.o, rs.status);
        float pol[c4::kActions] = {0, 0, 0, 0, 0, 0, 0};
        for (uint32_t k = 0; k < nch; ++k) {
            const float v = (float)stats[i * 8 + 1 + k];
            pol[c4::kth_bit(legal, (int)k)] = v;
            if (child_ids) child_ids[(size_t)i * 7 + k] = first + k;
            if (child_visits) child_visits[(size_t)i * 7 + k] = v;
        }
        for (uint32_t k = nch; k < 7; ++k) {
            if (child_ids) child_ids[(size_t)i * 7 + k] = kNoChildren;
            if (child_visits) child_visits[(size_t)i * 7 + k] = 0.f;
        }
        if (n_children) n_children[i] = nch;
        if (policy) normalize_policy(pol, policy + (size_t)i * 7);
    }
    return SPAI_OK;
}

int tree_use_subtree(spai_engine *e, uint32_t t, uint32_t child) {
    Trees &T = e->trees;
    SPAI_CHECK(t < T.n_trees, SPAI_ERR_INVALID, "tree %u out of range", t);
    const uint32_t first = T.h_root_first[t], nch = T.h_root_nch[t];
    SPAI_CHECK(nch > 0 && child >= first && child < first + nch, SPAI_ERR_INVALID,
               "node %u is not a child of tree %u's root (run spai_search first)", child, t);
    const c4::State &rs = T.h_root_state[t];
    c4::State ns;
    const int a = c4::kth_bit(c4::legal_mask(rs.x, rs.o, rs.status), (int)(child - first));
    SPAI_CHECK(c4::next_state(rs, a, ns) == 0, SPAI_ERR_INVALID, "internal: root child replay failed");
    T.h_root[t] = child;
    T.h_root_state[t] = ns;
    T.h_root_nch[t] = 0;
    return upload_roots(e, t, 1);
}

int tree_node(spai_engine *e, uint32_t t, uint32_t node, spai_c4_state *st, uint32_t *visits, float *w) {
    Trees &T = e->trees;
    SPAI_CHECK(t < T.n_trees, SPAI_ERR_INVALID, "tree %u out of range", t);
    c4::State s = T.h_root_state[t];
    if (node != T.h_root[t]) {
        const uint32_t first = T.h_root_first[t], nch = T.h_root_nch[t];
        SPAI_CHECK(nch > 0 && node >= first && node < first + nch, SPAI_ERR_INVALID,
                   "node %u: only the root and its children are addressable", node);
        const int a = c4::kth_bit(c4::legal_mask(s.x, s.o, s.status), (int)(node - first));
        c4::State ns;
        c4::next_state(s, a, ns);
        s = ns;
    }
    if (st) *st = to_abi(s);
    if (visits || w) {
        uint4 rec;
        SPAI_HIP(hipMemcpy(&rec, T.nodes.p + (size_t)t * T.cap + node, 16, hipMemcpyDeviceToHost));
        if (visits) *visits = rec.x;
        if (w) memcpy(w, &rec.y, 4);
    }
    return SPAI_OK;
}

int tree_size(spai_engine *e, uint32_t t, uint32_t *nodes) {
    Trees &T = e->trees;
    SPAI_CHECK(t < T.n_trees, SPAI_ERR_INVALID, "tree %u out of range", t);
    SPAI_HIP(hipMemcpy(nodes, T.next_free.p + t, 4, hipMemcpyDeviceToHost));
    return SPAI_OK;
}

// SelfPlayWorker::self_play (learner_concurrent.rs:169-242).  Per move: the search
// call, then k_advance samples every game's move on the device and moves its
// root, and one pinned copy brings back the records.  The next move's search is
// launched as soon as the host knows which games go on; this move's bookkeeping
// (policy targets, histories, finished games to the sink, in the reference's
// order) runs on the host while it searches.
// window < n_games (spai_selfplay_stream): the games run through `window` tree
// slots; a slot whose game ended takes the next game before the next search call.
// Each game's draws are keyed by its id and its own move number (per slot on the
// device), so every game is the one spai_selfplay_run would play.
int selfplay_run(spai_engine *e, uint32_t n_games, uint64_t gid_base, spai_sample_sink sink, void *user,
                 spai_selfplay_stats *stats, uint32_t window) {
    const auto t_start = std::chrono::steady_clock::now();
    const uint32_t W = (window == 0 || window >= n_games) ? n_games : window;   // tree slots
    SPAI_TRY(trees_create(e, W));
    SPAI_CHECK(e->cfg.eval != SPAI_EVAL_NET || e->net, SPAI_ERR_INVALID,
               "eval = NET but no net set (spai_engine_set_net)");
    Trees &T = e->trees;
    hipStream_t st = e->stream;
    const uint32_t ns = e->cfg.num_searches;
    // every game's history in flat per-game slabs of the longest game (42 plies):
    // growing 3 x n_games vectors made every game reallocate at the same moves
    constexpr size_t kPlies = c4::kCells;
    // (visits as f32).powf(T) for every count a root child can reach (a search call
    // adds at most ns visits to a root, a game has at most kPlies moves), by the
    // host's powf (the f32::powf of the reference), once per temperature
    const uint32_t pow_n = ns * (uint32_t)kPlies + 1;
    const float temp = e->cfg.temperature;
    if (e->pow_tab_t != temp || e->pow_tab.n < pow_n) {
        std::vector<float> tab(pow_n);
        for (uint32_t k = 0; k < pow_n; ++k) tab[k] = ::powf((float)k, temp);   // Rust f32::powf = libm powf
        e->pow_tab_t = -1.0f;
        SPAI_TRY(e->pow_tab.alloc(pow_n));
        SPAI_HIP(hipMemcpy(e->pow_tab.p, tab.data(), pow_n * sizeof(float), hipMemcpyHostToDevice));
        e->pow_tab_t = temp;
    }
    // records, then every chain's leaf counters (tail mode: up to ns + kTailChunk + 1)
    const size_t n_words = 2 + (size_t)W * kMoveRec +
                           (size_t)spai_engine::kChains * (std::max(ns, 1u) + kTailChunk + 1);
    if (e->h_move_n < n_words) {
        e->h_move_n = 0;
        for (uint32_t *&h : e->h_move) {
            if (h) (void)hipHostFree(h);
            h = nullptr;
            void *ph = nullptr;
            SPAI_HIP(hipHostMalloc(&ph, n_words * 4, hipHostMallocDefault));
            h = (uint32_t *)ph;
        }
        SPAI_TRY(e->move_out.alloc(n_words));
        e->h_move_n = n_words;
    }
    std::vector<c4::State> h_states((size_t)W * kPlies);   // per tree slot
    std::vector<float> h_pol((size_t)W * kPlies * 7);
    std::vector<int32_t> h_moves((size_t)W * kPlies);
    std::vector<uint32_t> h_len(W, 0);
    std::vector<uint32_t> act[2];   // this move's trees and the next move's (the launch reads them)
    act[0].resize(W);
    for (uint32_t i = 0; i < W; ++i) act[0][i] = i;
    std::vector<uint32_t> slot_game(W);   // the game (index < n_games) each slot plays
    for (uint32_t i = 0; i < W; ++i) slot_game[i] = i;
    uint32_t next_game = W;
    std::vector<uint32_t> refill[2];   // per move parity: [slots..., games...] uploaded for k_slots_start
    std::vector<float> enc, sv;
    double sims = 0, evals = 0, games = 0, positions = 0, moves = 0;
    // optional per-move trace (diagnostics): SPAI_TRACE_MOVES=<csv path>
    FILE *trace = nullptr;
    if (const char *tp = std::getenv("SPAI_TRACE_MOVES")) trace = std::fopen(tp, "a");
    struct TraceClose {
        FILE *f;
        ~TraceClose() {
            if (f) std::fclose(f);
        }
    } trace_close{trace};
    const TreeView tv = tree_view(e);
    const RootsOut ro{T.root.p, T.root_x.p, T.root_o.p, T.root_n.p, T.root_status.p};
    SearchRun R;
    // every slot starts its first game (id gid_base + slot) at move 0
    k_slots_start<<<(W + 255) / 256, 256, 0, st>>>(tv, ro, T.slot_gid.p, T.slot_move.p, nullptr, W, gid_base);
    SPAI_HIP(hipGetLastError());
    // enqueue a move over the trees a: slots in rf start their new games, the search
    // call, k_advance, the records' copy to dst
    auto launch = [&](const std::vector<uint32_t> &a, const std::vector<uint32_t> &rf, uint32_t *dst) -> int {
        const uint32_t na = (uint32_t)a.size();
        if (!rf.empty()) {
            const uint32_t nr = (uint32_t)(rf.size() / 2);
            SPAI_HIP(hipMemcpyAsync(T.refill.p, rf.data(), rf.size() * 4, hipMemcpyHostToDevice, st));
            k_slots_start<<<(nr + 255) / 256, 256, 0, st>>>(tv, ro, T.slot_gid.p, T.slot_move.p, T.refill.p, nr,
                                                           gid_base);
        }
        SPAI_TRY(search_launch(e, na, a.data(), ns, R));
        ChainCounts cc{};
        for (int h = 0; h < R.nchain; ++h) cc.p[h] = e->batch[h].iter_counts.p;
        k_advance<<<(na + 63) / 64, 64, 0, st>>>(tv, ro, e->active.p, na, e->pow_tab.p, (uint32_t)e->pow_tab.n,
                                                 e->cfg.seed, T.slot_gid.p, T.slot_move.p, e->err.p, cc, R.nchain,
                                                 R.n_counts, e->move_out.p);
        SPAI_HIP(hipGetLastError());
        const size_t words = 2 + (size_t)na * kMoveRec + (size_t)R.nchain * R.n_counts;
        SPAI_HIP(hipMemcpyAsync(dst, e->move_out.p, words * 4, hipMemcpyDeviceToHost, st));
        return SPAI_OK;
    };
    // every return below, errors included, leaves the engine quiescent: the next
    // move's search, k_advance and the record copy may be in flight when a
    // bookkeeping check fails (they write device roots and a pinned buffer)
    struct Quiesce {
        spai_engine *e;
        ~Quiesce() {
            (void)hipStreamSynchronize(e->stream);
            for (hipStream_t cs : e->chain_stream)
                if (cs) (void)hipStreamSynchronize(cs);
        }
    } quiesce{e};
    uint64_t move_no = 0;
    int cur = 0;
    auto tm0 = std::chrono::steady_clock::now();
    SPAI_TRY(launch(act[0], refill[0], e->h_move[0]));
    while (!act[cur].empty()) {
        const std::vector<uint32_t> &A = act[cur];
        const uint32_t na = (uint32_t)A.size();
        const uint32_t *mo = e->h_move[move_no & 1];
        SPAI_HIP(hipStreamSynchronize(st));
        const auto tm1 = std::chrono::steady_clock::now();
        const uint32_t passes = e->last_tail_passes;
        uint32_t max_ev = 0;
        bool stop = false;   // a game without a move: its error is raised in the bookkeeping below
        for (uint32_t i = 0; i < na; ++i) {
            const uint32_t *rec = mo + 2 + (size_t)i * kMoveRec;
            max_ev = std::max(max_ev, rec[9]);
            stop |= (rec[8] & kPickNone) != 0;
        }
        double ev = 0;
        SPAI_TRY(search_finish(e, R, ns, mo + 2 + (size_t)na * kMoveRec, mo[0], max_ev, &ev));
        sims += (double)na * ns;
        evals += ev;
        moves += 1;
        // the games that go on, in order (trees_vec.remove keeps it), and their next move;
        // streaming: slots whose game ended take the next games (appended)
        std::vector<uint32_t> &N = act[cur ^ 1];
        std::vector<uint32_t> &RF = refill[(move_no + 1) & 1];
        N.clear();
        RF.clear();
        auto tm2 = tm1;
        if (!stop) {
            for (uint32_t i = 0; i < na; ++i)
                if (((mo[2 + (size_t)i * kMoveRec + 8] >> 16) & 0xFFu) == c4::kOngoing) N.push_back(A[i]);
            for (uint32_t i = 0; i < na && next_game < n_games; ++i)
                if (((mo[2 + (size_t)i * kMoveRec + 8] >> 16) & 0xFFu) != c4::kOngoing) {
                    RF.push_back(A[i]);
                    RF.push_back(next_game++);
                }
            const size_t nr = RF.size() / 2;
            if (nr) {   // [slots..., games...]
                std::vector<uint32_t> tmp(RF);
                for (size_t j = 0; j < nr; ++j) {
                    RF[j] = tmp[2 * j];
                    RF[nr + j] = tmp[2 * j + 1];
                    N.push_back(RF[j]);
                }
            }
            tm2 = std::chrono::steady_clock::now();
            if (!N.empty()) SPAI_TRY(launch(N, RF, e->h_move[(move_no + 1) & 1]));
        }
        const auto tm3 = std::chrono::steady_clock::now();
        for (int k = (int)na - 1; k >= 0; --k) {   // for i in (0..trees_vec.len()).rev()
            const uint32_t t = A[k];
            const uint32_t *rec = mo + 2 + (size_t)k * kMoveRec;
            const uint32_t w = rec[0], pick = rec[8];
            if (pick & kPickNone) {
                SPAI_CHECK((pick & 0xFFu) != kPickNoTable, SPAI_ERR_INVALID,
                           "internal: game %u has a visit count beyond the visits^T table", t);
                SPAI_CHECK(false, SPAI_ERR_NAN, "WeightedIndex over all-zero visit counts (game %u)", t);
            }
            const uint32_t nch = w == kNoChildren ? 0 : w >> 24, first = w & 0xFFFFFFu;
            T.h_root_first[t] = first;
            T.h_root_nch[t] = (uint8_t)nch;
            const c4::State rs = T.h_root_state[t];
            const uint32_t legal = c4::legal_mask(rs.x, rs.o, rs.status);
            float pol[c4::kActions] = {0, 0, 0, 0, 0, 0, 0};   // root visit policy (mcts.rs:310-331)
            for (uint32_t j = 0; j < nch; ++j) pol[c4::kth_bit(legal, (int)j)] = (float)rec[1 + j];
            const int idx = (int)(pick & 0xFFu), a = (int)((pick >> 8) & 0xFFu);
            c4::State cs;
            SPAI_CHECK((uint32_t)idx < nch && a == c4::kth_bit(legal, idx) && c4::next_state(rs, a, cs) == 0 &&
                           cs.status == ((pick >> 16) & 0xFFu),
                       SPAI_ERR_INVALID, "internal: game %u's device move does not replay", t);
            const size_t m = ++h_len[t];   // plies so far, this one included
            SPAI_CHECK(m <= kPlies, SPAI_ERR_INVALID, "internal: game %u longer than %zu plies", t, kPlies);
            c4::State *hs = h_states.data() + (size_t)t * kPlies;
            float *hp = h_pol.data() + (size_t)t * kPlies * 7;
            int32_t *hm = h_moves.data() + (size_t)t * kPlies;
            hs[m - 1] = rs;
            normalize_policy(pol, hp + (m - 1) * 7);
            hm[m - 1] = a;
            if (cs.status != c4::kOngoing) {                  // is_terminal: emit, trees_vec.remove(i)
                const float v = c4::terminal_value(cs.status);
                enc.assign(sink ? m * 126 : 0, 0.f);
                sv.resize(m);
                for (size_t j = 0; j < (sink ? m : 0); ++j) {
                    const c4::State &s = hs[j];
                    const bool xm = c4::x_to_move(s.n);
                    const uint64_t mine = xm ? s.x : s.o, theirs = xm ? s.o : s.x;
                    for (int r = 0; r < 6; ++r)
                        for (int cc = 0; cc < 7; ++cc) {
                            const int b = cc * 7 + r, cell = r * 7 + cc;
                            if ((mine >> b) & 1) enc[j * 126 + cell] = 1.f;
                            else if ((theirs >> b) & 1) enc[j * 126 + 42 + cell] = 1.f;
                            else enc[j * 126 + 84 + cell] = 1.f;
                        }
                    // x.get_current_player() == state.get_current_player() ? value : -value
                    sv[j] = ((s.n & 1) == (cs.n & 1)) ? v : -v;
                }
                if (sink) sink(user, (uint32_t)(gid_base + slot_game[t]), (uint32_t)m, enc.data(), hp, sv.data(), hm);
                games += 1;
                positions += (double)m;
                h_len[t] = 0;
            } else {                                          // use_subtree(selected_id), already on the device
                T.h_root[t] = first + (uint32_t)idx;
                T.h_root_state[t] = cs;
                T.h_root_nch[t] = 0;
            }
        }
        {   // streaming: the refilled slots' host mirrors start their new games (k_slots_start
            // reset the device side ahead of the search call already in flight)
            const std::vector<uint32_t> &RFc = refill[(move_no + 1) & 1];
            const size_t nr = RFc.size() / 2;
            for (size_t j = 0; j < nr; ++j) {
                const uint32_t t = RFc[j];
                slot_game[t] = RFc[nr + j];
                T.h_root[t] = 0;
                T.h_root_state[t] = c4::State{0, 0, 0, c4::kOngoing};
                T.h_root_first[t] = 0;
                T.h_root_nch[t] = 0;
            }
        }
        if (trace)   // move, active trees, leaves evaluated, search seconds (launch to records), host seconds
                     // between the records and the next launch, search passes (tail mode; 0: one launch pair
                     // per iteration), bookkeeping seconds (overlapping the next search)
            std::fprintf(trace, "%llu,%u,%.0f,%.6f,%.6f,%u,%.6f\n", (unsigned long long)move_no, na, ev,
                         std::chrono::duration<double>(tm1 - tm0).count(),
                         std::chrono::duration<double>(tm2 - tm1).count(), passes,
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - tm3).count());
        tm0 = tm2;
        cur ^= 1;
        ++move_no;
    }
    if (stats) {
        stats->sims = sims;
        stats->evals = evals;
        stats->games = games;
        stats->positions = positions;
        stats->moves = moves;
        stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    }
    return SPAI_OK;
}

}  // namespace spai

// ttt.hip — TicTacToe on the device (BASELINE config 1):
// game/tictactoe.rs rules, model/tictactoe.rs net, and the game-generic
// mcts.rs search + learner_concurrent.rs self-play, behind spai_ttt_* in
// include/spai.h.
//
// The board is two 9-bit masks (bit r*3 + c; X moves first, X to move iff the
// move count is even).  Everything is small, so the design favours exactness
// over throughput: the net runs in fp32 on the VALU (one workgroup of 64
// threads = 64 channels per position, BN folded, weights transposed for
// coalesced reads), trees are 16-byte node records in HBM searched by one
// wavefront per tree (lane k scores child k), and the stub evaluators use the
// oracle's exact operation order so search and self-play are bit-exact against
// oracle/spai_oracle.c.
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "philox.h"
#include "spai_internal.h"

namespace spai {
namespace ttt {

constexpr int kCells = 9;
constexpr uint32_t kFull = 0x1FF;
constexpr uint32_t kNoChildren = 0xFFFFFFFFu;
constexpr int kHid = 64;
constexpr int kMaxBlocks = 16;
constexpr uint32_t kErrNan = 1, kErrCap = 2;

struct State {
    uint16_t x, o;
    uint8_t n, status;
};

SPAI_HD bool x_to_move(uint8_t n) { return (n & 1u) == 0; }

// get_next_state's winner test (tictactoe.rs:145-161): the mover's row, column,
// and the diagonals through the placed cell
SPAI_HD bool wins(uint32_t m, int cell) {
    const int r = cell / 3, c = cell % 3;
    const uint32_t row = 7u << (3 * r), col = 0x49u << c;
    if ((m & row) == row || (m & col) == col) return true;
    if (r == c && (m & 0x111u) == 0x111u) return true;
    if (r + c == 2 && (m & 0x54u) == 0x54u) return true;
    return false;
}

// returns 0, SPAI_ERR_GAME_OVER or SPAI_ERR_ILLEGAL_MOVE; s unchanged on error
SPAI_HD int apply(State &s, int a) {
    if (s.status != 0) return SPAI_ERR_GAME_OVER;
    if (a < 0 || a >= kCells || (((s.x | s.o) >> a) & 1u)) return SPAI_ERR_ILLEGAL_MOVE;
    const bool xm = x_to_move(s.n);
    uint32_t mover;
    if (xm) {
        s.x = (uint16_t)(s.x | (1u << a));
        mover = s.x;
    } else {
        s.o = (uint16_t)(s.o | (1u << a));
        mover = s.o;
    }
    s.n = (uint8_t)(s.n + 1);
    s.status = wins(mover, a) ? SPAI_WON : (s.n == kCells ? SPAI_TIED : SPAI_ONGOING);
    return SPAI_OK;
}

SPAI_HD uint32_t legal(const State &s) { return s.status ? 0u : (~(uint32_t)(s.x | s.o) & kFull); }

SPAI_HD int kth_bit(uint32_t m, int k) {
    for (int i = 0; i < k; ++i) m &= m - 1;
    return __builtin_ctz(m);
}

// ndarray sum of 9 floats (numeric_util::unrolled_fold: one chunk of 8, then the tail)
SPAI_HD float nd_sum9(const float *m) {
    float acc = 0.0f;
    acc = acc + (m[0] + m[4]);
    acc = acc + (m[1] + m[5]);
    acc = acc + (m[2] + m[6]);
    acc = acc + (m[3] + m[7]);
    return acc + m[8];
}

SPAI_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// raw (pre-mask) policy and value of the stub evaluators (oracle: stub_eval / or_hash_eval_raw)
SPAI_HD void stub_raw(int kind, const State &s, float *raw, float *value) {
    if (kind == SPAI_EVAL_UNIFORM) {
        for (int a = 0; a < kCells; ++a) raw[a] = 1.0f / 9.0f;
        *value = 0.0f;
        return;
    }
    const uint64_t h = splitmix64((uint64_t)s.x ^ ((uint64_t)s.o * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)s.n << 58));
    float w[kCells];
    float sum = 0.0f;
    for (int a = 0; a < kCells; ++a) {
        w[a] = (float)(1 + ((h >> (5 * a)) & 31));
        sum = sum + w[a];
    }
    for (int a = 0; a < kCells; ++a) raw[a] = w[a] / sum;
    *value = (float)((int)((h >> 48) & 255) - 127) / 128.0f;
}

// softmax(-1) of the 9 logits (model/mod.rs:63), as the search's expand step
__device__ inline void softmax9(const float *l, float *raw) {
    float mx = l[0];
    for (int a = 1; a < kCells; ++a) mx = fmaxf(mx, l[a]);
    float se = 0.0f;
    for (int a = 0; a < kCells; ++a) se += expf(l[a] - mx);
    for (int a = 0; a < kCells; ++a) raw[a] = expf(l[a] - mx) / se;
}

// mask_invalid_actions (tictactoe.rs:218-236): p * mask / ndarray sum
SPAI_HD void mask9(uint32_t lg, const float *p, float *out) {
    float m[kCells];
    for (int a = 0; a < kCells; ++a) m[a] = p[a] * (((lg >> a) & 1u) ? 1.0f : 0.0f);
    const float sum = nd_sum9(m);
    for (int a = 0; a < kCells; ++a) out[a] = m[a] / sum;
}

// get_encoding (tictactoe.rs:199-216): [3][3][3] current player's, opponent's, empty
SPAI_HD void encode(const State &s, float *out) {
    const uint32_t mine = x_to_move(s.n) ? s.x : s.o, theirs = x_to_move(s.n) ? s.o : s.x;
    for (int c = 0; c < kCells; ++c) {
        out[c] = ((mine >> c) & 1u) ? 1.0f : 0.0f;
        out[9 + c] = ((theirs >> c) & 1u) ? 1.0f : 0.0f;
        out[18 + c] = (((mine | theirs) >> c) & 1u) ? 0.0f : 1.0f;
    }
}

// ---------------------------------------------------------------- net (fp32 VALU)
struct NetW {
    const float *wt;   // per conv: [ci*9 + tap][co] (BN folded), stem, residual, policy conv, value conv
    const float *b;    // per conv: [co]
    const float *pl_w, *pl_b, *vl_w, *vl_b;   // policy linear [9][288], [9]; value linear [27], [1]
    int blocks;
};

// 3x3 conv (pad 1) on a 3x3 board, 512 threads: wave g (of 8) accumulates input
// channels [g*CI/8, (g+1)*CI/8) for output channel o = lane at all 9 cells (a
// weight load feeds 9 FMAs; the wave's 64 loads are one coalesced 256-B read),
// then thread t < co*9 sums the 8 partials in wave order.  Eight short
// dependent load chains instead of one 64-deep chain per thread.
constexpr int kNetWaves = 8;
constexpr int kNetThreads = 64 * kNetWaves;   // 512
template <int CI>
__device__ __forceinline__ void conv3(const float *in, float *out, const float *wt, const float *b, int co, int t,
                                      bool relu, const float *res, float *part) {
    const int o = t & 63, g = t >> 6;
    constexpr int CPG = (CI + kNetWaves - 1) / kNetWaves;   // input channels per wave
    if (o < co) {
        float acc[kCells];
#pragma unroll
        for (int c = 0; c < kCells; ++c) acc[c] = 0.0f;
        for (int ci = g * CPG; ci < CI && ci < (g + 1) * CPG; ++ci)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const float w = wt[(ci * 9 + tap) * co + o];
                const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
                for (int c = 0; c < kCells; ++c) {
                    const int y = c / 3 + dy, x = c % 3 + dx;
                    if ((unsigned)y < 3u && (unsigned)x < 3u) acc[c] = fmaf(w, in[ci * 9 + y * 3 + x], acc[c]);
                }
            }
#pragma unroll
        for (int c = 0; c < kCells; ++c) part[(g * kHid + o) * kCells + c] = acc[c];
    }
    __syncthreads();
    for (int i = t; i < co * kCells; i += kNetThreads) {
        float v = b[i / kCells];
#pragma unroll
        for (int gg = 0; gg < kNetWaves; ++gg) v += part[gg * kHid * kCells + i];
        if (res) v += res[i];
        out[i] = relu ? fmaxf(v, 0.0f) : v;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kNetThreads) void k_tnet(const uint32_t *__restrict__ d_count, uint32_t max_n,
                                                      const float *__restrict__ x, NetW W, float *__restrict__ logits,
                                                      float *__restrict__ value) {
    __shared__ float a[kHid * 9], bb[kHid * 9], cc[kHid * 9], head[32 * 9 + 3 * 9];
    __shared__ float part[kNetWaves * kHid * kCells];
    const uint32_t s = blockIdx.x;
    const uint32_t count = d_count ? min(*d_count, max_n) : max_n;
    if (s >= count) return;
    const int t = threadIdx.x;
    if (t < 27) cc[t] = x[(size_t)s * 27 + t];
    __syncthreads();
    const float *wt = W.wt, *b = W.b;
    conv3<3>(cc, a, wt, b, kHid, t, true, nullptr, part);
    wt += 27 * kHid;
    b += kHid;
    for (int l = 0; l < W.blocks; ++l) {
        conv3<kHid>(a, bb, wt, b, kHid, t, true, nullptr, part);
        wt += 576 * kHid;
        b += kHid;
        conv3<kHid>(bb, a, wt, b, kHid, t, true, a, part);   // relu(x + BN(conv(...))), in place: a is read before
        wt += 576 * kHid;                                    // the partial-sum barrier, written after it
        b += kHid;
    }
    conv3<kHid>(a, head, wt, b, 32, t, true, nullptr, part);                        // policy conv + BN + ReLU
    conv3<kHid>(a, head + 288, wt + 576 * 32, b + 32, 3, t, true, nullptr, part);   // value conv + BN + ReLU
    if (t < kCells) {   // flatten (c*9 + cell) + linear 288 -> 9
        float acc = W.pl_b[t];
        for (int k = 0; k < 288; ++k) acc = fmaf(W.pl_w[t * 288 + k], head[k], acc);
        logits[(size_t)s * kCells + t] = acc;
    }
    if (t == 64) {      // linear 27 -> 1 + tanh (a different wave than the policy lanes)
        float acc = W.vl_b[0];
        for (int k = 0; k < 27; ++k) acc = fmaf(W.vl_w[k], head[288 + k], acc);
        value[s] = tanhf(acc);
    }
}

// ---------------------------------------------------------------- search
struct TV {
    uint4 *nodes;                 // [n][cap]
    uint32_t *root;
    State *root_state;
    uint32_t *next_free;
    uint32_t *path;               // [n][10]
    uint32_t *depth;
    State *leaf;                  // [n]
    uint32_t cap;
};
struct BV {
    uint32_t *tree;
    float *x;                     // [cap][27]
    float *logits, *value;        // [cap][9], [cap]
};
constexpr int kMaxDepth = 10;

__device__ __forceinline__ float ucb(float sq, const uint4 &ch, float c) {   // mcts.rs:91-100
    const uint32_t n = ch.x;
    const float w = __uint_as_float(ch.y), prior = __uint_as_float(ch.z);
    const float q = n == 0 ? 0.0f : ((-w / (float)n) + 1.0f) / 2.0f;
    float u = c * prior;
    u = u * sq;
    u = u / (1.0f + (float)n);
    return q + u;
}

__device__ __forceinline__ void backup(uint4 *nodes, const uint32_t *path, int d, float v, int lane) {
    if (lane <= d) {
        uint32_t *nd = (uint32_t *)(nodes + path[lane]);
        const float sign = ((d - lane) & 1) ? -1.0f : 1.0f;
        nd[0] = nd[0] + 1u;
        nd[1] = __float_as_uint(__uint_as_float(nd[1]) + sign * v);
    }
}

__global__ __launch_bounds__(64) void k_tleaf(TV T, BV B, const uint32_t *__restrict__ active, uint32_t n_active,
                                             float c, uint32_t *count, uint32_t *err) {
    __shared__ uint32_t path[kMaxDepth + 1];
    const uint32_t gi = blockIdx.x;
    if (gi >= n_active) return;
    const int lane = threadIdx.x;
    const uint32_t t = active[gi];
    uint4 *nodes = T.nodes + (size_t)t * T.cap;
    State s = T.root_state[t];
    uint32_t node = T.root[t];
    int d = 0;
    if (lane == 0) path[0] = node;
    uint4 rec = nodes[node];
    while (rec.w != kNoChildren) {
        const uint32_t first = rec.w & 0xFFFFFFu, nch = rec.w >> 24;
        const float sq = sqrtf((float)rec.x);
        uint4 ch = make_uint4(0, 0, 0, 0);
        float u = -INFINITY;
        if ((uint32_t)lane < nch) {
            ch = nodes[first + lane];
            u = ucb(sq, ch, c);
        }
        // NaN on any child: the reference panics (mcts.rs:106-109); stop before the argmax
        if (__ballot(u != u)) {
            if (lane == 0) atomicOr(err, kErrNan);
            return;
        }
        float bu = u;
        int bi = (uint32_t)lane < nch ? lane : -1;
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {   // last max (Iterator::max_by, mcts.rs:110-113)
            const float ou = __shfl_xor(bu, m, 64);
            const int oi = __shfl_xor(bi, m, 64);
            if (oi >= 0 && (bi < 0 || ou > bu || (ou == bu && oi > bi))) {
                bu = ou;
                bi = oi;
            }
        }
        bi = __shfl(bi, 0, 64);
        rec.x = __shfl(ch.x, bi, 64);
        rec.y = __shfl(ch.y, bi, 64);
        rec.z = __shfl(ch.z, bi, 64);
        rec.w = __shfl(ch.w, bi, 64);
        apply(s, kth_bit(legal(s), bi));
        node = first + (uint32_t)bi;
        ++d;
        if (lane == 0) path[d] = node;
    }
    __syncthreads();
    if (s.status != SPAI_ONGOING) {   // terminal: Won -> -1, Tied -> 0 (tictactoe.rs:188-197)
        backup(nodes, path, d, s.status == SPAI_WON ? -1.0f : 0.0f, lane);
        return;
    }
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(count, 1u);
    slot = __shfl(slot, 0, 64);
    if (lane <= d) T.path[(size_t)t * (kMaxDepth + 1) + lane] = path[lane];
    if (lane == 0) {
        B.tree[slot] = t;
        T.depth[t] = (uint32_t)d;
        T.leaf[t] = s;
        encode(s, B.x + (size_t)slot * 27);
    }
}

__global__ __launch_bounds__(64) void k_texpand(TV T, BV B, uint32_t max_n, const uint32_t *__restrict__ count,
                                               int kind, uint32_t *err) {
    const uint32_t s = blockIdx.x;
    if (s >= min(*count, max_n)) return;
    const int lane = threadIdx.x;
    const uint32_t t = B.tree[s];
    uint4 *nodes = T.nodes + (size_t)t * T.cap;
    const int d = (int)T.depth[t];
    const uint32_t *path = T.path + (size_t)t * (kMaxDepth + 1);
    const State st = T.leaf[t];
    const uint32_t lg = legal(st);
    const int n = __builtin_popcount(lg);
    float pri[kCells], raw[kCells], v;
    if (kind == SPAI_EVAL_NET) {   // softmax(-1) then mask (model/mod.rs:62-93)
        softmax9(B.logits + (size_t)s * kCells, raw);
        v = B.value[s];
    } else {
        stub_raw(kind, st, raw, &v);
    }
    mask9(lg, raw, pri);
    const uint32_t first = T.next_free[t];
    if (first + (uint32_t)n > T.cap) {
        if (lane == 0) atomicOr(err, kErrCap);
        return;
    }
    if (lane < n) nodes[first + lane] = make_uint4(0u, 0u, __float_as_uint(pri[kth_bit(lg, lane)]), kNoChildren);
    if (lane == 0) {
        T.next_free[t] = first + (uint32_t)n;
        ((uint32_t *)(nodes + path[d]))[3] = first | ((uint32_t)n << 24);
    }
    backup(nodes, path, d, v, lane);
}

__global__ void k_troot_stats(TV T, const uint32_t *__restrict__ active, uint32_t n_active, uint32_t *out) {
    const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    const uint4 *nodes = T.nodes + (size_t)t * T.cap;
    const uint4 r = nodes[T.root[t]];
    uint32_t *o = out + (size_t)gi * 11;
    const uint32_t nch = r.w == kNoChildren ? 0 : r.w >> 24, first = r.w & 0xFFFFFFu;
    o[0] = nch;
    o[1] = first;
    for (uint32_t k = 0; k < kCells; ++k) o[2 + k] = k < nch ? nodes[first + k].x : 0u;
}

// trees [0, n) -- or the n trees of `list` (streaming refills) -- become one-node trees at the empty board
__global__ void k_ttrees_init(TV T, uint32_t n, const uint32_t *__restrict__ list) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = list ? list[i] : i;
    T.nodes[(size_t)t * T.cap] = make_uint4(0u, 0u, 0u, kNoChildren);
    T.root[t] = 0;
    T.next_free[t] = 1;
    T.root_state[t] = State{0, 0, 0, 0};
}

// Tree::with_root_state (mcts.rs:86-89): tree t becomes a one-node tree rooted at s
__global__ void k_ttree_reset(TV T, uint32_t t, State s) {
    T.nodes[(size_t)t * T.cap] = make_uint4(0u, 0u, 0u, kNoChildren);
    T.root[t] = 0;
    T.next_free[t] = 1;
    T.root_state[t] = s;
}

__global__ void k_tadvance(TV T, const uint32_t *__restrict__ active, uint32_t n_active,
                           const uint32_t *__restrict__ pick, State *out) {
    const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;
    if (gi >= n_active) return;
    const uint32_t t = active[gi];
    const uint4 r = T.nodes[(size_t)t * T.cap + T.root[t]];
    State s = T.root_state[t];
    apply(s, kth_bit(legal(s), (int)pick[gi]));
    T.root[t] = (r.w & 0xFFFFFFu) + pick[gi];
    T.root_state[t] = s;
    out[gi] = s;
}

// rules kernels over slots
__global__ void k_tslots(State *g, uint32_t first, uint32_t n, int op, const int32_t *in, int32_t *rc, uint32_t *mask,
                         float *fout, const float *fin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    State &s = g[first + i];
    if (op == 0) mask[i] = legal(s);
    else if (op == 1) rc[i] = apply(s, in[i]);
    else if (op == 2) encode(s, fout + (size_t)i * 27);
    else if (op == 3) mask9(legal(s), fin + (size_t)i * 9, fout + (size_t)i * 9);
    else {   // Model::predict's tail: softmax, then mask_invalid_actions
        float raw[kCells];
        softmax9(fin + (size_t)i * 9, raw);
        mask9(legal(s), raw, fout + (size_t)i * 9);
    }
}

// ---------------------------------------------------------------- engine
struct Engine {
    int device = 0;
    spai_config cfg{};
    hipStream_t stream = nullptr;
    DevBuf<State> slots;
    uint32_t n_slots = 0;
    DevBuf<int32_t> si;
    DevBuf<uint32_t> su;
    DevBuf<float> sf, sf2;
    // trees
    uint32_t n_trees = 0, cap = 0;
    DevBuf<uint4> nodes;
    DevBuf<uint32_t> root, next_free, path, depth, active, counts, err, stats, pick;
    DevBuf<State> root_state, leaf, adv;
    DevBuf<uint32_t> btree;
    DevBuf<float> bx, blogits, bvalue;
    struct Net *net = nullptr;
};

struct Net {
    Engine *eng = nullptr;
    int blocks = 0;
    DevBuf<float> wt, b, pl_w, pl_b, vl_w, vl_b;
    DevBuf<float> io_x, io_l, io_v;
    uint32_t io_cap = 0;
};

namespace {
TV view(Engine *e) {
    return TV{e->nodes.p, e->root.p, e->root_state.p, e->next_free.p, e->path.p, e->depth.p, e->leaf.p, e->cap};
}
BV bview(Engine *e) { return BV{e->btree.p, e->bx.p, e->blogits.p, e->bvalue.p}; }
NetW wview(const Net *n) {
    return NetW{n->wt.p, n->b.p, n->pl_w.p, n->pl_b.p, n->vl_w.p, n->vl_b.p, n->blocks};
}

size_t num_params(int blocks) {
    auto conv = [](size_t ci, size_t co) { return co * ci * 9 + co + 4 * co; };
    return conv(3, kHid) + (size_t)blocks * 2 * conv(kHid, kHid) + conv(kHid, 32) + 9 * 288 + 9 + conv(kHid, 3) +
           27 + 1;
}

float philox_unit(uint64_t seed, uint32_t tensor, uint64_t idx) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), tensor, 0x5EEDu};
    uint32_t o[4];
    philox4x32(ctr, key, o);
    return (float)(o[0] >> 8) * (1.0f / 16777216.0f);
}

int run_search(Engine *e, uint32_t na, uint32_t sims) {
    if (e->counts.n < sims) SPAI_TRY(e->counts.alloc(sims));
    SPAI_HIP(hipMemsetAsync(e->counts.p, 0, 4 * sims, e->stream));
    const int kind = (int)e->cfg.eval;
    SPAI_CHECK(kind != SPAI_EVAL_NET || e->net, SPAI_ERR_INVALID, "cfg.eval = NET but no net set (spai_ttt_set_net)");
    for (uint32_t it = 0; it < sims; ++it) {
        uint32_t *cnt = e->counts.p + it;
        k_tleaf<<<na, 64, 0, e->stream>>>(view(e), bview(e), e->active.p, na, e->cfg.c, cnt, e->err.p);
        if (kind == SPAI_EVAL_NET)
            k_tnet<<<na, kNetThreads, 0, e->stream>>>(cnt, na, e->bx.p, wview(e->net), e->blogits.p, e->bvalue.p);
        k_texpand<<<na, 64, 0, e->stream>>>(view(e), bview(e), na, cnt, kind, e->err.p);
    }
    SPAI_HIP(hipGetLastError());
    uint32_t f = 0;
    SPAI_HIP(hipMemcpyAsync(&f, e->err.p, 4, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    if (f) {
        SPAI_HIP(hipMemsetAsync(e->err.p, 0, 4, e->stream));   // stream-ordered (the stream is non-blocking)
        if (f & kErrNan) {
            set_error("NaN UCB score (the reference panics, mcts.rs:106-109)");
            return SPAI_ERR_NAN;
        }
        set_error("node arena full");
        return SPAI_ERR_CAPACITY;
    }
    return SPAI_OK;
}

int root_stats(Engine *e, uint32_t na, std::vector<uint32_t> &st) {
    k_troot_stats<<<(na + 63) / 64, 64, 0, e->stream>>>(view(e), e->active.p, na, e->stats.p);
    SPAI_HIP(hipGetLastError());
    st.resize((size_t)na * 11);
    SPAI_HIP(hipMemcpyAsync(st.data(), e->stats.p, 4ull * 11 * na, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int trees_create(Engine *e, uint32_t n) {
    SPAI_CHECK(n >= 1 && n <= e->cfg.max_trees, SPAI_ERR_INVALID, "trees: n=%u (max_trees %u)", n, e->cfg.max_trees);
    const uint32_t cap = 1 + 9 * e->cfg.num_searches * 9;
    if (e->n_trees != n || e->cap != cap) {
        e->n_trees = n;
        e->cap = cap;
        SPAI_TRY(e->nodes.alloc((size_t)n * cap));
        SPAI_TRY(e->root.alloc(n));
        SPAI_TRY(e->next_free.alloc(n));
        SPAI_TRY(e->path.alloc((size_t)n * (kMaxDepth + 1)));
        SPAI_TRY(e->depth.alloc(n));
        SPAI_TRY(e->active.alloc(n));
        SPAI_TRY(e->stats.alloc((size_t)n * 11));
        SPAI_TRY(e->pick.alloc(n));
        SPAI_TRY(e->root_state.alloc(n));
        SPAI_TRY(e->leaf.alloc(n));
        SPAI_TRY(e->adv.alloc(n));
        SPAI_TRY(e->btree.alloc(n));
        SPAI_TRY(e->bx.alloc((size_t)n * 27));
        SPAI_TRY(e->blogits.alloc((size_t)n * 9));
        SPAI_TRY(e->bvalue.alloc(n));
    }
    k_ttrees_init<<<(n + 63) / 64, 64, 0, e->stream>>>(view(e), n, nullptr);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

// visit policy (mcts.rs:318-328): set_prob(action, N), normalize (ndarray sum)
void visit_policy(const State &root, const uint32_t *st, float *pol, uint32_t *ids, float *vis) {
    float m[kCells] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t nch = st[0], lg = legal(root);
    for (uint32_t k = 0; k < nch; ++k) {
        m[kth_bit(lg, (int)k)] = (float)st[2 + k];
        if (ids) ids[k] = st[1] + k;
        if (vis) vis[k] = (float)st[2 + k];
    }
    const float sum = nd_sum9(m);
    if (pol)
        for (int a = 0; a < kCells; ++a) pol[a] = m[a] / sum;
}
}  // namespace

}  // namespace ttt
}  // namespace spai

struct spai_ttt : spai::ttt::Engine {};
struct spai_ttt_net : spai::ttt::Net {};

using namespace spai;
using namespace spai::ttt;

#define T_CHECK(e)                                                    \
    do {                                                              \
        if (!(e)) {                                                   \
            set_error("null handle");                                 \
            return SPAI_ERR_INVALID;                                  \
        }                                                             \
        if (hipSetDevice((e)->device) != hipSuccess) {                \
            set_error("hipSetDevice(%d) failed", (e)->device);        \
            return SPAI_ERR_DEVICE;                                   \
        }                                                             \
    } while (0)
#define T_PTR(p)                                                      \
    do {                                                              \
        if (!(p)) {                                                   \
            set_error("%s must not be NULL", #p);                     \
            return SPAI_ERR_INVALID;                                  \
        }                                                             \
    } while (0)

static State ttt_from_abi(const spai_ttt_state &s) { return State{s.x, s.o, s.num_actions_played, s.status}; }
static spai_ttt_state ttt_to_abi(const State &s) {
    spai_ttt_state r{};
    r.x = s.x;
    r.o = s.o;
    r.num_actions_played = s.n;
    r.status = s.status;
    return r;
}

static int slots_op(spai_ttt *e, uint32_t first, uint32_t n, int op, const int32_t *in, int32_t *rc, uint32_t *mask,
                    float *fout, const float *fin) {
    SPAI_CHECK((uint64_t)first + n <= e->n_slots, SPAI_ERR_INVALID, "slots [%u, %u) out of range (%u)", first,
               first + n, e->n_slots);
    if (!n) return SPAI_OK;
    if (in) SPAI_HIP(hipMemcpyAsync(e->si.p, in, 4 * n, hipMemcpyHostToDevice, e->stream));
    if (fin) SPAI_HIP(hipMemcpyAsync(e->sf2.p, fin, 36ull * n, hipMemcpyHostToDevice, e->stream));
    k_tslots<<<(n + 63) / 64, 64, 0, e->stream>>>(e->slots.p, first, n, op, e->si.p, e->si.p, e->su.p, e->sf.p,
                                                  e->sf2.p);
    SPAI_HIP(hipGetLastError());
    if (rc) SPAI_HIP(hipMemcpyAsync(rc, e->si.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (mask) SPAI_HIP(hipMemcpyAsync(mask, e->su.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    if (fout) SPAI_HIP(hipMemcpyAsync(fout, e->sf.p, (op == 2 ? 108ull : 36ull) * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

extern "C" {

int spai_ttt_create(const spai_config *cfg, int device, spai_ttt **out) {
    T_PTR(cfg);
    T_PTR(out);
    SPAI_CHECK(cfg->eval <= SPAI_EVAL_HASH, SPAI_ERR_INVALID, "bad eval kind %u", cfg->eval);
    SPAI_CHECK(cfg->max_trees >= 1 && cfg->num_searches >= 1 && cfg->num_searches <= (1u << 20), SPAI_ERR_INVALID,
               "max_trees and num_searches must be >= 1");
    int ndev = 0;
    SPAI_HIP(hipGetDeviceCount(&ndev));
    SPAI_CHECK(device >= 0 && device < ndev, SPAI_ERR_DEVICE, "device %d not present (%d visible)", device, ndev);
    SPAI_HIP(hipSetDevice(device));
    spai_ttt *e = new (std::nothrow) spai_ttt();
    SPAI_CHECK(e, SPAI_ERR_INVALID, "out of host memory");
    e->device = device;
    e->cfg = *cfg;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess || e->err.alloc(1) != SPAI_OK ||
        hipMemsetAsync(e->err.p, 0, 4, e->stream) != hipSuccess) {
        set_error("ttt engine stream / scratch allocation failed");
        delete e;
        return SPAI_ERR_DEVICE;
    }
    *out = e;
    return SPAI_OK;
}

int spai_ttt_destroy(spai_ttt *e) {
    if (!e) return SPAI_OK;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    for (auto *d : {&e->slots, &e->root_state, &e->leaf, &e->adv}) d->release();
    for (auto *d : {&e->su, &e->root, &e->next_free, &e->path, &e->depth, &e->active, &e->counts, &e->err, &e->stats,
                    &e->pick, &e->btree})
        d->release();
    for (auto *d : {&e->sf, &e->sf2, &e->bx, &e->blogits, &e->bvalue}) d->release();
    e->si.release();
    e->nodes.release();
    (void)hipStreamDestroy(e->stream);
    delete e;
    return SPAI_OK;
}

int spai_ttt_games_resize(spai_ttt *e, uint32_t n) {
    T_CHECK(e);
    SPAI_TRY(e->slots.alloc(n));
    SPAI_TRY(e->si.alloc(n));
    SPAI_TRY(e->su.alloc(n));
    SPAI_TRY(e->sf.alloc((size_t)n * 27));
    SPAI_TRY(e->sf2.alloc((size_t)n * 9));
    e->n_slots = n;
    if (n) {
        // on the engine's (non-blocking) stream: a plain hipMemset is not ordered before the
        // rules kernels that stream launches next, and one GPU run read the slots unzeroed
        SPAI_HIP(hipMemsetAsync(e->slots.p, 0, sizeof(State) * n, e->stream));
        SPAI_HIP(hipStreamSynchronize(e->stream));
    }
    return SPAI_OK;
}

int spai_ttt_games_write(spai_ttt *e, uint32_t first, uint32_t n, const spai_ttt_state *s) {
    T_CHECK(e);
    SPAI_CHECK((uint64_t)first + n <= e->n_slots, SPAI_ERR_INVALID, "slots out of range");
    std::vector<State> h(n);
    for (uint32_t i = 0; i < n; ++i) {
        h[i] = ttt_from_abi(s[i]);
        SPAI_CHECK(!(h[i].x & h[i].o) && h[i].x <= kFull && h[i].o <= kFull, SPAI_ERR_INVALID, "bad board %u", i);
    }
    if (n) SPAI_HIP(hipMemcpy(e->slots.p + first, h.data(), sizeof(State) * n, hipMemcpyHostToDevice));
    return SPAI_OK;
}

int spai_ttt_games_read(spai_ttt *e, uint32_t first, uint32_t n, spai_ttt_state *s) {
    T_CHECK(e);
    SPAI_CHECK((uint64_t)first + n <= e->n_slots, SPAI_ERR_INVALID, "slots out of range");
    std::vector<State> h(n);
    if (n) SPAI_HIP(hipMemcpy(h.data(), e->slots.p + first, sizeof(State) * n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) s[i] = ttt_to_abi(h[i]);
    return SPAI_OK;
}

int spai_ttt_legal_mask(spai_ttt *e, uint32_t first, uint32_t n, uint32_t *mask) {
    T_CHECK(e);
    return slots_op(e, first, n, 0, nullptr, nullptr, mask, nullptr, nullptr);
}

int spai_ttt_apply(spai_ttt *e, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc) {
    T_CHECK(e);
    std::vector<int32_t> r(n);
    SPAI_TRY(slots_op(e, first, n, 1, actions, r.data(), nullptr, nullptr, nullptr));
    int err = SPAI_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (rc) rc[i] = r[i];
        if (r[i] && err == SPAI_OK) err = r[i];
    }
    if (err == SPAI_ERR_GAME_OVER) set_error("Game has already ended");
    if (err == SPAI_ERR_ILLEGAL_MOVE) set_error("Illegal move: cell already occupied");
    return err;
}

int spai_ttt_encode(spai_ttt *e, uint32_t first, uint32_t n, float *out) {
    T_CHECK(e);
    return slots_op(e, first, n, 2, nullptr, nullptr, nullptr, out, nullptr);
}

int spai_ttt_mask_invalid(spai_ttt *e, uint32_t first, uint32_t n, const float *policy, uint32_t len, float *out) {
    T_CHECK(e);
    SPAI_CHECK(len == 9, SPAI_ERR_INVALID, "Expected policy shape to be (9,), found (%u,)", len);
    return slots_op(e, first, n, 3, nullptr, nullptr, nullptr, out, policy);
}

int spai_ttt_net_num_params(int blocks, size_t *count) {
    T_PTR(count);
    *count = num_params(blocks);
    return SPAI_OK;
}

// tch 0.13 default init (as spai_net_init_params), Philox keyed by (seed, tensor, index)
int spai_ttt_net_init_params(int blocks, uint64_t seed, float *params) {
    T_PTR(params);
    uint32_t t = 0;
    float *p = params;
    auto uni = [&](size_t n, float lo, float hi) {
        for (size_t i = 0; i < n; ++i) p[i] = lo + (hi - lo) * philox_unit(seed, t, i);
        p += n;
        ++t;
    };
    auto cst = [&](size_t n, float v) {
        for (size_t i = 0; i < n; ++i) p[i] = v;
        p += n;
        ++t;
    };
    auto conv = [&](int ci, int co) {
        const float b = (float)std::sqrt(6.0 / (double)(ci * 9));
        uni((size_t)co * ci * 9, -b, b);
        cst(co, 0.f);
        uni(co, 0.f, 1.f);
        cst(co, 0.f);
        cst(co, 0.f);
        cst(co, 1.f);
    };
    auto lin = [&](int in, int out) {
        const float b = (float)std::sqrt(6.0 / (double)in), bb = (float)(1.0 / std::sqrt((double)in));
        uni((size_t)out * in, -b, b);
        uni(out, -bb, bb);
    };
    conv(3, kHid);
    for (int i = 0; i < 2 * blocks; ++i) conv(kHid, kHid);
    conv(kHid, 32);
    lin(288, 9);
    conv(kHid, 3);
    lin(27, 1);
    return SPAI_OK;
}

int spai_ttt_net_create(spai_ttt *e, int blocks, const float *params, size_t n, spai_ttt_net **out) {
    T_CHECK(e);
    T_PTR(out);
    T_PTR(params);
    SPAI_CHECK(blocks >= 0 && blocks <= kMaxBlocks, SPAI_ERR_UNSUPPORTED, "ttt net: 0..%d blocks", kMaxBlocks);
    SPAI_CHECK(n == num_params(blocks), SPAI_ERR_INVALID, "expected %zu params, got %zu", num_params(blocks), n);
    std::vector<float> wt, b;
    const float *p = params;
    // conv + BN (eval) folded in double, weights transposed to [ci*9 + tap][co]
    auto conv = [&](int ci, int co) {
        const float *w = p, *bias = p + (size_t)co * ci * 9, *bn = bias + co;
        p = bn + 4 * co;
        const size_t base = wt.size();
        wt.resize(base + (size_t)ci * 9 * co);
        for (int o = 0; o < co; ++o) {
            const double sc = (double)bn[o] / std::sqrt((double)bn[3 * co + o] + 1e-5);
            b.push_back((float)(((double)bias[o] - (double)bn[2 * co + o]) * sc + (double)bn[co + o]));
            for (int k = 0; k < ci * 9; ++k) wt[base + (size_t)k * co + o] = (float)((double)w[(size_t)o * ci * 9 + k] * sc);
        }
    };
    conv(3, kHid);
    for (int i = 0; i < 2 * blocks; ++i) conv(kHid, kHid);
    conv(kHid, 32);
    std::vector<float> pl_w(p, p + 9 * 288), pl_b(p + 9 * 288, p + 9 * 288 + 9);
    p += 9 * 288 + 9;
    conv(kHid, 3);
    std::vector<float> vl_w(p, p + 27), vl_b(p + 27, p + 28);
    p += 28;
    spai_ttt_net *net = new spai_ttt_net();
    net->eng = e;
    net->blocks = blocks;
    auto up = [&](DevBuf<float> &d, const std::vector<float> &h) -> int {
        SPAI_TRY(d.alloc(h.size()));
        SPAI_HIP(hipMemcpy(d.p, h.data(), 4 * h.size(), hipMemcpyHostToDevice));
        return SPAI_OK;
    };
    int rc = up(net->wt, wt);
    if (rc == SPAI_OK) rc = up(net->b, b);
    if (rc == SPAI_OK) rc = up(net->pl_w, pl_w);
    if (rc == SPAI_OK) rc = up(net->pl_b, pl_b);
    if (rc == SPAI_OK) rc = up(net->vl_w, vl_w);
    if (rc == SPAI_OK) rc = up(net->vl_b, vl_b);
    if (rc != SPAI_OK) {
        delete net;
        return rc;
    }
    *out = net;
    return SPAI_OK;
}

int spai_ttt_net_destroy(spai_ttt_net *net) {
    if (!net) return SPAI_OK;
    (void)hipSetDevice(net->eng->device);
    if (net->eng->net == net) net->eng->net = nullptr;
    for (auto *d : {&net->wt, &net->b, &net->pl_w, &net->pl_b, &net->vl_w, &net->vl_b, &net->io_x, &net->io_l,
                    &net->io_v})
        d->release();
    delete net;
    return SPAI_OK;
}

int spai_ttt_net_forward(spai_ttt_net *net, uint32_t n, const float *x, float *logits, float *value) {
    T_PTR(net);
    T_CHECK(net->eng);
    if (!n) return SPAI_OK;
    T_PTR(x);
    T_PTR(logits);
    T_PTR(value);
    spai_ttt *e = static_cast<spai_ttt *>(net->eng);
    if (net->io_cap < n) {
        SPAI_TRY(net->io_x.alloc((size_t)n * 27));
        SPAI_TRY(net->io_l.alloc((size_t)n * 9));
        SPAI_TRY(net->io_v.alloc(n));
        net->io_cap = n;
    }
    SPAI_HIP(hipMemcpyAsync(net->io_x.p, x, 108ull * n, hipMemcpyHostToDevice, e->stream));
    k_tnet<<<n, kNetThreads, 0, e->stream>>>(nullptr, n, net->io_x.p, wview(net), net->io_l.p, net->io_v.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(logits, net->io_l.p, 36ull * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(value, net->io_v.p, 4ull * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

// Model::predict (model/mod.rs:36-98) over game slots [first, first+n)
int spai_ttt_predict(spai_ttt_net *net, uint32_t first, uint32_t n, float *priors, float *values) {
    T_PTR(net);
    T_CHECK(net->eng);
    spai_ttt *e = static_cast<spai_ttt *>(net->eng);
    SPAI_CHECK((uint64_t)first + n <= e->n_slots, SPAI_ERR_INVALID, "slots [%u, %u) out of range (%u)", first,
               first + n, e->n_slots);
    if (!n) return SPAI_OK;
    T_PTR(priors);
    T_PTR(values);
    if (net->io_cap < n) {
        SPAI_TRY(net->io_x.alloc((size_t)n * 27));
        SPAI_TRY(net->io_l.alloc((size_t)n * 9));
        SPAI_TRY(net->io_v.alloc(n));
        net->io_cap = n;
    }
    const uint32_t g = (n + 63) / 64;
    k_tslots<<<g, 64, 0, e->stream>>>(e->slots.p, first, n, 2, nullptr, nullptr, nullptr, net->io_x.p, nullptr);
    k_tnet<<<n, kNetThreads, 0, e->stream>>>(nullptr, n, net->io_x.p, wview(net), net->io_l.p, net->io_v.p);
    k_tslots<<<g, 64, 0, e->stream>>>(e->slots.p, first, n, 4, nullptr, nullptr, nullptr, e->sf2.p, net->io_l.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(priors, e->sf2.p, 36ull * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(values, net->io_v.p, 4ull * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int spai_ttt_set_net(spai_ttt *e, spai_ttt_net *net) {
    T_CHECK(e);
    SPAI_CHECK(!net || net->eng == e, SPAI_ERR_INVALID, "net belongs to another engine");
    e->net = net;
    return SPAI_OK;
}

int spai_ttt_trees_create(spai_ttt *e, uint32_t n) {
    T_CHECK(e);
    return trees_create(e, n);
}

int spai_ttt_search(spai_ttt *e, uint32_t n, const uint32_t *tree_idx, uint32_t num_searches, float *policy,
                    uint32_t *child_ids, float *child_visits, uint32_t *n_children) {
    T_CHECK(e);
    T_PTR(tree_idx);
    SPAI_CHECK(e->n_trees > 0 && n >= 1 && n <= e->n_trees, SPAI_ERR_INVALID, "search: n=%u trees (have %u)", n,
               e->n_trees);
    SPAI_CHECK(num_searches <= e->cfg.num_searches, SPAI_ERR_INVALID, "num_searches > cfg.num_searches");
    for (uint32_t i = 0; i < n; ++i) SPAI_CHECK(tree_idx[i] < e->n_trees, SPAI_ERR_INVALID, "tree index out of range");
    SPAI_HIP(hipMemcpyAsync(e->active.p, tree_idx, 4 * n, hipMemcpyHostToDevice, e->stream));
    SPAI_TRY(run_search(e, n, num_searches));
    std::vector<uint32_t> st;
    SPAI_TRY(root_stats(e, n, st));
    std::vector<State> roots(e->n_trees);
    SPAI_HIP(hipMemcpy(roots.data(), e->root_state.p, sizeof(State) * e->n_trees, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        visit_policy(roots[tree_idx[i]], st.data() + 11 * i, policy ? policy + 9 * i : nullptr,
                     child_ids ? child_ids + 9 * i : nullptr, child_visits ? child_visits + 9 * i : nullptr);
        if (n_children) n_children[i] = st[11 * i];
    }
    return SPAI_OK;
}

int spai_ttt_tree_reset(spai_ttt *e, uint32_t tree, const spai_ttt_state *root) {
    T_CHECK(e);
    T_PTR(root);
    SPAI_CHECK(tree < e->n_trees, SPAI_ERR_INVALID, "tree %u out of range (%u trees)", tree, e->n_trees);
    const State st = ttt_from_abi(*root);
    SPAI_CHECK(!(st.x & st.o) && st.x <= kFull && st.o <= kFull && st.status <= SPAI_WON, SPAI_ERR_INVALID,
               "bad TicTacToe state");
    k_ttree_reset<<<1, 1, 0, e->stream>>>(view(e), tree, st);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int spai_ttt_tree_use_subtree(spai_ttt *e, uint32_t tree, uint32_t child_index) {
    T_CHECK(e);
    SPAI_CHECK(tree < e->n_trees, SPAI_ERR_INVALID, "tree out of range");
    SPAI_HIP(hipMemcpyAsync(e->active.p, &tree, 4, hipMemcpyHostToDevice, e->stream));
    std::vector<uint32_t> st;
    SPAI_TRY(root_stats(e, 1, st));
    SPAI_CHECK(child_index < st[0], SPAI_ERR_INVALID, "child index %u >= %u root children", child_index, st[0]);
    SPAI_HIP(hipMemcpyAsync(e->pick.p, &child_index, 4, hipMemcpyHostToDevice, e->stream));
    k_tadvance<<<1, 64, 0, e->stream>>>(view(e), e->active.p, 1, e->pick.p, e->adv.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

}  // extern "C"

namespace {
// SelfPlayWorker::self_play (learner_concurrent.rs:169-242); window < n_games: the
// games through `window` tree slots, a slot whose game ended taking the next game
// (a fresh empty-board tree), each game's draws keyed by its id and own move number
int ttt_selfplay(spai_ttt *e, uint32_t n_games, uint64_t gid_base, spai_sample_sink sink, void *user,
                 spai_selfplay_stats *stats, uint32_t window) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t W = (window == 0 || window >= n_games) ? n_games : window;   // tree slots
    SPAI_TRY(trees_create(e, W));
    const uint32_t sims = e->cfg.num_searches;
    std::vector<uint32_t> slot_game(W), slot_move(W, 0);
    for (uint32_t i = 0; i < W; ++i) slot_game[i] = i;
    uint32_t next_game = W;
    struct Rec {
        State s;
        float pol[9];
        int32_t move;
    };
    std::vector<std::vector<Rec>> hist(W);
    std::vector<uint32_t> act(W);
    std::vector<uint32_t> refill;   // streaming: the slots reset at the end of a move
    std::vector<State> roots(W, State{0, 0, 0, 0});
    for (uint32_t i = 0; i < W; ++i) act[i] = i;
    double sims_done = 0, evals = 0, games = 0, positions = 0, moves = 0;
    std::vector<uint32_t> st, pick, cnt;
    std::vector<State> nb;
    while (!act.empty()) {
        const uint32_t na = (uint32_t)act.size();
        SPAI_HIP(hipMemcpyAsync(e->active.p, act.data(), 4 * na, hipMemcpyHostToDevice, e->stream));
        SPAI_TRY(run_search(e, na, sims));
        cnt.resize(sims);
        SPAI_HIP(hipMemcpy(cnt.data(), e->counts.p, 4 * sims, hipMemcpyDeviceToHost));
        for (uint32_t c : cnt) evals += c;
        sims_done += (double)na * sims;
        moves += 1;
        SPAI_TRY(root_stats(e, na, st));
        pick.assign(na, 0);
        for (int k = (int)na - 1; k >= 0; --k) {   // for i in (0..trees_vec.len()).rev()
            const uint32_t t = act[k];
            const uint32_t *s = st.data() + 11 * k;
            float vis[9];
            Rec r;
            r.s = roots[t];
            visit_policy(roots[t], s, r.pol, nullptr, vis);
            const float u = sample_u01_f32(e->cfg.seed, gid_base + slot_game[t], slot_move[t]++);
            const int idx = weighted_index(vis, (int)s[0], e->cfg.temperature, u);
            SPAI_CHECK(idx >= 0, SPAI_ERR_NAN, "WeightedIndex over all-zero visits (the reference panics)");
            pick[k] = (uint32_t)idx;
            r.move = kth_bit(legal(roots[t]), idx);
            hist[t].push_back(r);
        }
        SPAI_HIP(hipMemcpyAsync(e->pick.p, pick.data(), 4 * na, hipMemcpyHostToDevice, e->stream));
        k_tadvance<<<(na + 63) / 64, 64, 0, e->stream>>>(view(e), e->active.p, na, e->pick.p, e->adv.p);
        SPAI_HIP(hipGetLastError());
        nb.resize(na);
        SPAI_HIP(hipMemcpyAsync(nb.data(), e->adv.p, sizeof(State) * na, hipMemcpyDeviceToHost, e->stream));
        SPAI_HIP(hipStreamSynchronize(e->stream));
        std::vector<char> done(na, 0);
        for (int k = (int)na - 1; k >= 0; --k) {
            const uint32_t t = act[k];
            roots[t] = nb[k];
            if (nb[k].status == SPAI_ONGOING) continue;
            done[k] = 1;
            const float v = nb[k].status == SPAI_WON ? -1.0f : 0.0f;   // tictactoe.rs:188-197
            const bool cur_x = x_to_move(nb[k].n);
            const auto &H = hist[t];
            const size_t m = H.size();
            games += 1;
            positions += (double)m;
            if (sink) {
                std::vector<float> enc(m * 27), pol(m * 9), val(m);
                std::vector<int32_t> mv(m);
                for (size_t h = 0; h < m; ++h) {
                    encode(H[h].s, enc.data() + 27 * h);
                    memcpy(pol.data() + 9 * h, H[h].pol, 36);
                    val[h] = x_to_move(H[h].s.n) == cur_x ? v : -v;
                    mv[h] = H[h].move;
                }
                sink(user, (uint32_t)(gid_base + slot_game[t]), (uint32_t)m, enc.data(), pol.data(), val.data(),
                     mv.data());
            }
            hist[t].clear();
        }
        std::vector<uint32_t> keep;
        for (uint32_t k = 0; k < na; ++k)
            if (!done[k]) keep.push_back(act[k]);
        refill.clear();
        for (uint32_t k = 0; k < na && next_game < n_games; ++k)   // streaming: refill the ended games' slots
            if (done[k]) {
                const uint32_t t = act[k];
                slot_game[t] = next_game++;
                slot_move[t] = 0;
                roots[t] = State{0, 0, 0, 0};
                refill.push_back(t);
                keep.push_back(t);
            }
        if (!refill.empty()) {   // one launch resets every refilled slot (stream order: before the next search's
                                 // upload of the active list into the same buffer)
            const uint32_t nr = (uint32_t)refill.size();
            SPAI_HIP(hipMemcpyAsync(e->active.p, refill.data(), 4 * nr, hipMemcpyHostToDevice, e->stream));
            k_ttrees_init<<<(nr + 255) / 256, 256, 0, e->stream>>>(view(e), nr, e->active.p);
            SPAI_HIP(hipGetLastError());
        }
        act.swap(keep);
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
}  // namespace

extern "C" {

int spai_ttt_selfplay_run(spai_ttt *e, uint32_t n_games, uint64_t gid_base, spai_sample_sink sink, void *user,
                          spai_selfplay_stats *stats) {
    T_CHECK(e);
    return ttt_selfplay(e, n_games, gid_base, sink, user, stats, 0);
}

int spai_ttt_selfplay_stream(spai_ttt *e, uint32_t n_games, uint32_t window, uint64_t gid_base, spai_sample_sink sink,
                             void *user, spai_selfplay_stats *stats) {
    T_CHECK(e);
    SPAI_CHECK(window > 0, SPAI_ERR_INVALID, "window must be > 0");
    return ttt_selfplay(e, n_games, gid_base, sink, user, stats, window);
}

}  // extern "C"

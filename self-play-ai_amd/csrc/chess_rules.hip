// chess_rules.hip — the chess State trait (game/chess.rs:101-299) batched over
// engine-held game slots, one wavefront per slot (wave_movegen in chess.h).
//
// Each slot carries its transposition table as 64-bit hashes of the ordered
// legal-move lists of its earlier positions (chess.rs:27-29,51-61,121-122).
#include <cstring>

#include "chess_engine.h"

namespace spai {
namespace chess {
namespace {

constexpr int kWavesPerBlock = 4;

// get_num_repetitions (chess.rs:51-61): 1 + entries of the table equal to the
// current list (hash compare), lanes striding over the table.
__device__ __forceinline__ uint32_t count_matches(uint64_t h, const uint64_t *tab, uint32_t n, int lane) {
    uint32_t c = 0;
    for (uint32_t i = lane; i < n; i += 64) c += tab[i] == h ? 1u : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    return c;
}

// get_status (chess.rs:150-166): Checkmate -> Won, Stalemate -> Tied, then
// threefold (by the repetition count) or fifty-move counter >= 100 -> Tied
__device__ __forceinline__ int status_of(const GenOut &g, uint32_t reps, const Board &b) {
    if (g.n == 0) return g.in_check ? SPAI_WON : SPAI_TIED;
    if (reps >= 3 || b.fifty >= 100) return SPAI_TIED;
    return SPAI_ONGOING;
}

__global__ void k_slots_status(const Board *__restrict__ boards, const uint64_t *__restrict__ hist,
                               const uint32_t *__restrict__ n_hist, uint32_t max_hist, uint32_t first, uint32_t n,
                               uint16_t *moves, uint32_t *counts, uint8_t *status, uint32_t *reps_out) {
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t s = first + i;
    const Board b = boards[s];
    const GenOut g = wave_movegen(b, moves ? moves + (size_t)i * kMaxMoves : nullptr, lane);
    const uint32_t reps = 1 + count_matches(g.hash, hist + (size_t)s * max_hist, n_hist[s], lane);
    if (lane == 0) {
        if (counts) counts[i] = (uint32_t)g.n;
        if (status) status[i] = (uint8_t)status_of(g, reps, b);
        if (reps_out) reps_out[i] = reps;
    }
}

// get_next_state in place (chess.rs:108-146)
__global__ void k_slots_apply(Board *__restrict__ boards, uint64_t *__restrict__ hist, uint32_t *__restrict__ n_hist,
                              uint32_t max_hist, uint32_t first, uint32_t n, const uint16_t *__restrict__ mv_in,
                              int32_t *rc) {
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t s = first + i;
    Board b = boards[s];
    const int mv = mv_in[i];
    bool found = false;
    const GenOut g = wave_movegen(b, lane, [&](int, int m) { found |= m == mv; });
    found = __any(found);
    const uint32_t nh = n_hist[s];
    const uint32_t reps = 1 + count_matches(g.hash, hist + (size_t)s * max_hist, nh, lane);
    int code = SPAI_OK;
    if (status_of(g, reps, b) != SPAI_ONGOING) code = SPAI_ERR_GAME_OVER;
    else if (!found) code = SPAI_ERR_ILLEGAL_MOVE;
    else if (nh >= max_hist) code = SPAI_ERR_CAPACITY;
    if (lane == 0) {
        rc[i] = code;
        if (code == SPAI_OK) {
            hist[(size_t)s * max_hist + nh] = g.hash;
            n_hist[s] = nh + 1;
            apply_move(b, mv);
            boards[s] = b;
        }
    }
}

// get_encoding (chess.rs:176-249): lane = (row, col) cell of the side to move's view
__device__ __forceinline__ void encode_cell(const Board &b, uint32_t reps, int lane, float v[kPlanes]) {
    const int me = b.side;
    const int row = lane >> 3, col = lane & 7;
    const int rank = me == WHITE ? row : 7 - row;
    const int sq = rank * 8 + col;
    const bb mine = me == WHITE ? b.col[WHITE] : b.col[BLACK];
    const bb theirs = me == WHITE ? b.col[BLACK] : b.col[WHITE];
#pragma unroll
    for (int p = 0; p < 6; ++p) {
        v[p] = ((b.pc[p] & mine) >> sq) & 1 ? 1.0f : 0.0f;
        v[6 + p] = ((b.pc[p] & theirs) >> sq) & 1 ? 1.0f : 0.0f;
    }
    const int ck = me == WHITE ? 1 : 4, cq = me == WHITE ? 2 : 8, tk = me == WHITE ? 4 : 1, tq = me == WHITE ? 8 : 2;
    v[12] = (b.castle & ck) ? 1.0f : 0.0f;
    v[13] = (b.castle & cq) ? 1.0f : 0.0f;
    v[14] = (b.castle & tk) ? 1.0f : 0.0f;
    v[15] = (b.castle & tq) ? 1.0f : 0.0f;
    v[16] = (float)reps;
    v[17] = (float)b.fifty / 100.0f;
    v[18] = (float)(b.made / 2) / 50.0f;
}

__global__ void k_slots_encode(const Board *__restrict__ boards, const uint64_t *__restrict__ hist,
                               const uint32_t *__restrict__ n_hist, uint32_t max_hist, uint32_t first, uint32_t n,
                               float *out) {
    const int lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t s = first + i;
    const Board b = boards[s];
    const GenOut g = wave_movegen(b, nullptr, lane);
    const uint32_t reps = 1 + count_matches(g.hash, hist + (size_t)s * max_hist, n_hist[s], lane);
    float v[kPlanes];
    encode_cell(b, reps, lane, v);
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) out[(size_t)i * kPlanes * 64 + p * 64 + lane] = v[p];
}

// mask_invalid_actions (chess.rs:252-275): p * mask, then / ndarray sum (the
// 8-way unrolled fold of numeric_util, as oracle/spai_oracle.c or_nd_sum), so
// the result is bit-identical to the reference's arithmetic given p.  One wave
// per slot; prob(j) yields the unmasked policy entry j.
template <class P>
__device__ __forceinline__ void masked_normalize(const Board &b, int lane, P &&prob, float *m, float *part, float *o) {
    for (int j = lane; j < kPolicy; j += 64) m[j] = prob(j) * 0.0f;
    __syncthreads();
    wave_movegen(b, lane, [&](int, int mv) {
        const int idx = policy_index(b.side, mv);
        m[idx] = prob(idx) * 1.0f;
    });
    __syncthreads();
    if (lane < 8) {
        float acc = 0.0f;
        for (int j = lane; j < kPolicy; j += 8) acc = acc + m[j];
        part[lane] = acc;
    }
    __syncthreads();
    float sum = 0.0f;
    sum = sum + (part[0] + part[4]);
    sum = sum + (part[1] + part[5]);
    sum = sum + (part[2] + part[6]);
    sum = sum + (part[3] + part[7]);
    for (int j = lane; j < kPolicy; j += 64) o[j] = m[j] / sum;
}

__global__ void __launch_bounds__(64) k_slots_mask(const Board *__restrict__ boards, uint32_t first, uint32_t n,
                                                   const float *__restrict__ pol, float *out) {
    __shared__ float m[kPolicy];
    __shared__ float part[8];
    const int lane = threadIdx.x;
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const float *p = pol + (size_t)i * kPolicy;
    masked_normalize(boards[first + i], lane, [&](int j) { return p[j]; }, m, part, out + (size_t)i * kPolicy);
}

// Model::predict's tail (model/mod.rs:62-93): softmax(-1) over the 4672 logits
// (same reduction order as k_cexpand, so predict and search see the same
// priors), then mask_invalid_actions.
__global__ void __launch_bounds__(64) k_slots_softmax_mask(const Board *__restrict__ boards, uint32_t first,
                                                           uint32_t n, const float *__restrict__ logits, float *out) {
    __shared__ float m[kPolicy];
    __shared__ float part[8];
    const int lane = threadIdx.x;
    const uint32_t i = blockIdx.x;
    if (i >= n) return;
    const float *lg = logits + (size_t)i * kPolicy;
    float mx = -INFINITY;
    for (int j = lane; j < kPolicy; j += 64) mx = fmaxf(mx, lg[j]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float se = 0.0f;
    for (int j = lane; j < kPolicy; j += 64) se += expf(lg[j] - mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
    masked_normalize(boards[first + i], lane, [&](int j) { return expf(lg[j] - mx) / se; }, m, part,
                     out + (size_t)i * kPolicy);
}

}  // namespace

Board from_abi(const spai_chess_state &s) {
    Board b{};
    for (int p = 0; p < 6; ++p) b.pc[p] = s.pieces[p];
    b.col[0] = s.colors[0];
    b.col[1] = s.colors[1];
    b.side = s.side;
    b.castle = s.castle;
    b.ep = s.ep;
    b.status = 0;
    b.fifty = s.fifty;
    b.made = s.made;
    return b;
}

spai_chess_state to_abi(const Board &b, uint32_t reps) {
    spai_chess_state s{};
    for (int p = 0; p < 6; ++p) s.pieces[p] = b.pc[p];
    s.colors[0] = b.col[0];
    s.colors[1] = b.col[1];
    s.side = b.side;
    s.castle = b.castle;
    s.ep = b.ep;
    s.status = b.status;
    s.fifty = b.fifty;
    s.made = b.made;
    s.reps = reps;
    return s;
}

void encode_host(const Board &b, uint32_t reps, float *out) {
    const int me = b.side;
    const bb mine = b.col[me], theirs = b.col[me ^ 1];
    for (int cell = 0; cell < 64; ++cell) {
        const int row = cell >> 3, col = cell & 7;
        const int sq = (me == WHITE ? row : 7 - row) * 8 + col;
        for (int p = 0; p < 6; ++p) {
            out[p * 64 + cell] = ((b.pc[p] & mine) >> sq) & 1 ? 1.0f : 0.0f;
            out[(6 + p) * 64 + cell] = ((b.pc[p] & theirs) >> sq) & 1 ? 1.0f : 0.0f;
        }
    }
    const int ck = me == WHITE ? 1 : 4, cq = me == WHITE ? 2 : 8, tk = me == WHITE ? 4 : 1, tq = me == WHITE ? 8 : 2;
    const float fills[7] = {(b.castle & ck) ? 1.0f : 0.0f, (b.castle & cq) ? 1.0f : 0.0f,
                            (b.castle & tk) ? 1.0f : 0.0f, (b.castle & tq) ? 1.0f : 0.0f,
                            (float)reps, (float)b.fifty / 100.0f, (float)(b.made / 2) / 50.0f};
    for (int k = 0; k < 7; ++k)
        for (int c = 0; c < 64; ++c) out[(12 + k) * 64 + c] = fills[k];
}

// Policy::get_action (chess.rs:395-493), knight-underpromotion bug kept (:442)
int get_action_host(int side, int index) {
    const int ch = index / 64;
    int row = (index % 64) / 8;
    const int col = index % 8;
    const int promo = ch < 3 ? ROOK : ch < 6 ? BISHOP : ch < 9 ? KNIGHT : 0;
    int rd, fd;
    static const int kr[8] = {2, 1, -2, -1, 2, 1, -2, -1}, kf[8] = {-1, -2, -1, -2, 1, 2, 1, 2};
    if (ch < 9) rd = 1;
    else if (ch < 23) rd = 0;
    else if (ch < 37) rd = ch - 23 < 7 ? -(ch - 22) : ch - 29;
    else if (ch < 65) {
        const int o = ch - 37;
        rd = o < 7 ? ch - 36 : o < 14 ? -(ch - 43) : o < 21 ? ch - 50 : -(ch - 57);
    } else rd = kr[ch - 65];
    if (ch < 9) fd = ch < 3 ? ch - 1 : ch - 4;   // channels 6..8 take the bishop formula (the reference bug)
    else if (ch < 23) fd = ch - 9 < 7 ? -(ch - 8) : ch - 15;
    else if (ch < 37) fd = 0;
    else if (ch < 65) {
        const int o = ch - 37;
        fd = o < 7 ? -(ch - 36) : o < 14 ? -(ch - 43) : o < 21 ? ch - 50 : ch - 57;
    } else fd = kf[ch - 65];
    if (side == BLACK) {
        rd = -rd;
        row = 7 - row;
    }
    const int src = row * 8 + col;
    const int dst = ((row + rd) & 7) * 8 + ((col + fd) & 7);   // Rank/File::from_index mask with 7
    return src | (dst << 6) | (promo << 12);
}

int slots_resize(spai_chess *e, uint32_t n, uint32_t max_hist) {
    Slots &S = e->slots;
    SPAI_TRY(S.board.alloc(n));
    SPAI_TRY(S.hist.alloc((size_t)n * max_hist));
    SPAI_TRY(S.n_hist.alloc(n));
    SPAI_TRY(S.moves.alloc((size_t)n * kMaxMoves));
    SPAI_TRY(S.u32.alloc(n));
    SPAI_TRY(S.i32.alloc(n));
    SPAI_TRY(S.f32.alloc((size_t)n * kPolicy));
    SPAI_TRY(S.f32b.alloc((size_t)n * kPolicy));
    S.n = n;
    S.max_hist = max_hist;
    std::vector<Board> h(n);
    for (auto &b : h) start_board(b);
    if (n) {
        SPAI_HIP(hipMemcpyAsync(S.board.p, h.data(), sizeof(Board) * n, hipMemcpyHostToDevice, e->stream));
        SPAI_HIP(hipMemsetAsync(S.n_hist.p, 0, sizeof(uint32_t) * n, e->stream));
        SPAI_HIP(hipStreamSynchronize(e->stream));
    }
    return SPAI_OK;
}

#define RANGE_CHECK(e, first, n) \
    SPAI_CHECK((uint64_t)(first) + (n) <= (e)->slots.n, SPAI_ERR_INVALID, "slots [%u, %u) out of range (%u)", first, \
               (first) + (n), (e)->slots.n)

int slots_write(spai_chess *e, uint32_t first, uint32_t n, const spai_chess_state *s) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    std::vector<Board> h(n);
    for (uint32_t i = 0; i < n; ++i) {
        h[i] = from_abi(s[i]);
        SPAI_CHECK(popc(h[i].pc[KING] & h[i].col[WHITE]) == 1 && popc(h[i].pc[KING] & h[i].col[BLACK]) == 1,
                   SPAI_ERR_INVALID, "slot %u: each side needs exactly one king", first + i);
    }
    SPAI_HIP(hipMemcpyAsync(e->slots.board.p + first, h.data(), sizeof(Board) * n, hipMemcpyHostToDevice, e->stream));
    SPAI_HIP(hipMemsetAsync(e->slots.n_hist.p + first, 0, sizeof(uint32_t) * n, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int slots_status(spai_chess *e, uint32_t first, uint32_t n, uint8_t *status, uint32_t *reps, float *value,
                 uint8_t *terminated) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    uint8_t *d_st = (uint8_t *)S.i32.p;
    k_slots_status<<<(n + kWavesPerBlock - 1) / kWavesPerBlock, 64 * kWavesPerBlock, 0, e->stream>>>(
        S.board.p, S.hist.p, S.n_hist.p, S.max_hist, first, n, nullptr, nullptr, d_st, S.u32.p);
    SPAI_HIP(hipGetLastError());
    std::vector<uint8_t> st(n);
    std::vector<uint32_t> rp(n);
    SPAI_HIP(hipMemcpyAsync(st.data(), d_st, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(rp.data(), S.u32.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < n; ++i) {
        if (status) status[i] = st[i];
        if (reps) reps[i] = rp[i];
        if (value) value[i] = st[i] == SPAI_WON ? 1.0f : 0.0f;   // chess.rs:168-174 (Won -> +1, quirk Q7)
        if (terminated) terminated[i] = st[i] != SPAI_ONGOING;
    }
    return SPAI_OK;
}

int slots_read(spai_chess *e, uint32_t first, uint32_t n, spai_chess_state *s) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    std::vector<Board> h(n);
    std::vector<uint8_t> st(n);
    std::vector<uint32_t> rp(n);
    SPAI_TRY(slots_status(e, first, n, st.data(), rp.data(), nullptr, nullptr));
    SPAI_HIP(hipMemcpy(h.data(), e->slots.board.p + first, sizeof(Board) * n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        h[i].status = st[i];
        s[i] = to_abi(h[i], rp[i]);
    }
    return SPAI_OK;
}

int slots_legal(spai_chess *e, uint32_t first, uint32_t n, uint16_t *moves, uint32_t *counts) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    k_slots_status<<<(n + kWavesPerBlock - 1) / kWavesPerBlock, 64 * kWavesPerBlock, 0, e->stream>>>(
        S.board.p, S.hist.p, S.n_hist.p, S.max_hist, first, n, S.moves.p, S.u32.p, nullptr, nullptr);
    SPAI_HIP(hipGetLastError());
    if (moves)
        SPAI_HIP(hipMemcpyAsync(moves, S.moves.p, sizeof(uint16_t) * kMaxMoves * n, hipMemcpyDeviceToHost,
                                e->stream));
    std::vector<uint32_t> c(n);
    SPAI_HIP(hipMemcpyAsync(c.data(), S.u32.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    if (counts) memcpy(counts, c.data(), 4 * n);
    if (moves)
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t j = c[i]; j < (uint32_t)kMaxMoves; ++j) moves[(size_t)i * kMaxMoves + j] = 0;
    return SPAI_OK;
}

int slots_apply(spai_chess *e, uint32_t first, uint32_t n, const uint16_t *moves, int32_t *rc) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    uint16_t *d_in = (uint16_t *)S.f32.p;
    SPAI_HIP(hipMemcpyAsync(d_in, moves, sizeof(uint16_t) * n, hipMemcpyHostToDevice, e->stream));
    k_slots_apply<<<(n + kWavesPerBlock - 1) / kWavesPerBlock, 64 * kWavesPerBlock, 0, e->stream>>>(
        S.board.p, S.hist.p, S.n_hist.p, S.max_hist, first, n, d_in, S.i32.p);
    SPAI_HIP(hipGetLastError());
    std::vector<int32_t> r(n);
    SPAI_HIP(hipMemcpyAsync(r.data(), S.i32.p, 4 * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    int first_err = SPAI_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (rc) rc[i] = r[i];
        if (r[i] != SPAI_OK && first_err == SPAI_OK) first_err = r[i];
    }
    if (first_err == SPAI_ERR_GAME_OVER) set_error("Game is already over");
    else if (first_err == SPAI_ERR_ILLEGAL_MOVE) set_error("Failed to make move");
    else if (first_err == SPAI_ERR_CAPACITY) set_error("transposition table full (cfg.max_moves)");
    return first_err;
}

int slots_encode(spai_chess *e, uint32_t first, uint32_t n, float *out) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    k_slots_encode<<<(n + kWavesPerBlock - 1) / kWavesPerBlock, 64 * kWavesPerBlock, 0, e->stream>>>(
        S.board.p, S.hist.p, S.n_hist.p, S.max_hist, first, n, S.f32.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(out, S.f32.p, sizeof(float) * kPlanes * 64 * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int slots_mask(spai_chess *e, uint32_t first, uint32_t n, const float *policy, uint32_t len, float *out) {
    SPAI_CHECK(len == (uint32_t)kPolicy, SPAI_ERR_INVALID, "Expected policy shape to be (73 * 8 * 8,), found (%u,)",
               len);
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    SPAI_HIP(hipMemcpyAsync(S.f32.p, policy, sizeof(float) * kPolicy * n, hipMemcpyHostToDevice, e->stream));
    k_slots_mask<<<n, 64, 0, e->stream>>>(S.board.p, first, n, S.f32.p, S.f32b.p);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(out, S.f32b.p, sizeof(float) * kPolicy * n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

// Device time of the batched rules kernels over the current slots [first, first+n):
// ms[0] legal move lists + counts + status (k_slots_status), ms[1] f32 encoding
// (k_slots_encode); mean of `iters` launches after one warm-up launch.
int slots_rules_bench(spai_chess *e, uint32_t first, uint32_t n, uint32_t iters, double *ms) {
    RANGE_CHECK(e, first, n);
    SPAI_CHECK(n > 0 && iters > 0, SPAI_ERR_INVALID, "rules_bench needs n, iters > 0");
    Slots &S = e->slots;
    hipEvent_t ev[2];
    SPAI_HIP(hipEventCreate(&ev[0]));
    SPAI_HIP(hipEventCreate(&ev[1]));
    const uint32_t grid = (n + kWavesPerBlock - 1) / kWavesPerBlock;
    int rc = SPAI_OK;
    for (int k = 0; k < 2 && rc == SPAI_OK; ++k) {
        double tot = 0;
        for (uint32_t it = 0; it <= iters; ++it) {
            if (hipEventRecord(ev[0], e->stream) != hipSuccess) rc = SPAI_ERR_DEVICE;
            if (k == 0)
                k_slots_status<<<grid, 64 * kWavesPerBlock, 0, e->stream>>>(S.board.p, S.hist.p, S.n_hist.p,
                                                                            S.max_hist, first, n, S.moves.p,
                                                                            S.u32.p, (uint8_t *)S.i32.p, nullptr);
            else
                k_slots_encode<<<grid, 64 * kWavesPerBlock, 0, e->stream>>>(S.board.p, S.hist.p, S.n_hist.p,
                                                                            S.max_hist, first, n, S.f32.p);
            float t = 0;
            if (hipGetLastError() != hipSuccess || hipEventRecord(ev[1], e->stream) != hipSuccess ||
                hipEventSynchronize(ev[1]) != hipSuccess || hipEventElapsedTime(&t, ev[0], ev[1]) != hipSuccess) {
                set_error("chess rules bench launch failed");
                rc = SPAI_ERR_DEVICE;
                break;
            }
            if (it) tot += t;
        }
        ms[k] = tot / iters;
    }
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
    return rc;
}

// ---------------------------------------------------------------- perft
// Breadth-first perft on the device: the positions of one ply live in a flat
// Board array; each wave generates one position's legal moves (wave_movegen,
// the same routine as search and self-play) and either counts them or writes
// the children (apply_move) at slots taken by one atomic per wave.  Pins the
// device move generator to the public perft counts (the crate's MoveGen::new_legal
// + Board::make_move, game/chess.rs:54,117-118).
__global__ void k_perft_count(const Board *__restrict__ level, uint64_t n, unsigned long long *__restrict__ total) {
    const int lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const Board b = level[i];
    const GenOut g = wave_movegen(b, lane, [](int, int) {});
    if (lane == 0 && g.n) atomicAdd(total, (unsigned long long)g.n);
}

__global__ void k_perft_expand(const Board *__restrict__ level, uint64_t n, Board *__restrict__ next, uint64_t cap,
                               unsigned long long *__restrict__ fill) {
    const int lane = threadIdx.x & 63;
    const uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (i >= n) return;
    const Board b = level[i];
    const GenOut g = wave_movegen(b, lane, [](int, int) {});
    unsigned long long base = 0;
    if (lane == 0 && g.n) base = atomicAdd(fill, (unsigned long long)g.n);
    base = __shfl(base, 0, 64);
    wave_movegen(b, lane, [&](int off, int mv) {
        if (base + off < cap) {
            Board c = b;
            apply_move(c, mv);
            next[base + off] = c;
        }
    });
}

struct PerftBufs {   // DevBuf has no destructor: free the ply buffers on every exit
    DevBuf<Board> cur, nxt;
    DevBuf<unsigned long long> ctr;
    ~PerftBufs() {
        cur.release();
        nxt.release();
        ctr.release();
    }
};

// counts[d - 1] = perft(d) of slot `slot`'s position for d = 1..depth
int perft(spai_chess *e, uint32_t slot, int depth, uint64_t *counts) {
    SPAI_CHECK(slot < e->slots.n, SPAI_ERR_INVALID, "slot %u out of range (%u)", slot, e->slots.n);
    SPAI_CHECK(depth >= 1 && depth <= 8, SPAI_ERR_INVALID, "perft depth %d not in 1..8", depth);
    constexpr uint64_t kMaxLevel = 1ull << 26;   // 4.8 GB of boards per ply
    PerftBufs B;
    DevBuf<Board> &cur = B.cur, &nxt = B.nxt;
    DevBuf<unsigned long long> &ctr = B.ctr;
    SPAI_TRY(cur.alloc(1));
    SPAI_TRY(ctr.alloc(2));
    hipStream_t st = e->stream;
    SPAI_HIP(hipMemcpyAsync(cur.p, e->slots.board.p + slot, sizeof(Board), hipMemcpyDeviceToDevice, st));
    uint64_t n = 1;
    for (int d = 1; d <= depth; ++d) {
        unsigned long long h[2] = {0, 0};
        SPAI_HIP(hipMemsetAsync(ctr.p, 0, sizeof(h), st));
        const unsigned grid = (unsigned)((n + kWavesPerBlock - 1) / kWavesPerBlock);
        k_perft_count<<<grid, 64 * kWavesPerBlock, 0, st>>>(cur.p, n, ctr.p);
        SPAI_HIP(hipGetLastError());
        SPAI_HIP(hipMemcpyAsync(h, ctr.p, sizeof(h), hipMemcpyDeviceToHost, st));
        SPAI_HIP(hipStreamSynchronize(st));
        counts[d - 1] = h[0];
        if (d == depth || h[0] == 0) {
            for (int k = d; k < depth; ++k) counts[k] = 0;
            break;
        }
        SPAI_CHECK(h[0] <= kMaxLevel, SPAI_ERR_CAPACITY, "perft: ply %d holds %llu positions (limit %llu)", d,
                   (unsigned long long)h[0], (unsigned long long)kMaxLevel);
        SPAI_TRY(nxt.alloc(h[0]));
        k_perft_expand<<<grid, 64 * kWavesPerBlock, 0, st>>>(cur.p, n, nxt.p, h[0], ctr.p + 1);
        SPAI_HIP(hipGetLastError());
        SPAI_HIP(hipMemcpyAsync(&h[1], ctr.p + 1, sizeof(h[1]), hipMemcpyDeviceToHost, st));
        SPAI_HIP(hipStreamSynchronize(st));
        SPAI_CHECK(h[1] == h[0], SPAI_ERR_DEVICE, "perft: ply %d expanded %llu of %llu children", d,
                   (unsigned long long)h[1], (unsigned long long)h[0]);
        std::swap(cur, nxt);
        nxt.release();
        n = h[0];
    }
    return SPAI_OK;
}

int slots_encode_device(spai_chess *e, uint32_t first, uint32_t n, float *d_out) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    Slots &S = e->slots;
    k_slots_encode<<<(n + kWavesPerBlock - 1) / kWavesPerBlock, 64 * kWavesPerBlock, 0, e->stream>>>(
        S.board.p, S.hist.p, S.n_hist.p, S.max_hist, first, n, d_out);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

int slots_softmax_mask_device(spai_chess *e, uint32_t first, uint32_t n, const float *d_logits, float *d_out) {
    RANGE_CHECK(e, first, n);
    if (!n) return SPAI_OK;
    k_slots_softmax_mask<<<n, 64, 0, e->stream>>>(e->slots.board.p, first, n, d_logits, d_out);
    SPAI_HIP(hipGetLastError());
    return SPAI_OK;
}

}  // namespace chess
}  // namespace spai

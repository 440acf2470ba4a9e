// rules.hip — batched Connect4 rules kernels over struct-of-arrays bitboards.
//
// One lane per game slot for the per-game ops (8-byte coalesced x/o loads,
// 1-byte status/count/result streams); the encoder writes its output with one
// lane per 4-byte output word so every wave stores a contiguous 256 B run.
// These are HBM-bound byte kernels: algorithmic bytes per game
//   legal   16 (x,o) + 1 (status) in, 1 out                      = 18 B
//   apply   16 + 1 + 1 (n, status) + 4 (action) in, 8 + 1 + 1 + 1 out = 33 B
//   encode  16 + 1 in, 252 (bf16 [3][6][7]) out                  = 269 B
#include <cstring>

#include "spai_internal.h"

namespace spai {
namespace {

constexpr int kBlock = 256;

__global__ void k_reset(uint64_t *x, uint64_t *o, uint8_t *n, uint8_t *st, uint32_t first, uint32_t cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    i += first;
    x[i] = 0;
    o[i] = 0;
    n[i] = 0;
    st[i] = c4::kOngoing;
}

__global__ void k_legal(const uint64_t *__restrict__ x, const uint64_t *__restrict__ o,
                        const uint8_t *__restrict__ st, uint8_t *__restrict__ mask, uint32_t first, uint32_t cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    uint32_t g = first + i;
    mask[i] = (uint8_t)c4::legal_mask(x[g], o[g], st[g]);
}

__global__ void k_apply(uint64_t *__restrict__ x, uint64_t *__restrict__ o, uint8_t *__restrict__ n,
                        uint8_t *__restrict__ st, const int32_t *__restrict__ act, int8_t *__restrict__ rc,
                        uint32_t first, uint32_t cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    uint32_t g = first + i;
    c4::State s{x[g], o[g], n[g], st[g]}, r;
    int e = c4::next_state(s, act[i], r);
    if (e == 0) {
        if (c4::x_to_move(s.n)) x[g] = r.x;
        else o[g] = r.o;
        n[g] = r.n;
        st[g] = r.status;
    }
    rc[i] = (int8_t)(e == 0 ? SPAI_OK : e == -2 ? SPAI_ERR_ILLEGAL_MOVE : e == -3 ? SPAI_ERR_GAME_OVER : SPAI_ERR_INVALID);
}

// Four games per lane (slot range starting at a multiple of 4): 32-B x/o loads,
// 4-B status/count/result words, so each lane keeps 4x the bytes in flight of the
// one-game kernels above (which handle unaligned ranges).
__global__ void k_legal4(const uint64_t *__restrict__ x, const uint64_t *__restrict__ o,
                         const uint8_t *__restrict__ st, uint8_t *__restrict__ mask, uint32_t first, uint32_t cnt) {
    const uint32_t i = 4u * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= cnt) return;
    const uint32_t g = first + i;
    if (i + 4 <= cnt) {
        const ulonglong2 xa = *(const ulonglong2 *)(x + g), xb = *(const ulonglong2 *)(x + g + 2);
        const ulonglong2 oa = *(const ulonglong2 *)(o + g), ob = *(const ulonglong2 *)(o + g + 2);
        const uint32_t s4 = *(const uint32_t *)(st + g);
        *(uint32_t *)(mask + i) = c4::legal_mask(xa.x, oa.x, (uint8_t)s4) |
                                  c4::legal_mask(xa.y, oa.y, (uint8_t)(s4 >> 8)) << 8 |
                                  c4::legal_mask(xb.x, ob.x, (uint8_t)(s4 >> 16)) << 16 |
                                  c4::legal_mask(xb.y, ob.y, (uint8_t)(s4 >> 24)) << 24;
    } else {
        for (uint32_t k = i; k < cnt; ++k) mask[k] = (uint8_t)c4::legal_mask(x[first + k], o[first + k], st[first + k]);
    }
}

__device__ __forceinline__ int8_t apply_rc(int e) {
    return (int8_t)(e == 0 ? SPAI_OK : e == -2 ? SPAI_ERR_ILLEGAL_MOVE : e == -3 ? SPAI_ERR_GAME_OVER : SPAI_ERR_INVALID);
}

__global__ void k_apply4(uint64_t *__restrict__ x, uint64_t *__restrict__ o, uint8_t *__restrict__ n,
                         uint8_t *__restrict__ st, const int32_t *__restrict__ act, int8_t *__restrict__ rc,
                         uint32_t first, uint32_t cnt) {
    const uint32_t i = 4u * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= cnt) return;
    const uint32_t g = first + i;
    if (i + 4 <= cnt) {
        uint64_t xs[4], os[4];
        *(ulonglong2 *)xs = *(const ulonglong2 *)(x + g);
        *(ulonglong2 *)(xs + 2) = *(const ulonglong2 *)(x + g + 2);
        *(ulonglong2 *)os = *(const ulonglong2 *)(o + g);
        *(ulonglong2 *)(os + 2) = *(const ulonglong2 *)(o + g + 2);
        uint32_t n4 = *(const uint32_t *)(n + g), s4 = *(const uint32_t *)(st + g);
        const int4 a4 = *(const int4 *)(act + i);
        const int a[4] = {a4.x, a4.y, a4.z, a4.w};
        uint32_t r4 = 0, nn = 0, ss = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            c4::State s{xs[k], os[k], (uint8_t)(n4 >> (8 * k)), (uint8_t)(s4 >> (8 * k))}, r;
            const int e = c4::next_state(s, a[k], r);
            if (e == 0) {
                xs[k] = r.x;
                os[k] = r.o;
                s = r;
            }
            nn |= (uint32_t)s.n << (8 * k);
            ss |= (uint32_t)s.status << (8 * k);
            r4 |= (uint32_t)(uint8_t)apply_rc(e) << (8 * k);
        }
        *(ulonglong2 *)(x + g) = *(const ulonglong2 *)xs;
        *(ulonglong2 *)(x + g + 2) = *(const ulonglong2 *)(xs + 2);
        *(ulonglong2 *)(o + g) = *(const ulonglong2 *)os;
        *(ulonglong2 *)(o + g + 2) = *(const ulonglong2 *)(os + 2);
        *(uint32_t *)(n + g) = nn;
        *(uint32_t *)(st + g) = ss;
        *(uint32_t *)(rc + i) = r4;
    } else {
        for (uint32_t k = i; k < cnt; ++k) {
            const uint32_t gk = first + k;
            c4::State s{x[gk], o[gk], n[gk], st[gk]}, r;
            const int e = c4::next_state(s, act[k], r);
            if (e == 0) {
                x[gk] = r.x;
                o[gk] = r.o;
                n[gk] = r.n;
                st[gk] = r.status;
            }
            rc[k] = apply_rc(e);
        }
    }
}

__global__ void k_value_term(const uint8_t *__restrict__ st, float *__restrict__ v, uint8_t *__restrict__ t,
                             uint32_t first, uint32_t cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    uint8_t s = st[first + i];
    v[i] = s == c4::kOngoing ? 0.0f : c4::terminal_value(s);
    t[i] = s != c4::kOngoing;
}

// get_encoding (connect_four.rs:242-259): [3][6][7] planes (mine, theirs,
// empty) of the player to move; element e = plane*42 + row*7 + col reads bit
// col*7 + row.  One wave per 64 games: each lane builds its game's output words
// in LDS (stride D words, odd, so the writes are conflict-free), then the wave
// stores the 64 games' contiguous D*256-byte run with 16-B coalesced stores.
// BF16: D = 63 words of 2 bf16 (the layout the net stem would read); else D = 126 f32.
template <bool BF16>
__global__ __launch_bounds__(64) void k_encode(const uint64_t *__restrict__ x, const uint64_t *__restrict__ o,
                                               const uint8_t *__restrict__ n, uint32_t *__restrict__ out,
                                               uint32_t first, uint32_t cnt) {
    constexpr int D = BF16 ? 63 : 126;
    __shared__ uint32_t buf[64 * D];
    const int lane = threadIdx.x;
    const uint32_t g0 = blockIdx.x * 64u;
    const uint32_t ng = min(64u, cnt - g0);
    if ((uint32_t)lane < ng) {
        const uint32_t g = first + g0 + lane;
        const bool xm = c4::x_to_move(n[g]);
        const uint64_t xv = x[g], ov = o[g];
        const uint64_t mine = xm ? xv : ov, theirs = xm ? ov : xv;
        const uint64_t pl[3] = {mine, theirs, ~(mine | theirs)};
        uint32_t *dst = buf + lane * D;
#pragma unroll
        for (int w = 0; w < D; ++w) {
            if (BF16) {
                const int e0 = 2 * w, e1 = 2 * w + 1;
                const int c0 = e0 % 42, c1 = e1 % 42;
                const uint32_t b0 = (uint32_t)(pl[e0 / 42] >> ((c0 % 7) * 7 + c0 / 7)) & 1u;
                const uint32_t b1 = (uint32_t)(pl[e1 / 42] >> ((c1 % 7) * 7 + c1 / 7)) & 1u;
                dst[w] = (b0 ? 0x3F80u : 0u) | (b1 ? 0x3F800000u : 0u);
            } else {
                const int c = w % 42;
                dst[w] = ((pl[w / 42] >> ((c % 7) * 7 + c / 7)) & 1u) ? 0x3F800000u : 0u;
            }
        }
    }
    __syncthreads();
    const uint32_t words = ng * D;
    uint32_t *base = out + (size_t)g0 * D;
    const uint32_t v4 = words / 4;   // g0 * D * 4 B is a multiple of 16 B (64 | g0)
    for (uint32_t j = lane; j < v4; j += 64) *(uint4 *)(base + 4 * j) = *(const uint4 *)(buf + 4 * j);
    for (uint32_t j = 4 * v4 + lane; j < words; j += 64) base[j] = buf[j];
}

__global__ void k_mask(const uint64_t *__restrict__ x, const uint64_t *__restrict__ o,
                       const uint8_t *__restrict__ st, const float *__restrict__ p, float *__restrict__ out,
                       uint32_t first, uint32_t cnt) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    uint32_t g = first + i;
    float pi[c4::kActions], r[c4::kActions];
    for (int a = 0; a < c4::kActions; ++a) pi[a] = p[(size_t)i * c4::kActions + a];
    c4::mask_renorm(pi, c4::legal_mask(x[g], o[g], st[g]), r);
    for (int a = 0; a < c4::kActions; ++a) out[(size_t)i * c4::kActions + a] = r[a];
}

// random reachable positions for the bench: k random legal moves per slot
__global__ void k_random_positions(uint64_t *x, uint64_t *o, uint8_t *n, uint8_t *st, uint32_t cnt, uint64_t seed) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    uint64_t h = c4::splitmix64(seed ^ ((uint64_t)i << 20));
    c4::State s{0, 0, 0, c4::kOngoing};
    int plies = (int)(h % 30);
    for (int k = 0; k < plies; ++k) {
        uint32_t lm = c4::legal_mask(s.x, s.o, s.status);
        if (!lm) break;
        h = c4::splitmix64(h);
        int pick = (int)(h % c4::popc32(lm));
        c4::State r;
        c4::next_state(s, c4::kth_bit(lm, pick), r);
        if (r.status != c4::kOngoing) break;
        s = r;
    }
    x[i] = s.x;
    o[i] = s.o;
    n[i] = s.n;
    st[i] = s.status;
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kBlock - 1) / kBlock); }

int check_range(spai_engine *e, uint32_t first, uint32_t n) {
    SPAI_CHECK((uint64_t)first + n <= e->games.count, SPAI_ERR_INVALID,
               "game slots [%u, %u) out of range (%u allocated)", first, first + n, e->games.count);
    return SPAI_OK;
}

}  // namespace

int rules_resize(spai_engine *e, uint32_t n) {
    GameSlots &g = e->games;
    SPAI_TRY(g.x.alloc(n));
    SPAI_TRY(g.o.alloc(n));
    SPAI_TRY(g.n.alloc(n));
    SPAI_TRY(g.status.alloc(n));
    g.count = n;
    return n ? rules_reset(e, 0, n) : SPAI_OK;
}

int rules_reset(spai_engine *e, uint32_t first, uint32_t n) {
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    GameSlots &g = e->games;
    k_reset<<<blocks_for(n), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.n.p, g.status.p, first, n);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int rules_write(spai_engine *e, uint32_t first, uint32_t n, const spai_c4_state *s) {
    SPAI_TRY(check_range(e, first, n));
    std::vector<uint64_t> x(n), o(n);
    std::vector<uint8_t> nn(n), st(n);
    for (uint32_t i = 0; i < n; ++i) {
        SPAI_CHECK(!(s[i].x & s[i].o) && !((s[i].x | s[i].o) & ~c4::kBoard) && s[i].status <= c4::kWon,
                   SPAI_ERR_INVALID, "state %u is not a Connect4 bitboard", i);
        x[i] = s[i].x;
        o[i] = s[i].o;
        nn[i] = s[i].num_actions_played;
        st[i] = s[i].status;
    }
    GameSlots &g = e->games;
    SPAI_HIP(hipMemcpyAsync(g.x.p + first, x.data(), n * 8, hipMemcpyHostToDevice, e->stream));
    SPAI_HIP(hipMemcpyAsync(g.o.p + first, o.data(), n * 8, hipMemcpyHostToDevice, e->stream));
    SPAI_HIP(hipMemcpyAsync(g.n.p + first, nn.data(), n, hipMemcpyHostToDevice, e->stream));
    SPAI_HIP(hipMemcpyAsync(g.status.p + first, st.data(), n, hipMemcpyHostToDevice, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int rules_read(spai_engine *e, uint32_t first, uint32_t n, spai_c4_state *s) {
    SPAI_TRY(check_range(e, first, n));
    std::vector<uint64_t> x(n), o(n);
    std::vector<uint8_t> nn(n), st(n);
    GameSlots &g = e->games;
    SPAI_HIP(hipMemcpyAsync(x.data(), g.x.p + first, n * 8, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(o.data(), g.o.p + first, n * 8, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(nn.data(), g.n.p + first, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(st.data(), g.status.p + first, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < n; ++i) {
        s[i] = spai_c4_state{};
        s[i].x = x[i];
        s[i].o = o[i];
        s[i].num_actions_played = nn[i];
        s[i].status = st[i];
    }
    return SPAI_OK;
}

int rules_legal(spai_engine *e, uint32_t first, uint32_t n, uint32_t *mask) {
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    DevBuf<uint8_t> d;
    SPAI_TRY(d.alloc(n));
    GameSlots &g = e->games;
    if (first % 4 == 0)
        k_legal4<<<blocks_for((n + 3) / 4), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.status.p, d.p, first, n);
    else
        k_legal<<<blocks_for(n), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.status.p, d.p, first, n);
    SPAI_HIP(hipGetLastError());
    std::vector<uint8_t> h(n);
    SPAI_HIP(hipMemcpyAsync(h.data(), d.p, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    d.release();
    for (uint32_t i = 0; i < n; ++i) mask[i] = h[i];
    return SPAI_OK;
}

int rules_apply(spai_engine *e, uint32_t first, uint32_t n, const int32_t *actions, int32_t *rc) {
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    DevBuf<int32_t> da;
    DevBuf<int8_t> dr;
    SPAI_TRY(da.alloc(n));
    SPAI_TRY(dr.alloc(n));
    SPAI_HIP(hipMemcpyAsync(da.p, actions, n * 4, hipMemcpyHostToDevice, e->stream));
    GameSlots &g = e->games;
    if (first % 4 == 0)
        k_apply4<<<blocks_for((n + 3) / 4), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.n.p, g.status.p, da.p, dr.p,
                                                                    first, n);
    else
        k_apply<<<blocks_for(n), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.n.p, g.status.p, da.p, dr.p, first, n);
    SPAI_HIP(hipGetLastError());
    std::vector<int8_t> h(n);
    SPAI_HIP(hipMemcpyAsync(h.data(), dr.p, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    int first_err = SPAI_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (rc) rc[i] = h[i];
        if (h[i] != SPAI_OK && first_err == SPAI_OK) first_err = h[i];
    }
    if (first_err != SPAI_OK)
        set_error("get_next_state failed for at least one slot: %s",
                  first_err == SPAI_ERR_ILLEGAL_MOVE ? "Illegal move: column already filled"
                  : first_err == SPAI_ERR_GAME_OVER ? "Game has already ended" : "action out of range");
    return first_err;
}

int rules_value_term(spai_engine *e, uint32_t first, uint32_t n, float *v, uint8_t *t) {
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    DevBuf<float> dv;
    DevBuf<uint8_t> dt;
    SPAI_TRY(dv.alloc(n));
    SPAI_TRY(dt.alloc(n));
    k_value_term<<<blocks_for(n), kBlock, 0, e->stream>>>(e->games.status.p, dv.p, dt.p, first, n);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(v, dv.p, n * 4, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipMemcpyAsync(t, dt.p, n, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int rules_encode(spai_engine *e, uint32_t first, uint32_t n, float *out) {
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    DevBuf<float> d;
    SPAI_TRY(d.alloc((size_t)n * 126));
    GameSlots &g = e->games;
    k_encode<false><<<(n + 63) / 64, 64, 0, e->stream>>>(g.x.p, g.o.p, g.n.p, (uint32_t *)d.p, first, n);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(out, d.p, (size_t)n * 126 * 4, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int rules_mask(spai_engine *e, uint32_t first, uint32_t n, const float *p, uint32_t len, float *out) {
    SPAI_CHECK(len == c4::kActions, SPAI_ERR_INVALID, "Expected policy shape to be (7,), found (%u,)", len);
    SPAI_TRY(check_range(e, first, n));
    if (!n) return SPAI_OK;
    DevBuf<float> dp, dq;
    SPAI_TRY(dp.alloc((size_t)n * 7));
    SPAI_TRY(dq.alloc((size_t)n * 7));
    SPAI_HIP(hipMemcpyAsync(dp.p, p, (size_t)n * 28, hipMemcpyHostToDevice, e->stream));
    GameSlots &g = e->games;
    k_mask<<<blocks_for(n), kBlock, 0, e->stream>>>(g.x.p, g.o.p, g.status.p, dp.p, dq.p, first, n);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(out, dq.p, (size_t)n * 28, hipMemcpyDeviceToHost, e->stream));
    SPAI_HIP(hipStreamSynchronize(e->stream));
    return SPAI_OK;
}

int rules_bench(spai_engine *e, uint32_t n, uint32_t iters, double *ms) {
    SPAI_CHECK(n > 0 && iters > 0, SPAI_ERR_INVALID, "rules_bench needs n, iters > 0");
    DevBuf<uint64_t> x, o;
    DevBuf<uint8_t> nn, st, mask;
    DevBuf<int32_t> act;
    DevBuf<int8_t> rc;
    DevBuf<uint32_t> enc;
    SPAI_TRY(x.alloc(n));
    SPAI_TRY(o.alloc(n));
    SPAI_TRY(nn.alloc(n));
    SPAI_TRY(st.alloc(n));
    SPAI_TRY(mask.alloc(n));
    SPAI_TRY(act.alloc(n));
    SPAI_TRY(rc.alloc(n));
    SPAI_TRY(enc.alloc((size_t)n * 63));
    DevBuf<uint64_t> x0, o0;   // pristine positions: every timed apply starts from them
    DevBuf<uint8_t> nn0, st0;
    SPAI_TRY(x0.alloc(n));
    SPAI_TRY(o0.alloc(n));
    SPAI_TRY(nn0.alloc(n));
    SPAI_TRY(st0.alloc(n));
    hipStream_t s = e->stream;
    k_random_positions<<<blocks_for(n), kBlock, 0, s>>>(x.p, o.p, nn.p, st.p, n, 12345);
    SPAI_HIP(hipGetLastError());
    SPAI_HIP(hipMemcpyAsync(x0.p, x.p, 8ull * n, hipMemcpyDeviceToDevice, s));
    SPAI_HIP(hipMemcpyAsync(o0.p, o.p, 8ull * n, hipMemcpyDeviceToDevice, s));
    SPAI_HIP(hipMemcpyAsync(nn0.p, nn.p, n, hipMemcpyDeviceToDevice, s));
    SPAI_HIP(hipMemcpyAsync(st0.p, st.p, n, hipMemcpyDeviceToDevice, s));
    {
        std::vector<int32_t> a(n);
        for (uint32_t i = 0; i < n; ++i) a[i] = (int32_t)((i * 2654435761u) % 7);
        SPAI_HIP(hipMemcpyAsync(act.p, a.data(), (size_t)n * 4, hipMemcpyHostToDevice, s));
    }
    hipEvent_t ev[2];
    SPAI_HIP(hipEventCreate(&ev[0]));
    SPAI_HIP(hipEventCreate(&ev[1]));
    for (int k = 0; k < 3; ++k) {
        float best = 0;
        for (uint32_t it = 0; it < iters + 1; ++it) {   // first launch is warmup
            if (k == 1) {   // restore the positions (outside the timed region) so every apply does its writes
                SPAI_HIP(hipMemcpyAsync(x.p, x0.p, 8ull * n, hipMemcpyDeviceToDevice, s));
                SPAI_HIP(hipMemcpyAsync(o.p, o0.p, 8ull * n, hipMemcpyDeviceToDevice, s));
                SPAI_HIP(hipMemcpyAsync(nn.p, nn0.p, n, hipMemcpyDeviceToDevice, s));
                SPAI_HIP(hipMemcpyAsync(st.p, st0.p, n, hipMemcpyDeviceToDevice, s));
            }
            SPAI_HIP(hipEventRecord(ev[0], s));
            if (k == 0) {
                k_legal4<<<blocks_for((n + 3) / 4), kBlock, 0, s>>>(x.p, o.p, st.p, mask.p, 0, n);
            } else if (k == 1) {
                k_apply4<<<blocks_for((n + 3) / 4), kBlock, 0, s>>>(x.p, o.p, nn.p, st.p, act.p, rc.p, 0, n);
            } else {
                k_encode<true><<<(n + 63) / 64, 64, 0, s>>>(x.p, o.p, nn.p, enc.p, 0, n);
            }
            SPAI_HIP(hipGetLastError());
            SPAI_HIP(hipEventRecord(ev[1], s));
            SPAI_HIP(hipEventSynchronize(ev[1]));
            float t;
            SPAI_HIP(hipEventElapsedTime(&t, ev[0], ev[1]));
            if (it > 0) best += t;
        }
        ms[k] = best / iters;
    }
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
    return SPAI_OK;
}

}  // namespace spai

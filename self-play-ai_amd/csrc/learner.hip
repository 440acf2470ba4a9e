// learner.hip — the training step of the C4 policy/value ResNet on the device
// (SURVEY.md §8f.1): ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85)
// = Net::forward(x, train=true) (model/mod.rs:152-184, model/connect_four.rs:50-81),
// loss -(log_softmax(p)·π).sum()/B + MSE(v, z) (model/mod.rs:128-135), and
// tch's Adam::default() step (β1 0.9, β2 0.999, eps 1e-8, no weight decay,
// lr 1e-3; model/mod.rs:107).  BatchNorm runs in train mode: batch statistics
// over (B, 6, 7), running statistics updated with momentum 0.1 and the
// unbiased batch variance (tch/libtorch batch_norm semantics).
//
// Data-parallel learner: with a communicator set, the flat gradient is summed
// over ranks with RCCL (ncclAllReduce over xGMI) and scaled by 1/world before
// Adam, and the BN running statistics are averaged, so every rank holds the
// same parameters after every step.
//
// Layout: fp32 NCHW activations [B][C][42] (the training batch is small —
// 128 in the reference — and the step is ~15 GFLOP, far from any roofline
// that matters next to self-play; kernels are LDS-tiled fp32 and
// deterministic: every reduction has a fixed order, no float atomics).
// Parameters, gradients and Adam moments share the flat construction-order
// layout of spai_net_create (conv w, b, BN γ, β, μ, σ²; linears w, b).
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "spai_internal.h"

namespace spai {
namespace {

constexpr int kCells = 42, kRows = 6, kCols = 7;
constexpr int kPad = 72;          // (6+2) x (7+2) zero-padded plane
constexpr int kThreads = 256;
constexpr int kWgradSplit = 8;    // batch chunks of the weight-gradient reduction

// ------------------------------------------------------------------ conv 3x3
// out[b][co][p] (+)= bias[co] + sum_ci sum_tap w[co][ci][tap] * in[b][ci][p + off(tap)]
// One workgroup per (sample, block of up to 16 output channels): the sample's
// zero-padded input planes and the block's weights are staged in LDS.
// Also the data gradient: dx = conv(dz, w') with w'[ci][co][8 - tap].
__global__ __launch_bounds__(kThreads) void k_conv3x3(const float *__restrict__ in, int ci_n,
                                                      const float *__restrict__ w, const float *__restrict__ bias,
                                                      int co_n, int cob, float *__restrict__ out, int accumulate) {
    extern __shared__ float sm[];
    float *xs = sm;                      // [ci_n][kPad]
    float *ws = sm + ci_n * kPad;        // [cob][ci_n][9]
    const int b = blockIdx.y, co0 = blockIdx.x * cob;
    const int ncob = min(cob, co_n - co0);
    const float *xb = in + (size_t)b * ci_n * kCells;
    for (int i = threadIdx.x; i < ci_n * kPad; i += kThreads) {
        const int c = i / kPad, r = i - c * kPad, h = r / 9 - 1, x = r % 9 - 1;
        xs[i] = (h >= 0 && h < kRows && x >= 0 && x < kCols) ? xb[c * kCells + h * kCols + x] : 0.f;
    }
    for (int i = threadIdx.x; i < ncob * ci_n * 9; i += kThreads) ws[i] = w[(size_t)co0 * ci_n * 9 + i];
    __syncthreads();
    for (int o = threadIdx.x; o < ncob * kCells; o += kThreads) {
        const int co = o / kCells, p = o - co * kCells, h = p / kCols, x = p - h * kCols;
        const float *wr = ws + co * ci_n * 9;
        float acc = 0.f;
        for (int c = 0; c < ci_n; ++c) {
            const float *xp = xs + c * kPad + h * 9 + x;   // top-left of the 3x3 window
            const float *wc = wr + c * 9;
#pragma unroll
            for (int t = 0; t < 9; ++t) acc += wc[t] * xp[(t / 3) * 9 + t % 3];
        }
        if (bias) acc += bias[co0 + co];
        float *dst = out + ((size_t)b * co_n + co0 + co) * kCells + p;
        *dst = accumulate ? *dst + acc : acc;
    }
}

// w'[ci][co][8 - tap] = w[co][ci][tap] (data-gradient weights)
__global__ void k_flip_transpose(const float *__restrict__ w, int co_n, int ci_n, float *__restrict__ wt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= co_n * ci_n * 9) return;
    const int co = i / (ci_n * 9), r = i - co * ci_n * 9, c = r / 9, t = r % 9;
    wt[((size_t)c * co_n + co) * 9 + (8 - t)] = w[i];
}

// partial weight/bias gradients over batch chunk blockIdx.y:
// part[y][co][ci*9+tap] = sum_{b in chunk} sum_p dz[b][co][p] * x[b][ci][p + off(tap)]
// partb[y][co] = sum_{b in chunk} sum_p dz[b][co][p]
__global__ __launch_bounds__(kThreads) void k_conv_wgrad_part(const float *__restrict__ x, int ci_n,
                                                              const float *__restrict__ dz, int co_n, int B,
                                                              float *__restrict__ part, float *__restrict__ partb) {
    extern __shared__ float sm[];
    float *xs = sm;                 // [ci_n][kPad]
    float *ds = sm + ci_n * kPad;   // [kCells]
    const int co = blockIdx.x, y = blockIdx.y;
    const int b0 = (int)((int64_t)B * y / gridDim.y), b1 = (int)((int64_t)B * (y + 1) / gridDim.y);
    const int nout = ci_n * 9;
    float acc[3] = {0.f, 0.f, 0.f};   // outputs tid, tid+256, tid+512 (nout <= 576)
    float accb = 0.f;
    for (int b = b0; b < b1; ++b) {
        const float *xb = x + (size_t)b * ci_n * kCells;
        for (int i = threadIdx.x; i < ci_n * kPad; i += kThreads) {
            const int c = i / kPad, r = i - c * kPad, h = r / 9 - 1, xx = r % 9 - 1;
            xs[i] = (h >= 0 && h < kRows && xx >= 0 && xx < kCols) ? xb[c * kCells + h * kCols + xx] : 0.f;
        }
        if (threadIdx.x < kCells) ds[threadIdx.x] = dz[((size_t)b * co_n + co) * kCells + threadIdx.x];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int o = threadIdx.x + k * kThreads;
            if (o < nout) {
                const int c = o / 9, t = o - c * 9;
                const float *xp = xs + c * kPad + (t / 3) * 9 + t % 3;
                float s = 0.f;
                for (int p = 0; p < kCells; ++p) s += ds[p] * xp[(p / kCols) * 9 + p % kCols];
                acc[k] += s;
            }
        }
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int p = 0; p < kCells; ++p) s += ds[p];
            accb += s;
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int o = threadIdx.x + k * kThreads;
        if (o < nout) part[((size_t)y * co_n + co) * nout + o] = acc[k];
    }
    if (threadIdx.x == 0) partb[(size_t)y * co_n + co] = accb;
}

// g[i] = sum_y part[y][i] in fixed order (deterministic)
__global__ void k_sum_parts(const float *__restrict__ part, int n, int ny, float *__restrict__ g) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
    for (int y = 0; y < ny; ++y) s += part[(size_t)y * n + i];
    g[i] = s;
}

// ------------------------------------------------------------------ batch norm
__device__ __forceinline__ float block_sum(float v, float *red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}

// per channel: batch mean and biased variance over (B, 42) (two passes),
// invstd = 1/sqrt(var + eps); running stats: r = (1 - m) r + m * stat (unbiased var)
__global__ __launch_bounds__(kThreads) void k_bn_stats(const float *__restrict__ z, int c_n, int B, float eps,
                                                       float momentum, float *__restrict__ mean,
                                                       float *__restrict__ invstd, float *__restrict__ run_mean,
                                                       float *__restrict__ run_var) {
    __shared__ float red[kThreads];
    const int c = blockIdx.x, n = B * kCells;
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += kThreads) s += z[((size_t)(i / kCells) * c_n + c) * kCells + i % kCells];
    const float mu = block_sum(s, red) / (float)n;
    float q = 0.f;
    for (int i = threadIdx.x; i < n; i += kThreads) {
        const float d = z[((size_t)(i / kCells) * c_n + c) * kCells + i % kCells] - mu;
        q += d * d;
    }
    const float var = block_sum(q, red) / (float)n;
    if (threadIdx.x == 0) {
        mean[c] = mu;
        invstd[c] = 1.0f / sqrtf(var + eps);
        run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * mu;
        run_var[c] = (1.0f - momentum) * run_var[c] + momentum * (n > 1 ? var * (float)n / (float)(n - 1) : var);
    }
}

// a = relu(gamma * (z - mean) * invstd + beta [+ res])
__global__ void k_bn_act(const float *__restrict__ z, int c_n, int B, const float *__restrict__ mean,
                         const float *__restrict__ invstd, const float *__restrict__ gamma,
                         const float *__restrict__ beta, const float *__restrict__ res, float *__restrict__ a) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * c_n * kCells) return;
    const int c = (int)((i / kCells) % c_n);
    float y = gamma[c] * ((z[i] - mean[c]) * invstd[c]) + beta[c];
    if (res) y += res[i];
    a[i] = fmaxf(y, 0.f);
}

// backward of a = relu(bn(z) [+ res]): dy = da * (a > 0); per channel
// dbeta = sum dy, dgamma = sum dy * xhat;  dz = gamma*invstd/N * (N dy - dbeta - xhat dgamma)
__global__ __launch_bounds__(kThreads) void k_bn_bwd(const float *__restrict__ da, const float *__restrict__ a,
                                                     const float *__restrict__ z, int c_n, int B,
                                                     const float *__restrict__ mean, const float *__restrict__ invstd,
                                                     const float *__restrict__ gamma, float *__restrict__ dgamma,
                                                     float *__restrict__ dbeta, float *__restrict__ dz) {
    __shared__ float red[kThreads];
    const int c = blockIdx.x, n = B * kCells;
    const float mu = mean[c], is = invstd[c];
    float s1 = 0.f, s2 = 0.f;
    for (int i = threadIdx.x; i < n; i += kThreads) {
        const size_t k = ((size_t)(i / kCells) * c_n + c) * kCells + i % kCells;
        const float dy = a[k] > 0.f ? da[k] : 0.f;
        s1 += dy;
        s2 += dy * ((z[k] - mu) * is);
    }
    const float sb = block_sum(s1, red), sg = block_sum(s2, red);
    if (threadIdx.x == 0) {
        dbeta[c] = sb;
        dgamma[c] = sg;
    }
    const float g = gamma[c] * is / (float)n;
    for (int i = threadIdx.x; i < n; i += kThreads) {
        const size_t k = ((size_t)(i / kCells) * c_n + c) * kCells + i % kCells;
        const float dy = a[k] > 0.f ? da[k] : 0.f;
        dz[k] = g * ((float)n * dy - sb - ((z[k] - mu) * is) * sg);
    }
}

// dt = da * (a > 0) (the residual block's skip-path gradient)
__global__ void k_relu_mask(const float *__restrict__ da, const float *__restrict__ a, size_t n, float *__restrict__ dt) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dt[i] = a[i] > 0.f ? da[i] : 0.f;
}

// ------------------------------------------------------------------ heads + loss
// one workgroup per sample: policy logits (1344 -> 7), value (126 -> 1, tanh),
// loss terms and the output gradients
//   dlogits = (softmax * sum(pi) - pi) / B,  dpre = 2 (v - z) / B * (1 - v^2)
__global__ __launch_bounds__(kThreads) void k_heads_loss(const float *__restrict__ rp, const float *__restrict__ rv,
                                                         const float *__restrict__ wp, const float *__restrict__ bp,
                                                         const float *__restrict__ wv, const float *__restrict__ bv,
                                                         const float *__restrict__ pi, const float *__restrict__ zv,
                                                         int B, float *__restrict__ dlogits, float *__restrict__ dpre,
                                                         float *__restrict__ loss_terms) {
    __shared__ float red[kThreads];
    const int b = blockIdx.x;
    const float *xp = rp + (size_t)b * 32 * kCells, *xv = rv + (size_t)b * 3 * kCells;
    float lg[7];
    for (int o = 0; o < 7; ++o) {
        float s = 0.f;
        for (int k = threadIdx.x; k < 32 * kCells; k += kThreads) s += xp[k] * wp[o * 32 * kCells + k];
        lg[o] = block_sum(s, red) + bp[o];
    }
    float s = 0.f;
    for (int k = threadIdx.x; k < 3 * kCells; k += kThreads) s += xv[k] * wv[k];
    const float pre = block_sum(s, red) + bv[0];
    if (threadIdx.x == 0) {
        float mx = lg[0];
        for (int o = 1; o < 7; ++o) mx = fmaxf(mx, lg[o]);
        float se = 0.f;
        for (int o = 0; o < 7; ++o) se += expf(lg[o] - mx);
        const float lse = mx + logf(se);
        float nll = 0.f, spi = 0.f;
        for (int o = 0; o < 7; ++o) {
            nll += (lg[o] - lse) * pi[b * 7 + o];
            spi += pi[b * 7 + o];
        }
        for (int o = 0; o < 7; ++o) dlogits[b * 7 + o] = (expf(lg[o] - lse) * spi - pi[b * 7 + o]) / (float)B;
        const float v = tanhf(pre), d = v - zv[b];
        dpre[b] = 2.0f * d / (float)B * (1.0f - v * v);
        loss_terms[2 * b] = -nll;      // policy term of sample b
        loss_terms[2 * b + 1] = d * d; // value term
    }
}

// linear backward, out features O, in features K:
//   dW[o][k] = sum_b dy[b][o] x[b][k];  db[o] = sum_b dy[b][o];  dx[b][k] = sum_o dy[b][o] W[o][k]
__global__ void k_linear_bwd_w(const float *__restrict__ x, const float *__restrict__ dy, int B, int O, int K,
                               float *__restrict__ dw, float *__restrict__ db) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < O * K) {
        const int o = i / K, k = i - o * K;
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += dy[b * O + o] * x[(size_t)b * K + k];
        dw[i] = s;
    }
    if (i < O) {
        float s = 0.f;
        for (int b = 0; b < B; ++b) s += dy[b * O + i];
        db[i] = s;
    }
}

__global__ void k_linear_bwd_x(const float *__restrict__ dy, const float *__restrict__ w, int B, int O, int K,
                               float *__restrict__ dx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)B * K) return;
    const int b = (int)(i / K), k = (int)(i - (size_t)b * K);
    float s = 0.f;
    for (int o = 0; o < O; ++o) s += dy[b * O + o] * w[o * K + k];
    dx[i] = s;
}

// ------------------------------------------------------------------ Adam (torch semantics)
// m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;
// p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)      (g scaled by gscale)
__global__ void k_adam(float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                       float *__restrict__ v, size_t n, float gscale, float lr, float b1, float b2, float eps,
                       float bc1, float bc2_sqrt) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i] * gscale;
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= (lr / bc1) * (mi / (sqrtf(vi) / bc2_sqrt + eps));
}

// running stats gathered into / scattered from a packed buffer (cross-rank average)
__global__ void k_gather(const float *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t n,
                         float *__restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}
__global__ void k_scatter_scaled(const float *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t n,
                                 float scale, float *__restrict__ dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[idx[i]] = src[i] * scale;
}

inline unsigned blocks_of(size_t n, int t = kThreads) { return (unsigned)((n + t - 1) / t); }

}  // namespace
}  // namespace spai

// ---------------------------------------------------------------------- host
namespace spai {
namespace {

int learner_alloc_batch(spai_learner *L, uint32_t B) {
    if (B <= L->max_batch) return SPAI_OK;
    const size_t act = (size_t)B * std::max(L->hidden, 32) * kCells;   // also the 32-channel policy head
    SPAI_TRY(L->x_in.alloc((size_t)B * 3 * kCells));
    SPAI_TRY(L->pi.alloc((size_t)B * 7));
    SPAI_TRY(L->zv.alloc(B));
    for (size_t l = 0; l < L->convs.size(); ++l) {
        SPAI_TRY(L->z[l].alloc((size_t)B * L->convs[l].co * kCells));
        SPAI_TRY(L->a[l].alloc((size_t)B * L->convs[l].co * kCells));
    }
    SPAI_TRY(L->d0.alloc(act));
    SPAI_TRY(L->d1.alloc(act));
    SPAI_TRY(L->d2.alloc(act));
    SPAI_TRY(L->dlogits.alloc((size_t)B * 7));
    SPAI_TRY(L->dpre.alloc(B));
    SPAI_TRY(L->loss_terms.alloc((size_t)B * 2));
    L->max_batch = B;
    return SPAI_OK;
}

void launch_conv(const float *in, int ci, const float *w, const float *bias, int co, float *out, int B, bool acc,
                 hipStream_t st) {
    const int cob = std::min(16, co);
    const size_t lds = ((size_t)ci * kPad + (size_t)cob * ci * 9) * sizeof(float);
    k_conv3x3<<<dim3((co + cob - 1) / cob, B), kThreads, lds, st>>>(in, ci, w, bias, co, cob, out, acc ? 1 : 0);
}

// dW, db of one conv: split-batch partials, then a fixed-order sum
void launch_wgrad(spai_learner *L, const float *x, int ci, const float *dz, int co, int B, float *dw, float *db,
                  hipStream_t st) {
    const size_t lds = ((size_t)ci * kPad + kCells) * sizeof(float);
    const int ny = std::min(kWgradSplit, B);
    k_conv_wgrad_part<<<dim3(co, ny), kThreads, lds, st>>>(x, ci, dz, co, B, L->wpart.p, L->bpart.p);
    k_sum_parts<<<blocks_of((size_t)co * ci * 9), kThreads, 0, st>>>(L->wpart.p, co * ci * 9, ny, dw);
    k_sum_parts<<<blocks_of(co), kThreads, 0, st>>>(L->bpart.p, co, ny, db);
}

// data gradient of one conv: dx (+)= conv(dz, flip-transposed w)
void launch_dgrad(spai_learner *L, const float *dz, int co, const float *w, int ci, float *dx, int B, bool acc,
                  hipStream_t st) {
    k_flip_transpose<<<blocks_of((size_t)co * ci * 9), kThreads, 0, st>>>(w, co, ci, L->wt.p);
    launch_conv(dz, co, L->wt.p, nullptr, ci, dx, B, acc, st);
}

}  // namespace

int learner_create(spai_engine *e, int blocks, int hidden, const float *params, size_t n, const spai_adam_config *cfg,
                   spai_learner **out) {
    SPAI_CHECK(e->game == SPAI_GAME_CONNECT4, SPAI_ERR_UNSUPPORTED, "learner: only Connect4 is built");
    SPAI_CHECK(hidden >= 1 && hidden <= 64, SPAI_ERR_UNSUPPORTED, "learner: hidden 1..64 (got %d)", hidden);
    SPAI_CHECK(blocks >= 0 && blocks <= 40, SPAI_ERR_UNSUPPORTED, "learner: 0..40 blocks (got %d)", blocks);
    SPAI_CHECK(params && n == net_num_params(e->game, blocks, hidden), SPAI_ERR_INVALID, "expected %zu params, got %zu",
               net_num_params(e->game, blocks, hidden), n);
    spai_learner *L = new spai_learner();
    L->eng = e;
    L->blocks = blocks;
    L->hidden = hidden;
    if (cfg) L->cfg = *cfg;
    else spai_adam_config_default(&L->cfg);
    size_t off = 0;
    auto conv = [&](int ci, int co) {
        spai_learner::Conv c{ci, co, 0, 0, 0, 0, 0, 0};
        c.w = off;
        off += (size_t)co * ci * 9;
        c.b = off;
        off += co;
        c.g = off;
        c.be = off + co;
        c.mu = off + 2 * co;
        c.var = off + 3 * co;
        off += 4 * (size_t)co;
        L->convs.push_back(c);
    };
    conv(3, hidden);
    for (int i = 0; i < 2 * blocks; ++i) conv(hidden, hidden);
    conv(hidden, 32);
    L->pol_w = off;
    off += 7 * 32 * kCells;
    L->pol_b = off;
    off += 7;
    conv(hidden, 3);
    L->val_w = off;
    off += 3 * kCells;
    L->val_b = off;
    off += 1;
    L->n_params = off;
    int rc = SPAI_OK;
    auto chk = [&](int r) {
        if (rc == SPAI_OK) rc = r;
    };
    chk(L->p.alloc(n));
    chk(L->g.alloc(n));
    chk(L->m.alloc(n));
    chk(L->v.alloc(n));
    const size_t cmax = (size_t)std::max(hidden, 32);
    chk(L->wt.alloc(cmax * hidden * 9));
    chk(L->wpart.alloc((size_t)kWgradSplit * cmax * hidden * 9));
    chk(L->bpart.alloc((size_t)kWgradSplit * cmax));
    L->z.resize(L->convs.size());
    L->a.resize(L->convs.size());
    L->mean.resize(L->convs.size());
    L->invstd.resize(L->convs.size());
    std::vector<uint32_t> ridx;
    for (size_t l = 0; l < L->convs.size(); ++l) {
        chk(L->mean[l].alloc(L->convs[l].co));
        chk(L->invstd[l].alloc(L->convs[l].co));
        for (int c = 0; c < L->convs[l].co; ++c) ridx.push_back((uint32_t)(L->convs[l].mu + c));
        for (int c = 0; c < L->convs[l].co; ++c) ridx.push_back((uint32_t)(L->convs[l].var + c));
    }
    chk(L->run_idx.alloc(ridx.size()));
    chk(L->run_buf.alloc(ridx.size()));
    if (rc == SPAI_OK) {
        hipStream_t st = e->stream;
        if (hipMemcpyAsync(L->p.p, params, n * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(L->run_idx.p, ridx.data(), ridx.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(L->m.p, 0, n * 4, st) != hipSuccess || hipMemsetAsync(L->v.p, 0, n * 4, st) != hipSuccess ||
            hipMemsetAsync(L->g.p, 0, n * 4, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            set_error("learner: upload failed");
            rc = SPAI_ERR_DEVICE;
        }
    }
    if (rc != SPAI_OK) {
        learner_destroy(L);
        return rc;
    }
    *out = L;
    return SPAI_OK;
}

void learner_destroy(spai_learner *L) {
    if (!L) return;
    if (L->eng) (void)hipStreamSynchronize(L->eng->stream);
    if (L->comm) (void)ncclCommDestroy((ncclComm_t)L->comm);
    for (auto *b : {&L->p, &L->g, &L->m, &L->v, &L->wt, &L->x_in, &L->pi, &L->zv, &L->d0, &L->d1, &L->d2, &L->dlogits,
                    &L->dpre, &L->loss_terms, &L->wpart, &L->bpart, &L->run_buf})
        b->release();
    L->run_idx.release();
    for (auto *vec : {&L->z, &L->a, &L->mean, &L->invstd})
        for (auto &b : *vec) b.release();
    delete L;
}

int learner_train_batch(spai_learner *L, uint32_t B, const float *states, const float *policies, const float *values,
                        float *loss3) {
    SPAI_CHECK(B >= 1, SPAI_ERR_INVALID, "train_batch: empty batch");
    SPAI_TRY(learner_alloc_batch(L, B));
    hipStream_t st = L->eng->stream;
    const int H = L->hidden;
    float *P = L->p.p, *G = L->g.p;
    SPAI_HIP(hipMemcpyAsync(L->x_in.p, states, (size_t)B * 3 * kCells * 4, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(L->pi.p, policies, (size_t)B * 7 * 4, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemcpyAsync(L->zv.p, values, (size_t)B * 4, hipMemcpyHostToDevice, st));
    SPAI_HIP(hipMemsetAsync(G, 0, L->n_params * 4, st));
    const float eps = L->cfg.bn_eps, mom = L->cfg.bn_momentum;
    const size_t nl = L->convs.size();
    const int pol = (int)nl - 2, val = (int)nl - 1;

    // ---------------- forward (train mode)
    auto conv_bn_act = [&](int l, const float *in, const float *res) {
        const spai_learner::Conv &c = L->convs[l];
        launch_conv(in, c.ci, P + c.w, P + c.b, c.co, L->z[l].p, (int)B, false, st);
        k_bn_stats<<<c.co, kThreads, 0, st>>>(L->z[l].p, c.co, (int)B, eps, mom, L->mean[l].p, L->invstd[l].p, P + c.mu,
                                              P + c.var);
        k_bn_act<<<blocks_of((size_t)B * c.co * kCells), kThreads, 0, st>>>(L->z[l].p, c.co, (int)B, L->mean[l].p,
                                                                          L->invstd[l].p, P + c.g, P + c.be, res,
                                                                          L->a[l].p);
    };
    conv_bn_act(0, L->x_in.p, nullptr);
    const float *h = L->a[0].p;
    for (int k = 0; k < L->blocks; ++k) {   // relu(h + BN(conv(relu(BN(conv(h)))))) (model/mod.rs:152-165)
        conv_bn_act(1 + 2 * k, h, nullptr);
        conv_bn_act(2 + 2 * k, L->a[1 + 2 * k].p, h);
        h = L->a[2 + 2 * k].p;
    }
    conv_bn_act(pol, h, nullptr);
    conv_bn_act(val, h, nullptr);
    k_heads_loss<<<B, kThreads, 0, st>>>(L->a[pol].p, L->a[val].p, P + L->pol_w, P + L->pol_b, P + L->val_w,
                                         P + L->val_b, L->pi.p, L->zv.p, (int)B, L->dlogits.p, L->dpre.p,
                                         L->loss_terms.p);

    // ---------------- backward
    const size_t nact = (size_t)B * H * kCells;
    // heads: linears -> relu/BN -> conv; dh (d0) = dgrad(policy) + dgrad(value)
    k_linear_bwd_w<<<blocks_of(7 * 32 * kCells), kThreads, 0, st>>>(L->a[pol].p, L->dlogits.p, (int)B, 7, 32 * kCells,
                                                                     G + L->pol_w, G + L->pol_b);
    k_linear_bwd_x<<<blocks_of((size_t)B * 32 * kCells), kThreads, 0, st>>>(L->dlogits.p, P + L->pol_w, (int)B, 7,
                                                                             32 * kCells, L->d1.p);
    auto bn_conv_bwd = [&](int l, const float *da, const float *in, float *dx, bool acc) {
        const spai_learner::Conv &c = L->convs[l];
        k_bn_bwd<<<c.co, kThreads, 0, st>>>(da, L->a[l].p, L->z[l].p, c.co, (int)B, L->mean[l].p, L->invstd[l].p,
                                            P + c.g, G + c.g, G + c.be, L->d2.p);
        launch_wgrad(L, in, c.ci, L->d2.p, c.co, (int)B, G + c.w, G + c.b, st);
        if (dx) launch_dgrad(L, L->d2.p, c.co, P + c.w, c.ci, dx, (int)B, acc, st);
    };
    bn_conv_bwd(pol, L->d1.p, h, L->d0.p, false);
    k_linear_bwd_w<<<blocks_of(3 * kCells), kThreads, 0, st>>>(L->a[val].p, L->dpre.p, (int)B, 1, 3 * kCells,
                                                                G + L->val_w, G + L->val_b);
    k_linear_bwd_x<<<blocks_of((size_t)B * 3 * kCells), kThreads, 0, st>>>(L->dpre.p, P + L->val_w, (int)B, 1,
                                                                            3 * kCells, L->d1.p);
    bn_conv_bwd(val, L->d1.p, h, L->d0.p, true);
    // residual blocks in reverse; d0 holds dL/d(block output)
    for (int k = L->blocks - 1; k >= 0; --k) {
        const int l1 = 1 + 2 * k, l2 = 2 + 2 * k;
        const float *hin = k == 0 ? L->a[0].p : L->a[l2 - 2].p;
        // dt = d(out) * (out > 0): gradient of the pre-ReLU sum, shared by the skip path and BN2
        k_relu_mask<<<blocks_of(nact), kThreads, 0, st>>>(L->d0.p, L->a[l2].p, nact, L->d1.p);
        // BN2/conv2 backward on dy2 = dt (the mask a[l2] > 0 inside k_bn_bwd is idempotent on dt);
        // conv2's input is a[l1]; its data gradient overwrites d0 with dL/d(relu1 output)
        {
            const spai_learner::Conv &c = L->convs[l2];
            k_bn_bwd<<<c.co, kThreads, 0, st>>>(L->d1.p, L->a[l2].p, L->z[l2].p, c.co, (int)B, L->mean[l2].p,
                                                L->invstd[l2].p, P + c.g, G + c.g, G + c.be, L->d2.p);
            launch_wgrad(L, L->a[l1].p, c.ci, L->d2.p, c.co, (int)B, G + c.w, G + c.b, st);
            launch_dgrad(L, L->d2.p, c.co, P + c.w, c.ci, L->d0.p, (int)B, false, st);
        }
        // BN1/conv1 backward: da = d0 (gradient wrt relu1 output), mask a[l1]; its input is hin;
        // dgrad accumulates into d1 (= dt, the skip gradient) -> d(block input)
        bn_conv_bwd(l1, L->d0.p, hin, L->d1.p, true);
        std::swap(L->d0, L->d1);   // d0 = dL/d(block input)
    }
    // stem: no data gradient
    bn_conv_bwd(0, L->d0.p, L->x_in.p, nullptr, false);

    // ---------------- cross-rank reduction + Adam
    float gscale = 1.0f;
    if (L->comm) {   // (a 1-rank communicator reduces to a copy)
        if (ncclAllReduce(G, G, L->n_params, ncclFloat32, ncclSum, (ncclComm_t)L->comm, st) != ncclSuccess) {
            set_error("ncclAllReduce of the gradients failed");
            return SPAI_ERR_DEVICE;
        }
        gscale = 1.0f / (float)L->world;
    }
    L->step += 1;
    const double t = (double)L->step;
    const float bc1 = (float)(1.0 - std::pow((double)L->cfg.beta1, t));
    const float bc2s = (float)std::sqrt(1.0 - std::pow((double)L->cfg.beta2, t));
    k_adam<<<blocks_of(L->n_params), kThreads, 0, st>>>(P, G, L->m.p, L->v.p, L->n_params, gscale, L->cfg.lr,
                                                        L->cfg.beta1, L->cfg.beta2, L->cfg.eps, bc1, bc2s);
    if (L->comm) {   // average the BN running statistics so replicas stay identical
        const uint32_t nr = (uint32_t)L->run_idx.n;
        k_gather<<<blocks_of(nr), kThreads, 0, st>>>(P, L->run_idx.p, nr, L->run_buf.p);
        if (ncclAllReduce(L->run_buf.p, L->run_buf.p, nr, ncclFloat32, ncclSum, (ncclComm_t)L->comm, st) != ncclSuccess) {
            set_error("ncclAllReduce of the BN running statistics failed");
            return SPAI_ERR_DEVICE;
        }
        k_scatter_scaled<<<blocks_of(nr), kThreads, 0, st>>>(L->run_buf.p, L->run_idx.p, nr, 1.0f / (float)L->world, P);
    }
    SPAI_HIP(hipGetLastError());
    std::vector<float> terms((size_t)B * 2);
    SPAI_HIP(hipMemcpyAsync(terms.data(), L->loss_terms.p, terms.size() * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    double lp = 0, lv = 0;   // fixed-order host sums
    for (uint32_t b = 0; b < B; ++b) {
        lp += terms[2 * b];
        lv += terms[2 * b + 1];
    }
    if (loss3) {
        loss3[1] = (float)(lp / B);
        loss3[2] = (float)(lv / B);
        loss3[0] = loss3[1] + loss3[2];
    }
    return SPAI_OK;
}

int learner_params(spai_learner *L, float *params, size_t n, bool grads) {
    SPAI_CHECK(n == L->n_params, SPAI_ERR_INVALID, "expected %zu params, got %zu", L->n_params, n);
    hipStream_t st = L->eng->stream;
    SPAI_HIP(hipMemcpyAsync(params, grads ? L->g.p : L->p.p, n * 4, hipMemcpyDeviceToHost, st));
    SPAI_HIP(hipStreamSynchronize(st));
    return SPAI_OK;
}

int learner_set_comm(spai_learner *L, int rank, int world, const uint8_t *id) {
    SPAI_CHECK(world >= 1 && rank >= 0 && rank < world, SPAI_ERR_INVALID, "bad rank %d / world %d", rank, world);
    if (L->comm) {
        (void)ncclCommDestroy((ncclComm_t)L->comm);
        L->comm = nullptr;
    }
    L->rank = rank;
    L->world = world;
    if (!id) return SPAI_OK;   // world == 1 without an id: no communicator
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == SPAI_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(uid.internal, id, SPAI_COMM_ID_BYTES);
    SPAI_HIP(hipSetDevice(L->eng->device));
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, world, uid, rank);
    SPAI_CHECK(r == ncclSuccess, SPAI_ERR_DEVICE, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
    L->comm = c;
    return SPAI_OK;
}

int comm_unique_id(uint8_t *id) {
    ncclUniqueId uid;
    const ncclResult_t r = ncclGetUniqueId(&uid);
    SPAI_CHECK(r == ncclSuccess, SPAI_ERR_DEVICE, "ncclGetUniqueId failed: %s", ncclGetErrorString(r));
    memcpy(id, uid.internal, SPAI_COMM_ID_BYTES);
    return SPAI_OK;
}

}  // namespace spai

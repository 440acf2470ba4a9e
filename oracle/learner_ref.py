"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a numpy float64
restatement of the reference training step, ModelTrainerWorker::train_batch
(learner_concurrent.rs:72-85):

  * Net::forward(x, train=true) (model/mod.rs:152-184, model/connect_four.rs:50-81):
    stem conv3x3+BN+ReLU, blocks relu(x + BN(conv(relu(BN(conv(x)))))),
    policy head conv(64->32)+BN+ReLU, flatten (NCHW), linear 1344->7;
    value head conv(64->3)+BN+ReLU, flatten, linear 126->1, tanh.
    BatchNorm in train mode (libtorch batch_norm, via tch 0.13 / libtorch 2.0,
    not vendored): batch mean and biased variance over (B, 6, 7) normalise;
    running stats r <- (1 - 0.1) r + 0.1 * stat with the unbiased variance.
  * loss = -(log_softmax(p) * pi).sum() / B + mean((v - z)^2)   (model/mod.rs:128-135)
  * backward, then Adam (libtorch torch::optim::Adam as tch's Adam::default():
    beta 0.9/0.999, eps 1e-8, no weight decay, lr 1e-3, model/mod.rs:107):
    m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
    p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).

Parameters are the flat construction-order vector of spai_net_create.
Pinned against PyTorch CPU fp32 (tests/golden/learner_c4_1x64.npz, made by
tests/golden/gen_golden.py) in tests/test_oracle_golden.py.
"""
import numpy as np

ROWS, COLS, CELLS = 6, 7, 42


def _layout(blocks, hidden):
    """offsets of every tensor in the flat parameter vector"""
    convs, off = [], 0

    def conv(ci, co):
        nonlocal off
        c = dict(ci=ci, co=co, w=off)
        off += co * ci * 9
        c["b"] = off
        off += co
        c["g"], c["be"], c["mu"], c["var"] = off, off + co, off + 2 * co, off + 3 * co
        off += 4 * co
        convs.append(c)

    conv(3, hidden)
    for _ in range(2 * blocks):
        conv(hidden, hidden)
    conv(hidden, 32)
    lin = {"pw": off}
    off += 7 * 32 * CELLS
    lin["pb"] = off
    off += 7
    conv(hidden, 3)
    lin["vw"] = off
    off += 3 * CELLS
    lin["vb"] = off
    off += 1
    return convs, lin, off


def _im2col(x):
    """[B][C][6][7] -> [B*42][C*9], column order (ci, kh, kw) = w.reshape(co, ci*9)"""
    B, C = x.shape[:2]
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)))
    cols = np.empty((B, C, 9, ROWS, COLS), x.dtype)
    for t in range(9):
        kh, kw = divmod(t, 3)
        cols[:, :, t] = xp[:, :, kh:kh + ROWS, kw:kw + COLS]
    return cols.transpose(0, 3, 4, 1, 2).reshape(B * CELLS, C * 9)


def _col2im(dcols, B, C):
    d = dcols.reshape(B, ROWS, COLS, C, 9).transpose(0, 3, 4, 1, 2)
    dxp = np.zeros((B, C, ROWS + 2, COLS + 2), dcols.dtype)
    for t in range(9):
        kh, kw = divmod(t, 3)
        dxp[:, :, kh:kh + ROWS, kw:kw + COLS] += d[:, :, t]
    return dxp[:, :, 1:-1, 1:-1]


def train_step(params, adam_m, adam_v, step, x, pi, z, blocks, hidden, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8,
               momentum=0.1, bn_eps=1e-5, masks=None, diag=None):
    """one optimizer step; returns (new params, m, v, loss[3], grads) — all float64.

    masks: optional per-conv-layer boolean [B][co][6][7] ReLU masks to use instead of
    (pre-activation > 0) — e.g. the device step's own (post-ReLU activation > 0), so
    that a pre-activation within rounding of 0 takes the same side of the kink in
    both.  diag: optional dict that receives the pre-activations ("pre", per layer)."""
    P, G, loss = forward_backward(params, x, pi, z, blocks, hidden, momentum, bn_eps, masks, diag)
    P, m, vv = adam(P, G, adam_m, adam_v, step, lr, b1, b2, eps)
    return P, m, vv, loss, G


def adam(P, G, adam_m, adam_v, step, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """Adam (running statistics have zero gradient, so their moments stay 0 and they are not moved)"""
    m = b1 * np.asarray(adam_m, np.float64) + (1 - b1) * G
    vv = b2 * np.asarray(adam_v, np.float64) + (1 - b2) * G * G
    t = step + 1
    P = P - (lr / (1 - b1 ** t)) * m / (np.sqrt(vv) / np.sqrt(1 - b2 ** t) + eps)
    return P, m, vv


def train_step_dp(params, adam_m, adam_v, step, rank_batches, blocks, hidden, lr=1e-3, b1=0.9, b2=0.999,
                  eps=1e-8, momentum=0.1, bn_eps=1e-5, rank_masks=None, rank_diags=None):
    """one data-parallel optimizer step over len(rank_batches) ranks, as DDP without
    SyncBN (the distribution learner_concurrent.rs:72-85 would get from torch DDP):
    every rank runs the train-mode forward/backward on its own batch (its own BN
    batch statistics, its own running-statistic update), the step's gradient is the
    mean over the union of the batches, sum_r (B_r / sum B) * g_r, one Adam step on
    it, and the running statistics are the ranks' updated ones averaged.  Returns
    (params, m, v, per-rank losses, the reduced gradient, per-rank gradients)."""
    parts = []
    for r, (x, pi, z) in enumerate(rank_batches):
        parts.append(forward_backward(params, x, pi, z, blocks, hidden, momentum, bn_eps,
                                      None if rank_masks is None else rank_masks[r],
                                      None if rank_diags is None else rank_diags[r]))
    sizes = np.array([len(np.asarray(b[2]).reshape(-1)) for b in rank_batches], np.float64)
    G = sum((sizes[r] / sizes.sum()) * parts[r][1] for r in range(len(parts)))
    convs, _, _ = _layout(blocks, hidden)
    P = np.asarray(parts[0][0], np.float64).copy()
    for c in convs:   # running statistics: the mean of the ranks' updated values
        for key in ("mu", "var"):
            sl = slice(c[key], c[key] + c["co"])
            P[sl] = np.mean([p[0][sl] for p in parts], axis=0)
    P, m, vv = adam(P, G, adam_m, adam_v, step, lr, b1, b2, eps)
    return P, m, vv, [p[2] for p in parts], G, [p[1] for p in parts]


def forward_backward(params, x, pi, z, blocks, hidden, momentum=0.1, bn_eps=1e-5, masks=None, diag=None):
    """train-mode forward + backward of one batch; returns (params with the BN running
    statistics updated, gradients, loss[3]) — float64"""
    convs, lin, n = _layout(blocks, hidden)
    P = np.asarray(params, np.float64).copy()
    G = np.zeros(n)
    B = x.shape[0]
    x = np.asarray(x, np.float64).reshape(B, 3, ROWS, COLS)
    cache = []

    def conv_bn_act(l, inp, res=None):
        c = convs[l]
        ci, co = c["ci"], c["co"]
        W = P[c["w"]:c["w"] + co * ci * 9].reshape(co, ci * 9)
        cols = _im2col(inp)
        zz = (cols @ W.T + P[c["b"]:c["b"] + co]).reshape(B, ROWS, COLS, co).transpose(0, 3, 1, 2)
        mu = zz.mean((0, 2, 3))
        var = zz.var((0, 2, 3))
        nn_ = B * CELLS
        P[c["mu"]:c["mu"] + co] = (1 - momentum) * P[c["mu"]:c["mu"] + co] + momentum * mu
        P[c["var"]:c["var"] + co] = (1 - momentum) * P[c["var"]:c["var"] + co] + momentum * var * nn_ / (nn_ - 1)
        inv = 1.0 / np.sqrt(var + bn_eps)
        xhat = (zz - mu[None, :, None, None]) * inv[None, :, None, None]
        y = P[c["g"]:c["g"] + co][None, :, None, None] * xhat + P[c["be"]:c["be"] + co][None, :, None, None]
        if res is not None:
            y = y + res
        mask = (y > 0.0) if masks is None else np.asarray(masks[l], bool).reshape(y.shape)
        a = np.where(mask, y, 0.0)
        if diag is not None:
            diag.setdefault("pre", [None] * len(convs))[l] = y
        cache[l] = dict(cols=cols, W=W, xhat=xhat, inv=inv, a=a, m=mask, inp_shape=inp.shape)
        return a

    cache = [None] * len(convs)
    h = conv_bn_act(0, x)
    for k in range(blocks):
        r1 = conv_bn_act(1 + 2 * k, h)
        h = conv_bn_act(2 + 2 * k, r1, res=h)
    npol, nval = len(convs) - 2, len(convs) - 1
    rp = conv_bn_act(npol, h).reshape(B, -1)
    rv = conv_bn_act(nval, h).reshape(B, -1)
    Wp = P[lin["pw"]:lin["pw"] + 7 * 32 * CELLS].reshape(7, -1)
    Wv = P[lin["vw"]:lin["vw"] + 3 * CELLS].reshape(1, -1)
    logits = rp @ Wp.T + P[lin["pb"]:lin["pb"] + 7]
    pre = (rv @ Wv.T + P[lin["vb"]:lin["vb"] + 1]).reshape(-1)
    v = np.tanh(pre)
    lse = np.log(np.exp(logits - logits.max(1, keepdims=True)).sum(1)) + logits.max(1)
    logsm = logits - lse[:, None]
    pi = np.asarray(pi, np.float64).reshape(B, 7)
    zz_ = np.asarray(z, np.float64).reshape(-1)
    lp = -(logsm * pi).sum() / B
    lv = ((v - zz_) ** 2).mean()
    # backward
    dlogits = (np.exp(logsm) * pi.sum(1, keepdims=True) - pi) / B
    dpre = 2.0 * (v - zz_) / B * (1.0 - v * v)
    G[lin["pw"]:lin["pw"] + Wp.size] = (dlogits.T @ rp).reshape(-1)
    G[lin["pb"]:lin["pb"] + 7] = dlogits.sum(0)
    G[lin["vw"]:lin["vw"] + Wv.size] = (dpre[:, None].T @ rv).reshape(-1)
    G[lin["vb"]] = dpre.sum()

    def bn_conv_bwd(l, da, want_dx=True):
        c, cc = convs[l], cache[l]
        co, ci = c["co"], c["ci"]
        dy = da * cc["m"]
        xhat, inv = cc["xhat"], cc["inv"]
        nn_ = B * CELLS
        sb = dy.sum((0, 2, 3))
        sg = (dy * xhat).sum((0, 2, 3))
        G[c["be"]:c["be"] + co] = sb
        G[c["g"]:c["g"] + co] = sg
        gam = P[c["g"]:c["g"] + co]  # gamma is not changed by the forward
        dz = (gam * inv / nn_)[None, :, None, None] * (nn_ * dy - sb[None, :, None, None] - xhat * sg[None, :, None, None])
        dzf = dz.transpose(0, 2, 3, 1).reshape(B * CELLS, co)
        G[c["w"]:c["w"] + co * ci * 9] = (dzf.T @ cc["cols"]).reshape(-1)
        G[c["b"]:c["b"] + co] = dzf.sum(0)
        if not want_dx:
            return None
        return _col2im(dzf @ cc["W"], B, ci)

    dh = bn_conv_bwd(npol, (dlogits @ Wp).reshape(B, 32, ROWS, COLS))
    dh = dh + bn_conv_bwd(nval, (dpre[:, None] @ Wv).reshape(B, 3, ROWS, COLS))
    for k in reversed(range(blocks)):
        l1, l2 = 1 + 2 * k, 2 + 2 * k
        dt = dh * cache[l2]["m"]
        dr1 = bn_conv_bwd(l2, dt)
        dh = dt + bn_conv_bwd(l1, dr1)
    bn_conv_bwd(0, dh, want_dx=False)
    return P, G, np.array([lp + lv, lp, lv])


def train(params, batches, blocks, hidden, **kw):
    """run train_step over [(x, pi, z), ...]; returns params, losses, grads of each step"""
    n = len(params)
    m, v = np.zeros(n), np.zeros(n)
    P = np.asarray(params, np.float64)
    losses, grads = [], []
    for k, (x, pi, z) in enumerate(batches):
        P, m, v, loss, g = train_step(P, m, v, k, x, pi, z, blocks, hidden, **kw)
        losses.append(loss)
        grads.append(g)
    return P, np.array(losses), grads

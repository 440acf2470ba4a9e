#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Runs in the build container only (needs torch CPU).  The reference itself
(Rust + tch 0.13, hardcoded Device::Mps) cannot be built or run here and it
ships no tests or fixtures, so the fixtures come from two restatements that
are independent of the C oracle under oracle/:

* a pure-Python line-by-line transliteration of the reference rules
  (game/connect_four.rs:128-283, game/tictactoe.rs:127-241), the MCTS
  (mcts.rs:91-192,214-331) and the self-play loop
  (learner_concurrent.rs:169-242), driven by the deterministic hash stub
  evaluator and the Philox sampler that the oracle and the engine share;
* the net forward (model/mod.rs:36-98,152-184, model/connect_four.rs:50-81,
  model/tictactoe.rs:50-81) in PyTorch CPU fp32 -- the same libtorch
  conv2d / batch_norm / linear / softmax ops that tch wraps.

Outputs (all small):
  rules_c4.json, rules_ttt.json   random-game traces + hand-derived KATs
  mcts_hash.json                  root visits after K sims, self-play streams
  net_c4_2x64.npz, net_ttt_2x64.npz  params, inputs, logits, values, priors
"""
import ctypes
import ctypes.util
import json
import math
import os
import sys
import random
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

# ---------------------------------------------------------------- f32 helpers
def f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def fadd(a, b):
    return f32(a + b)


def fmul(a, b):
    return f32(a * b)


def fdiv(a, b):
    if b == 0.0:  # IEEE semantics (Rust f32 division never traps)
        return math.nan if (a == 0.0 or math.isnan(a)) else math.copysign(math.inf, a) * math.copysign(1.0, b)
    return f32(a / b)


def nd_sum(xs):
    """ndarray 0.15 sum() = numeric_util::unrolled_fold over a contiguous slice."""
    p = [0.0] * 8
    i = 0
    n = len(xs)
    while n - i >= 8:
        for k in range(8):
            p[k] = fadd(p[k], xs[i + k])
        i += 8
    acc = 0.0
    acc = fadd(acc, fadd(p[0], p[4]))
    acc = fadd(acc, fadd(p[1], p[5]))
    acc = fadd(acc, fadd(p[2], p[6]))
    acc = fadd(acc, fadd(p[3], p[7]))
    while i < n:
        acc = fadd(acc, xs[i])
        i += 1
    return acc


# ---------------------------------------------------------------- Connect4
ONGOING, TIED, WON = 0, 1, 2
X, O = 1, 2


class C4:
    A = 7

    def __init__(self):
        self.board = [[0] * 7 for _ in range(6)]  # board[row][col], row 0 bottom
        self.cur = X
        self.n = 0
        self.status = ONGOING

    def clone(self):
        s = C4.__new__(C4)
        s.board = [r[:] for r in self.board]
        s.cur, s.n, s.status = self.cur, self.n, self.status
        return s

    def winner(self, lr, lc):
        b = self.board
        row = b[lr]
        for i in range(0, 7 - 4 + 1):
            if row[i] and row[i] == row[i + 1] == row[i + 2] == row[i + 3]:
                return row[i]
        for i in range(0, 6 - 4 + 1):
            if b[i][lc] and b[i][lc] == b[i + 1][lc] == b[i + 2][lc] == b[i + 3][lc]:
                return b[i][lc]
        start = max(-4, -min(lc, lr))
        end = min(0, min(7 - (lc + 4), 6 - (lr + 4)))
        for i in range(start, end + 1):
            r, c = lr + i, lc + i
            if b[r][c] and b[r][c] == b[r + 1][c + 1] == b[r + 2][c + 2] == b[r + 3][c + 3]:
                return b[r][c]
        return 0

    def next_state(self, a):
        if self.status != ONGOING:
            raise ValueError("Game has already ended")
        r = next((i for i in range(6) if self.board[i][a] == 0), None)
        if r is None:
            raise ValueError("Illegal move: column already filled")
        s = self.clone()
        s.board[r][a] = self.cur
        s.cur = O if self.cur == X else X
        s.n += 1
        if s.winner(r, a):
            s.status = WON
        elif s.n == 42:
            s.status = TIED
        return s

    def valid(self):
        if self.status != ONGOING:
            return []
        return [c for c in range(7) if self.board[5][c] == 0]

    def value_term(self):
        return {WON: (-1.0, True), TIED: (0.0, True)}.get(self.status, (0.0, False))

    def encoding(self):
        e = np.zeros((3, 6, 7), np.float32)
        for r in range(6):
            for c in range(7):
                p = self.board[r][c]
                if p:
                    e[0 if p == self.cur else 1, r, c] = 1.0
                else:
                    e[2, r, c] = 1.0
        return e

    def mask(self, p):
        m = [0.0] * 7
        for a in self.valid():
            m[a] = 1.0
        mp = [fmul(p[i], m[i]) for i in range(7)]
        s = nd_sum(mp)
        return [fdiv(v, s) for v in mp]

    def bitboards(self):
        x = o = 0
        for r in range(6):
            for c in range(7):
                if self.board[r][c] == X:
                    x |= 1 << (c * 7 + r)
                elif self.board[r][c] == O:
                    o |= 1 << (c * 7 + r)
        return x, o


class TTT:
    A = 9

    def __init__(self):
        self.board = [[0] * 3 for _ in range(3)]
        self.cur = X
        self.n = 0
        self.status = ONGOING

    def clone(self):
        s = TTT.__new__(TTT)
        s.board = [r[:] for r in self.board]
        s.cur, s.n, s.status = self.cur, self.n, self.status
        return s

    def next_state(self, a):
        if self.status != ONGOING:
            raise ValueError("Game has already ended")
        r, c = divmod(a, 3)
        if self.board[r][c]:
            raise ValueError("Illegal move")
        s = self.clone()
        b = s.board
        b[r][c] = self.cur
        s.cur = O if self.cur == X else X
        s.n += 1
        roww = b[r][0] == b[r][1] == b[r][2]
        colw = b[0][c] == b[1][c] == b[2][c]
        d1 = r == c and b[0][0] == b[1][1] == b[2][2]
        d2 = ((r == 1 and c == 1) or abs(r - c) == 2) and b[0][2] == b[1][1] == b[2][0]
        if roww or colw or d1 or d2:
            s.status = WON
        elif s.n == 9:
            s.status = TIED
        return s

    def valid(self):
        if self.status != ONGOING:
            return []
        return [r * 3 + c for r in range(3) for c in range(3) if self.board[r][c] == 0]

    def value_term(self):
        return {WON: (-1.0, True), TIED: (0.0, True)}.get(self.status, (0.0, False))

    def encoding(self):
        e = np.zeros((3, 3, 3), np.float32)
        for r in range(3):
            for c in range(3):
                p = self.board[r][c]
                if p:
                    e[0 if p == self.cur else 1, r, c] = 1.0
                else:
                    e[2, r, c] = 1.0
        return e

    def mask(self, p):
        m = [0.0] * 9
        for a in self.valid():
            m[a] = 1.0
        mp = [fmul(p[i], m[i]) for i in range(9)]
        s = nd_sum(mp)
        return [fdiv(v, s) for v in mp]

    def bitboards(self):
        x = o = 0
        for r in range(3):
            for c in range(3):
                if self.board[r][c] == X:
                    x |= 1 << (r * 3 + c)
                elif self.board[r][c] == O:
                    o |= 1 << (r * 3 + c)
        return x, o


# ---------------------------------------------------------------- RNG + stub evaluator
def philox4x32(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def u01_f32(seed, game_id, move_no):
    """rand 0.8's UniformFloat<f32> draw: the top 23 bits of the first Philox word
    as a float in [1, 2), minus 1"""
    o = philox4x32((move_no & M32, move_no >> 32, game_id & M32, game_id >> 32), (seed & M32, seed >> 32))
    one_two = struct.unpack("<f", struct.pack("<I", (o[0] >> 9) | 0x3F800000))[0]
    return f32(one_two - 1.0)


_LIBM = ctypes.CDLL(ctypes.util.find_library("m"))
_LIBM.powf.restype = ctypes.c_float
_LIBM.powf.argtypes = [ctypes.c_float, ctypes.c_float]


def powf(x, y):
    """f32::powf (Rust calls the C library's powf)"""
    return float(_LIBM.powf(x, y))


def weighted_index(visits, temperature, u01):
    """WeightedIndex::<f32>::new(visits.powf(T)).sample (rand 0.8,
    learner_concurrent.rs:189-193): f32 running totals, Uniform::new(0, total)
    shrinking its scale one ulp at a time while scale * (1 - 2^-23) >= total,
    chosen = u01 * scale, index = #running totals <= chosen"""
    w = [f32(powf(f32(v), f32(temperature))) for v in visits]
    cum, total = [], w[0]
    for x in w[1:]:
        cum.append(total)
        total = f32(total + x)
    max_rand = f32(1.0 - 1.1920929e-7)
    scale = total
    while f32(scale * max_rand) >= total:
        scale = struct.unpack("<f", struct.pack("<I", struct.unpack("<I", struct.pack("<f", scale))[0] - 1))[0]
    chosen = f32(f32(u01 * scale) + 0.0)
    return sum(1 for c in cum if c <= chosen)


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def hash_eval(state):
    x, o = state.bitboards()
    h = splitmix64(x ^ ((o * 0x9E3779B97F4A7C15) & M64) ^ ((state.n << 58) & M64))
    A = state.A
    w = [float(1 + ((h >> (5 * a)) & 31)) for a in range(A)]
    s = 0.0
    for v in w:
        s = fadd(s, v)
    raw = [fdiv(v, s) for v in w]
    value = f32(float(((h >> 48) & 255) - 127) / 128.0)
    return state.mask(raw), value


# ---------------------------------------------------------------- MCTS (mcts.rs)
class Node:
    __slots__ = ("state", "parent", "action", "prior", "children", "N", "W")

    def __init__(self, state, parent=None, action=None, prior=None):
        self.state, self.parent, self.action, self.prior = state, parent, action, prior
        self.children, self.N, self.W = [], 0, 0.0


class Tree:
    def __init__(self, state):
        self.arena = [Node(state)]
        self.to_expand = None

    def ucb(self, pid, cid, c):
        p, ch = self.arena[pid], self.arena[cid]
        q = 0.0 if ch.N == 0 else fdiv(fadd(fdiv(-ch.W, f32(float(ch.N))), 1.0), 2.0)
        u = fmul(fmul(c, ch.prior), f32(math.sqrt(f32(float(p.N)))))
        u = fdiv(u, fadd(1.0, f32(float(ch.N))))
        return fadd(q, u)

    def select(self, pid, c):
        best, bu = None, None
        for cid in self.arena[pid].children:
            u = self.ucb(pid, cid, c)
            if best is None or not (u < bu):
                best, bu = cid, u
        return best

    def expand(self, pid, policy):
        st = self.arena[pid].state
        acts = st.valid()
        first = len(self.arena)
        self.arena[pid].children.extend(range(first, first + len(acts)))
        for a in acts:
            self.arena.append(Node(st.next_state(a), pid, a, policy[a]))

    def backprop(self, nid, v):
        sign = 1.0
        node = self.arena[nid]
        node.N += 1
        node.W = fadd(node.W, fmul(sign, v))
        sign = -sign
        while node.parent is not None:
            node = self.arena[node.parent]
            node.N += 1
            node.W = fadd(node.W, fmul(sign, v))
            sign = -sign

    def use_subtree(self, rid):
        old = self.arena
        new = []
        root = old[rid]
        q = [(root, None)]
        qi = 0
        while qi < len(q):
            node, parent = q[qi]
            qi += 1
            nid = len(new)
            copy = Node(node.state, parent, node.action, node.prior)
            copy.N, copy.W = node.N, node.W
            for ch in node.children:
                q.append((old[ch], nid))
            if parent is not None:
                new[parent].children.append(nid)
            new.append(copy)
        self.arena = new


def search(trees, num_searches, c=2.0):
    c = f32(c)
    for _ in range(num_searches):
        batch = []
        for t in trees:
            node = 0
            while t.arena[node].children:
                node = t.select(node, c)
            v, term = t.arena[node].state.value_term()
            if term:
                t.backprop(node, v)
                t.to_expand = None
            else:
                t.to_expand = node
                batch.append(t)
        for t in batch:
            pol, v = hash_eval(t.arena[t.to_expand].state)
            t.expand(t.to_expand, pol)
            t.backprop(t.to_expand, v)
    out = []
    for t in trees:
        root = t.arena[0]
        A = root.state.A
        pol = [0.0] * A
        kids = []
        for cid in root.children:
            ch = t.arena[cid]
            pol[ch.action] = float(ch.N)
            kids.append((cid, ch.action, ch.N))
        s = nd_sum(pol)
        out.append(([fdiv(v, s) for v in pol], kids))
    return out


def self_play(game_cls, n_games, num_searches, temperature=1.25, seed=7, c=2.0):
    trees = [Tree(game_cls()) for _ in range(n_games)]
    hist = [([], []) for _ in range(n_games)]
    active = list(range(n_games))
    samples = []
    moves = [[] for _ in range(n_games)]
    move_no = 0
    while active:
        res = search([trees[g] for g in active], num_searches, c)
        for k in range(len(active) - 1, -1, -1):
            g = active[k]
            t = trees[g]
            pol, kids = res[k]
            idx = weighted_index([n for (_, _, n) in kids], temperature, u01_f32(seed, g, move_no))
            sel = kids[idx][0]
            hist[g][0].append(t.arena[0].state)
            hist[g][1].append(pol)
            moves[g].append(t.arena[sel].action)
            st = t.arena[sel].state
            v, term = st.value_term()
            if term:
                for h, (hs, hp) in enumerate(zip(*hist[g])):
                    samples.append({"game": g, "ply": h, "policy": hp,
                                    "value": v if hs.cur == st.cur else -v,
                                    "enc_sum": float(hs.encoding().ravel() @ np.arange(hs.encoding().size))})
                active.pop(k)
            else:
                t.use_subtree(sel)
        move_no += 1
    return samples, moves


# ---------------------------------------------------------------- rules fixtures
def rules_traces(game_cls, n_games, seed):
    rng = random.Random(seed)
    games = []
    for _ in range(n_games):
        s = game_cls()
        plies = []
        while True:
            va = s.valid()
            mask = sum(1 << a for a in va)
            x, o = s.bitboards()
            v, term = s.value_term()
            enc = s.encoding()
            plies.append({"legal": mask, "status": s.status, "n": s.n, "cur": s.cur,
                          "x": str(x), "o": str(o), "value": v, "term": bool(term),
                          "enc_sum": float(enc.ravel() @ np.arange(enc.size))})
            if term:
                break
            s = s.next_state(rng.choice(va))
        games.append({"plies": plies})
    return games


def moves_of(game_cls, n_games, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n_games):
        s = game_cls()
        mv = []
        while s.status == ONGOING:
            a = rng.choice(s.valid())
            mv.append(a)
            s = s.next_state(a)
        out.append(mv)
    return out


def c4_kats():
    kats = []
    # anti-diagonal four stays Ongoing (quirk Q1)
    seq = [1, 3, 2, 6, 4, 1, 3, 1, 1, 2, 2]
    s = C4()
    for a in seq:
        s = s.next_state(a)
    kats.append({"name": "anti_diagonal_ignored", "moves": seq, "status": s.status, "n": s.n})
    for name, seq in [("horizontal", [0, 0, 1, 1, 2, 2, 3]), ("vertical", [0, 1, 0, 1, 0, 1, 0]),
                      ("diagonal", [0, 1, 1, 2, 2, 3, 2, 3, 3, 6, 3])]:
        s = C4()
        for a in seq:
            s = s.next_state(a)
        kats.append({"name": name, "moves": seq, "status": s.status, "n": s.n})
    # full column -> Err
    s = C4()
    for _ in range(6):
        s = s.next_state(0)
    kats.append({"name": "full_column_error", "moves": [0] * 6, "illegal": 0, "legal": sum(1 << a for a in s.valid())})
    return kats


# ---------------------------------------------------------------- nets
def philox_params(game, blocks, hidden, seed):
    """Mirror of or_net_init_params (tch 0.13 default inits, Philox stream)."""
    C, H, W, A = (3, 6, 7, 7) if game == "c4" else (3, 3, 3, 9)
    parts = []
    t = [0]
    key = (seed & M32, seed >> 32)

    def unit(i):
        o = philox4x32((i & M32, i >> 32, t[0], 0x5EED), key)
        return np.float32(o[0] >> 8) * np.float32(1.0 / 16777216.0)

    def uni(n, lo, hi):
        lo, hi = np.float32(lo), np.float32(hi)
        u = np.array([unit(i) for i in range(n)], np.float32)
        t[0] += 1
        return (lo + (hi - lo) * u).astype(np.float32)

    def const(n, v):
        t[0] += 1
        return np.full(n, v, np.float32)

    def conv(ci, co):
        b = np.float32(math.sqrt(6.0 / (ci * 9)))
        return [uni(co * ci * 9, -b, b), const(co, 0.0)]

    def bn(c):
        return [uni(c, 0.0, 1.0), const(c, 0.0), const(c, 0.0), const(c, 1.0)]

    def lin(i, o):
        b = np.float32(math.sqrt(6.0 / i))
        bb = np.float32(1.0 / math.sqrt(i))
        return [uni(o * i, -b, b), uni(o, -bb, bb)]

    parts += conv(C, hidden) + bn(hidden)
    for _ in range(blocks):
        parts += conv(hidden, hidden) + bn(hidden) + conv(hidden, hidden) + bn(hidden)
    parts += conv(hidden, 32) + bn(32) + lin(32 * H * W, A)
    parts += conv(hidden, 3) + bn(3) + lin(3 * H * W, 1)
    return np.concatenate(parts), (C, H, W, A)


def torch_forward(params, dims, blocks, hidden, x):
    import torch
    import torch.nn.functional as F
    C, H, W, A = dims
    p = torch.from_numpy(params)
    off = [0]

    def take(*shape):
        n = int(np.prod(shape))
        v = p[off[0]:off[0] + n].reshape(shape)
        off[0] += n
        return v

    def conv_bn(t, ci, co, relu):
        w, b = take(co, ci, 3, 3), take(co)
        g, be, mu, var = take(co), take(co), take(co), take(co)
        t = F.conv2d(t, w, b, padding=1)
        t = F.batch_norm(t, mu, var, g, be, training=False, eps=1e-5)
        return F.relu(t) if relu else t

    with torch.no_grad():
        t = torch.from_numpy(x).view(-1, C, H, W)
        t = conv_bn(t, C, hidden, True)
        for _ in range(blocks):
            y = conv_bn(t, hidden, hidden, True)
            y = conv_bn(y, hidden, hidden, False)
            t = F.relu(t + y)
        pp = conv_bn(t, hidden, 32, True).flatten(1)
        lw, lb = take(A, 32 * H * W), take(A)
        logits = F.linear(pp, lw, lb)
        vv = conv_bn(t, hidden, 3, True).flatten(1)
        vw, vb = take(1, 3 * H * W), take(1)
        value = torch.tanh(F.linear(vv, vw, vb))
        assert off[0] == p.numel()
        sm = torch.softmax(logits, -1)
    return logits.numpy(), value.numpy().reshape(-1), sm.numpy()


def net_golden(game, blocks, hidden, seed, n_pos, pos_seed):
    params, dims = philox_params(game, blocks, hidden, seed)
    cls = C4 if game == "c4" else TTT
    rng = random.Random(pos_seed)
    states = []
    while len(states) < n_pos:
        s = cls()
        while s.status == ONGOING and len(states) < n_pos:
            states.append(s)
            s = s.next_state(rng.choice(s.valid()))
    x = np.stack([s.encoding() for s in states]).astype(np.float32)
    logits, value, sm = torch_forward(params, dims, blocks, hidden, x)
    priors = np.stack([np.array(s.mask([float(v) for v in sm[i]]), np.float32) for i, s in enumerate(states)])
    bb = np.array([[*s.bitboards(), s.n] for s in states], np.uint64)
    return dict(params=params, x=x, logits=logits, value=value, softmax=sm, priors=priors,
                boards=bb, meta=np.array([blocks, hidden, seed], np.int64))


def learner_golden(blocks=1, hidden=64, seed=0, B=32, K=3, data_seed=21):
    """ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85) in PyTorch CPU
    fp32: train-mode forward (BN batch stats, running stats momentum 0.1),
    -(log_softmax(p)*pi).sum()/B + mse(v, z), backward, torch.optim.Adam(lr=1e-3)
    (tch Adam::default(): betas 0.9/0.999, eps 1e-8, no weight decay)."""
    import torch
    import torch.nn.functional as F
    params, dims = philox_params("c4", blocks, hidden, seed)
    C, H, W, A = dims
    # flat construction order -> tensors; running stats are buffers (no grad)
    flat = torch.from_numpy(params.copy())
    tensors, trainable, off = [], [], [0]

    def take(shape, train=True):
        n = int(np.prod(shape))
        t = flat[off[0]:off[0] + n].clone().reshape(shape)
        if train:
            t.requires_grad_(True)
            trainable.append(t)
        tensors.append(t)
        off[0] += n
        return t

    def conv(ci, co):
        return dict(w=take((co, ci, 3, 3)), b=take((co,)), g=take((co,)), be=take((co,)),
                    mu=take((co,), False), var=take((co,), False))

    stem = conv(C, hidden)
    res = [(conv(hidden, hidden), conv(hidden, hidden)) for _ in range(blocks)]
    pconv = conv(hidden, 32)
    plw, plb = take((A, 32 * H * W)), take((A,))
    vconv = conv(hidden, 3)
    vlw, vlb = take((1, 3 * H * W)), take((1,))
    assert off[0] == len(params)

    def cbn(t, c, relu=True):
        t = F.conv2d(t, c["w"], c["b"], padding=1)
        t = F.batch_norm(t, c["mu"], c["var"], c["g"], c["be"], training=True, momentum=0.1, eps=1e-5)
        return F.relu(t) if relu else t

    def forward(x):
        t = cbn(x.view(-1, C, H, W), stem)
        for c1, c2 in res:
            t = F.relu(t + cbn(cbn(t, c1), c2, relu=False))
        logits = F.linear(cbn(t, pconv).flatten(1), plw, plb)
        value = torch.tanh(F.linear(cbn(t, vconv).flatten(1), vlw, vlb))
        return logits, value

    opt = torch.optim.Adam(trainable, lr=1e-3, foreach=False)
    rng = random.Random(data_seed)
    nprng = np.random.default_rng(data_seed)
    xs, pis, zs = [], [], []
    for _ in range(K):
        st = []
        while len(st) < B:
            g = C4()
            for _ in range(rng.randrange(0, 30)):
                if g.status != ONGOING:
                    break
                g = g.next_state(rng.choice(g.valid()))
            if g.status == ONGOING:
                st.append(g)
        xs.append(np.stack([g.encoding() for g in st]).astype(np.float32))
        pi = nprng.random((B, A)).astype(np.float32) ** 3
        pis.append((pi / pi.sum(1, keepdims=True)).astype(np.float32))
        zs.append(nprng.choice(np.array([-1.0, 0.0, 1.0], np.float32), B))
    losses, grads1, params1 = [], None, None

    def flat_now(use_grad):
        out = []
        for t in tensors:
            if use_grad:
                out.append((t.grad if t.grad is not None else torch.zeros_like(t)).detach().reshape(-1))
            else:
                out.append(t.detach().reshape(-1))
        return torch.cat(out).numpy().astype(np.float32)

    for k in range(K):
        x, pi, z = torch.from_numpy(xs[k]), torch.from_numpy(pis[k]), torch.from_numpy(zs[k]).view(-1, 1)
        opt.zero_grad()
        logits, value = forward(x)
        lp = -(logits.log_softmax(-1) * pi).sum() / logits.shape[0]
        lv = F.mse_loss(value, z)
        loss = lp + lv
        loss.backward()
        if k == 0:
            grads1 = flat_now(True)
        opt.step()
        losses.append([loss.item(), lp.item(), lv.item()])
        if k == 0:
            params1 = flat_now(False)
    return dict(states=np.stack(xs), policies=np.stack(pis), values=np.stack(zs), loss=np.array(losses, np.float32),
                grads1=grads1, params1=params1, params3=flat_now(False),
                meta=np.array([blocks, hidden, seed, B, K], np.int64))


def main():
    rules = {"traces": rules_traces(C4, 200, 1), "kats": c4_kats(), "games": moves_of(C4, 50, 2)}
    with open(os.path.join(HERE, "rules_c4.json"), "w") as f:
        json.dump(rules, f, separators=(",", ":"))
    with open(os.path.join(HERE, "rules_ttt.json"), "w") as f:
        json.dump({"traces": rules_traces(TTT, 300, 3)}, f, separators=(",", ":"))
    mcts_main()
    np.savez_compressed(os.path.join(HERE, "net_c4_2x64.npz"), **net_golden("c4", 2, 64, 1234, 256, 5))
    np.savez_compressed(os.path.join(HERE, "net_ttt_2x64.npz"), **net_golden("ttt", 2, 64, 99, 64, 6))
    learner_main()


def mcts_main():
    mcts = {"search": [], "selfplay": {}}
    rng = random.Random(11)
    for case in range(12):
        s = C4()
        for _ in range(rng.randrange(0, 12)):
            if s.status != ONGOING:
                break
            s = s.next_state(rng.choice(s.valid()))
        if s.status != ONGOING:
            continue
        sims = [1, 2, 7, 16, 64, 200][case % 6]
        (pol, kids), = search([Tree(s)], sims)
        x, o = s.bitboards()
        mcts["search"].append({"x": str(x), "o": str(o), "n": s.n, "cur": s.cur, "sims": sims,
                               "policy": pol, "visits": [n for (_, _, n) in kids],
                               "actions": [a for (_, a, _) in kids]})
    # uniform-prior KAT: first selection after the root expands goes to column 6
    t = Tree(C4())
    t.expand(0, [1.0 / 7] * 7)
    t.backprop(0, 0.0)
    mcts["uniform_first_select"] = t.arena[t.select(0, f32(2.0))].action
    samples, moves = self_play(C4, 6, 24, seed=7)
    mcts["selfplay"]["c4"] = {"n_games": 6, "sims": 24, "seed": 7, "samples": samples, "moves": moves}
    samples, moves = self_play(TTT, 4, 32, seed=9)
    mcts["selfplay"]["ttt"] = {"n_games": 4, "sims": 32, "seed": 9, "samples": samples, "moves": moves}
    with open(os.path.join(HERE, "mcts_hash.json"), "w") as f:
        json.dump(mcts, f, separators=(",", ":"))


def learner_main():
    np.savez_compressed(os.path.join(HERE, "learner_c4_1x64.npz"), **learner_golden())


if __name__ == "__main__":
    # `gen_golden.py learner` regenerates only the training fixture
    if len(sys.argv) > 1 and sys.argv[1] == "learner":
        learner_main()
    elif len(sys.argv) > 1 and sys.argv[1] == "mcts":   # `gen_golden.py mcts`: only mcts_hash.json
        mcts_main()
    else:
        main()

"""ctypes binding of the chess oracle (oracle/chess_oracle.c) + a numpy
restatement of the chess ResNet (model/chess.rs:48-77, model/mod.rs:152-184).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker; never by the product path.
"""
import ctypes as C

import numpy as np

import oracle as _o

POLICY, ENC, MAX_MOVES = 4672, 1216, 256
PAWN, KNIGHT, BISHOP, ROOK, QUEEN, KING = range(6)
WHITE, BLACK = 0, 1
NO_EP = 64
START_FEN = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


class Board(C.Structure):
    _fields_ = [("pieces", C.c_uint64 * 6), ("color", C.c_uint64 * 2), ("side", C.c_uint8),
                ("castle", C.c_uint8 * 2), ("ep", C.c_uint8)]


class State(C.Structure):
    _fields_ = [("b", Board), ("made", C.c_uint32), ("fifty", C.c_uint32), ("n_tt", C.c_uint32),
                ("tt", C.c_void_p)]


EVAL_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.POINTER(C.POINTER(State)), C.POINTER(C.c_float),
                      C.POINTER(C.c_float))

_ready = False


def lib():
    global _ready
    L = _o.lib()
    if not _ready:
        vp, i, u64, f = C.c_void_p, C.c_int, C.c_uint64, C.c_float
        fp, ip, i32p = C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_int32)
        u16p = C.POINTER(C.c_uint16)
        L.orc_board_start.argtypes = [vp]
        L.orc_board_from_fen.argtypes = [C.c_char_p, vp]
        L.orc_legal_moves.argtypes = [vp, u16p]
        L.orc_in_check.argtypes = [vp]
        L.orc_board_make_move.argtypes = [vp, i, vp]
        L.orc_perft.restype = u64
        L.orc_perft.argtypes = [vp, i]
        L.orc_state_init.argtypes = [vp]
        L.orc_state_from_board.argtypes = [vp, vp, C.c_uint32, C.c_uint32]
        L.orc_next_state.argtypes = [vp, i, vp]
        L.orc_status.argtypes = [vp]
        L.orc_num_repetitions.argtypes = [vp]
        L.orc_value_terminated.argtypes = [vp, fp, ip]
        L.orc_encoding.argtypes = [vp, fp]
        L.orc_mask_invalid.argtypes = [vp, fp, i, fp]
        L.orc_get_channel.argtypes = [i, i]
        L.orc_policy_index.argtypes = [i, i]
        L.orc_get_action.argtypes = [i, i]
        L.orc_position_key.restype = u64
        L.orc_position_key.argtypes = [vp]
        L.orc_hash_eval_raw.argtypes = [vp, fp, fp]
        L.orc_tree_create.restype = vp
        L.orc_tree_with_root.restype = vp
        L.orc_tree_with_root.argtypes = [C.POINTER(State)]
        L.orc_tree_destroy.argtypes = [vp]
        L.orc_tree_use_subtree.argtypes = [vp, i]
        L.orc_tree_node_state.restype = C.POINTER(State)
        L.orc_tree_node_state.argtypes = [vp, i]
        L.orc_tree_size.argtypes = [vp]
        L.orc_search.argtypes = [C.POINTER(vp), i, i, f, EVAL_FN, vp, fp, ip, fp, ip, ip]
        L.orc_self_play.restype = C.c_long
        L.orc_self_play.argtypes = [i, i, f, f, u64, u64, EVAL_FN, vp, C.c_long, fp, fp, fp, i32p, i32p, i,
                                    i32p, i32p, C.POINTER(C.c_double)]
        _ready = True
    return L


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def move(src, dst, promo=0):
    return src | (dst << 6) | (promo << 12)


def sq(name):
    return (ord(name[1]) - ord("1")) * 8 + ord(name[0]) - ord("a")


def uci(m):
    s, d, p = m & 63, (m >> 6) & 63, (m >> 12) & 7
    n = "abcdefgh"[s & 7] + str(s // 8 + 1) + "abcdefgh"[d & 7] + str(d // 8 + 1)
    return n + ("", "n", "b", "r", "q")[p] if p else n


def board_from_fen(fen):
    b = Board()
    if lib().orc_board_from_fen(fen.encode(), C.byref(b)) != 0:
        raise ValueError(fen)
    return b


def legal_moves(b):
    out = (C.c_uint16 * MAX_MOVES)()
    n = lib().orc_legal_moves(C.byref(b), out)
    return [int(out[i]) for i in range(n)]


def perft(b, depth):
    return int(lib().orc_perft(C.byref(b), depth))


def make_move(b, m):
    out = Board()
    lib().orc_board_make_move(C.byref(b), int(m), C.byref(out))
    return out


class ChessState:
    """game/chess.rs State backed by the oracle (transposition table kept in C)."""

    def __init__(self, st=None, fen=None, made=0, fifty=0):
        if st is not None:
            self.st = st
        else:
            self.st = State()
            if fen is None:
                lib().orc_state_init(C.byref(self.st))
            else:
                b = board_from_fen(fen)
                lib().orc_state_from_board(C.byref(self.st), C.byref(b), made, fifty)

    def next_state(self, m):
        out = State()
        rc = lib().orc_next_state(C.byref(self.st), int(m), C.byref(out))
        if rc != 0:
            raise ValueError(f"next_state({uci(m)}) rc={rc}")
        return ChessState(out)

    def valid_actions(self):
        return legal_moves(self.st.b)

    @property
    def side(self):
        return int(self.st.b.side)

    @property
    def status(self):
        return int(lib().orc_status(C.byref(self.st)))

    def repetitions(self):
        return int(lib().orc_num_repetitions(C.byref(self.st)))

    def value_terminated(self):
        v, t = C.c_float(), C.c_int()
        lib().orc_value_terminated(C.byref(self.st), C.byref(v), C.byref(t))
        return v.value, bool(t.value)

    def encoding(self):
        e = np.zeros((19, 8, 8), np.float32)
        lib().orc_encoding(C.byref(self.st), _f(e))
        return e

    def mask_invalid(self, p):
        p = np.ascontiguousarray(p, np.float32)
        out = np.zeros(POLICY, np.float32)
        if lib().orc_mask_invalid(C.byref(self.st), _f(p), p.size, _f(out)) != 0:
            raise ValueError("policy shape")
        return out

    def hash_eval_raw(self):
        raw = np.zeros(POLICY, np.float32)
        v = C.c_float()
        lib().orc_hash_eval_raw(C.byref(self.st), _f(raw), C.byref(v))
        return raw, v.value


def policy_index(side, m):
    return int(lib().orc_policy_index(side, int(m)))


def get_channel(side, m):
    return int(lib().orc_get_channel(side, int(m)))


def get_action(side, index):
    return int(lib().orc_get_action(side, int(index)))


def arena_reset():
    lib().orc_arena_reset()


def search(n_trees, num_searches, c=2.0, states=None):
    """Mcts::search with the hash stub over n fresh trees from the start position,
    or (states = list of ChessState) over Tree::with_root_state(state) trees."""
    L = lib()
    if states is not None:
        n_trees = len(states)
        trees = [L.orc_tree_with_root(C.byref(st.st)) for st in states]
    else:
        trees = [L.orc_tree_create() for _ in range(n_trees)]
    arr = (C.c_void_p * n_trees)(*trees)
    pol = np.zeros((n_trees, POLICY), np.float32)
    ids = np.zeros((n_trees, MAX_MOVES), np.int32)
    vis = np.zeros((n_trees, MAX_MOVES), np.float32)
    mv = np.zeros((n_trees, MAX_MOVES), np.int32)
    nc = np.zeros(n_trees, np.int32)
    rc = L.orc_search(arr, n_trees, num_searches, c, EVAL_FN(), None, _f(pol), ids.ctypes.data_as(C.POINTER(C.c_int)),
                      _f(vis), mv.ctypes.data_as(C.POINTER(C.c_int)), nc.ctypes.data_as(C.POINTER(C.c_int)))
    for t in trees:
        L.orc_tree_destroy(t)
    return rc, pol, ids, vis, mv, nc


def self_play(n_games, num_searches, seed, c=2.0, temperature=1.25, game_id_base=0, max_plies=1024,
              with_policy=True, cap=None):
    L = lib()
    cap = cap if cap is not None else n_games * max_plies
    enc = np.zeros((cap, ENC), np.float32)
    pol = np.zeros((cap, POLICY), np.float32) if with_policy else None
    val = np.zeros(cap, np.float32)
    gid = np.zeros(cap, np.int32)
    ply = np.zeros(cap, np.int32)
    moves = np.full((n_games, max_plies), -1, np.int32)
    nmv = np.zeros(n_games, np.int32)
    stats = np.zeros(2, np.float64)
    i32 = C.POINTER(C.c_int32)
    n = L.orc_self_play(n_games, num_searches, c, temperature, seed, game_id_base, EVAL_FN(), None, cap, _f(enc),
                        _f(pol) if pol is not None else None, _f(val), gid.ctypes.data_as(i32),
                        ply.ctypes.data_as(i32), max_plies, moves.ctypes.data_as(i32), nmv.ctypes.data_as(i32),
                        stats.ctypes.data_as(C.POINTER(C.c_double)))
    if n < 0:
        raise RuntimeError(f"orc_self_play rc={n}")
    n = min(n, cap)
    return dict(enc=enc[:n], policy=pol[:n] if pol is not None else None, value=val[:n], game=gid[:n],
                ply=ply[:n], moves=moves, n_moves=nmv, sims=stats[0], evals=stats[1])


# ---------------------------------------------------------------- net (numpy, fp64 accumulate)
def net_param_shapes(blocks, hidden=256):
    """tch construction order of model/chess.rs:48-70 (torso, policy head, value head)."""
    s = [("conv", (hidden, 19, 3, 3)), ("bias", (hidden,)), ("bn", hidden)]
    for _ in range(blocks):
        s += [("conv", (hidden, hidden, 3, 3)), ("bias", (hidden,)), ("bn", hidden)] * 2
    s += [("conv", (256, hidden, 1, 1)), ("bias", (256,)), ("conv", (73, 256, 1, 1)), ("bias", (73,))]
    s += [("conv", (1, hidden, 1, 1)), ("bias", (1,)), ("lin", (256, 64)), ("bias", (256,)),
          ("lin", (1, 256)), ("bias", (1,))]
    return s


def unpack_params(params, blocks, hidden=256):
    out, off = [], 0
    for kind, shp in net_param_shapes(blocks, hidden):
        if kind == "bn":
            c = shp
            g, b, m, v = (params[off + k * c: off + (k + 1) * c] for k in range(4))
            out.append(("bn", (g, b, m, v)))
            off += 4 * c
        else:
            n = int(np.prod(shp))
            out.append((kind, params[off:off + n].reshape(shp)))
            off += n
    assert off == params.size, (off, params.size)
    return out


def _conv(x, w, b):
    """x [B][C][8][8], w [O][C][k][k] (pad k//2) -> [B][O][8][8] in float64"""
    B, Ci = x.shape[:2]
    k = w.shape[2]
    p = k // 2
    xp = np.zeros((B, Ci, 8 + 2 * p, 8 + 2 * p))
    xp[:, :, p:p + 8, p:p + 8] = x
    cols = np.stack([xp[:, :, dy:dy + 8, dx:dx + 8] for dy in range(k) for dx in range(k)], 2)  # B,C,k*k,8,8
    cols = cols.reshape(B, Ci * k * k, 64)
    return (np.matmul(w.reshape(w.shape[0], -1).astype(np.float64)[None], cols) +
            b.astype(np.float64)[None, :, None]).reshape(B, -1, 8, 8)


def _bn(x, g, b, m, v, eps=1e-5):
    s = (g.astype(np.float64) / np.sqrt(v.astype(np.float64) + eps))
    return (x - m[None, :, None, None]) * s[None, :, None, None] + b[None, :, None, None]


def net_forward(params, blocks, x, hidden=256):
    """Net::forward(x, train=false) for the chess net; x [B][19][8][8] -> logits [B][4672], value [B]"""
    P = unpack_params(np.asarray(params, np.float32), blocks, hidden)
    x = np.asarray(x, np.float64).reshape(-1, 19, 8, 8)
    it = iter(P)

    def nxt():
        return next(it)[1]

    h = np.maximum(_bn(_conv(x, nxt(), nxt()), *nxt()), 0)
    for _ in range(blocks):
        y = np.maximum(_bn(_conv(h, nxt(), nxt()), *nxt()), 0)
        y = _bn(_conv(y, nxt(), nxt()), *nxt())
        h = np.maximum(h + y, 0)
    p = np.maximum(_conv(h, nxt(), nxt()), 0)
    p = _conv(p, nxt(), nxt()).reshape(-1, 73 * 64)
    v = np.maximum(_conv(h, nxt(), nxt()), 0).reshape(-1, 64)
    w1, b1, w2, b2 = nxt(), nxt(), nxt(), nxt()
    v = np.maximum(v @ w1.T.astype(np.float64) + b1, 0)
    v = np.tanh(v @ w2.T.astype(np.float64) + b2)[:, 0]
    return p, v

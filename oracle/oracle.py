"""ctypes binding of the CPU oracle (oracle/spai_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker (or the timed CPU
baseline), never by the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libspai_oracle.so")

GAME_TICTACTOE, GAME_CONNECT4 = 0, 1
EVAL_NET, EVAL_UNIFORM, EVAL_HASH = 0, 1, 2
ONGOING, TIED, WON = 0, 1, 2
X, O = 1, 2


class C4State(C.Structure):
    _fields_ = [("board", (C.c_int8 * 7) * 6), ("current_player", C.c_uint8),
                ("num_actions_played", C.c_uint8), ("status", C.c_uint8)]


class TTTState(C.Structure):
    _fields_ = [("board", (C.c_int8 * 3) * 3), ("current_player", C.c_uint8),
                ("num_actions_played", C.c_uint8), ("status", C.c_uint8)]


EVAL_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_float),
                      C.POINTER(C.c_float))

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, i, u64, f, d = C.c_void_p, C.c_int, C.c_uint64, C.c_float, C.c_double
        fp = C.POINTER(C.c_float)
        ip = C.POINTER(C.c_int)
        i32p = C.POINTER(C.c_int32)
        L.or_nd_sum.restype = f
        L.or_nd_sum.argtypes = [fp, i]
        L.or_c4_init.argtypes = [vp]
        L.or_c4_next_state.argtypes = [vp, i, vp]
        L.or_c4_valid_actions.argtypes = [vp, ip]
        L.or_c4_encoding.argtypes = [vp, fp]
        L.or_c4_mask_invalid.argtypes = [vp, fp, i, fp]
        L.or_c4_bitboards.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
        L.or_c4_replay.restype = C.c_long
        L.or_c4_replay.argtypes = [i, i, i32p, vp, vp, vp, vp, i32p]
        L.or_encode_states.argtypes = [i, i, C.POINTER(vp), fp]
        L.or_ttt_init.argtypes = [vp]
        L.or_ttt_next_state.argtypes = [vp, i, vp]
        L.or_u01_f32.restype = f
        L.or_u01_f32.argtypes = [u64, u64, u64]
        L.or_weighted_index.argtypes = [fp, i, f, f]
        L.or_policy_best_action.argtypes = [fp, i]
        L.or_policy_sample.argtypes = [fp, i, f, f]
        L.or_splitmix64.restype = u64
        L.or_splitmix64.argtypes = [u64]
        L.or_hash_eval_raw.argtypes = [u64, u64, i, i, fp, fp]
        L.or_net_num_params.restype = C.c_size_t
        L.or_net_num_params.argtypes = [i, i, i]
        L.or_net_create.restype = vp
        L.or_net_create.argtypes = [i, i, i, fp, C.c_size_t]
        L.or_net_destroy.argtypes = [vp]
        L.or_net_forward.argtypes = [vp, i, fp, fp, fp]
        L.or_net_init_params.argtypes = [i, i, i, u64, fp]
        L.or_predict.argtypes = [vp, i, C.POINTER(vp), fp, fp]
        L.or_tree_create.restype = vp
        L.or_tree_create.argtypes = [i]
        L.or_tree_with_root.restype = vp
        L.or_tree_with_root.argtypes = [i, vp]
        L.or_tree_destroy.argtypes = [vp]
        L.or_tree_size.argtypes = [vp]
        L.or_tree_use_subtree.argtypes = [vp, i]
        L.or_tree_node_state.restype = vp
        L.or_tree_node_state.argtypes = [vp, i]
        L.or_tree_node_info.argtypes = [vp, i, ip, ip, fp, C.POINTER(C.c_uint32), fp, ip, ip]
        L.or_search.argtypes = [C.POINTER(vp), i, i, f, i, vp, EVAL_FN, vp, fp, ip, fp, ip]
        L.or_self_play.restype = C.c_long
        L.or_self_play.argtypes = [i, i, i, f, f, u64, u64, i, vp, EVAL_FN, vp, C.c_long, fp, fp, fp,
                                   i32p, i32p, i, i32p, i32p, C.POINTER(d)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def _i32(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


GAME_DIMS = {GAME_CONNECT4: (3, 6, 7, 7), GAME_TICTACTOE: (3, 3, 3, 9)}


# ---------------------------------------------------------------- rules
class C4:
    """Connect4 State (game/connect_four.rs) backed by the oracle."""

    def __init__(self, st=None):
        self.st = st if st is not None else C4State()
        if st is None:
            lib().or_c4_init(C.byref(self.st))

    def next_state(self, a):
        out = C4State()
        rc = lib().or_c4_next_state(C.byref(self.st), int(a), C.byref(out))
        if rc != 0:
            raise ValueError(f"illegal move {a} (rc={rc})")
        return C4(out)

    def valid_actions(self):
        acts = np.zeros(7, np.int32)
        n = lib().or_c4_valid_actions(C.byref(self.st), _i(acts))
        return [int(a) for a in acts[:n]]

    def legal_mask(self):
        return sum(1 << a for a in self.valid_actions())

    @property
    def status(self):
        return self.st.status

    @property
    def current_player(self):
        return self.st.current_player

    @property
    def n(self):
        return self.st.num_actions_played

    def value_terminated(self):
        return {WON: (-1.0, True), TIED: (0.0, True)}.get(self.status, (0.0, False))

    def encoding(self):
        e = np.zeros((3, 6, 7), np.float32)
        lib().or_c4_encoding(C.byref(self.st), _f(e))
        return e

    def mask_invalid(self, p):
        p = np.ascontiguousarray(p, np.float32)
        out = np.zeros(7, np.float32)
        if lib().or_c4_mask_invalid(C.byref(self.st), _f(p), len(p), _f(out)) != 0:
            raise ValueError("policy shape")
        return out

    def bitboards(self):
        x, o = C.c_uint64(), C.c_uint64()
        lib().or_c4_bitboards(C.byref(self.st), C.byref(x), C.byref(o))
        return x.value, o.value


class TTT:
    def __init__(self, st=None):
        self.st = st if st is not None else TTTState()
        if st is None:
            lib().or_ttt_init(C.byref(self.st))

    def next_state(self, a):
        out = TTTState()
        if lib().or_ttt_next_state(C.byref(self.st), int(a), C.byref(out)) != 0:
            raise ValueError("illegal")
        return TTT(out)

    @property
    def status(self):
        return self.st.status


def c4_replay(actions):
    """actions [n][P] int32 (-1 = stop) -> dict of per-ply arrays [n][P+1]"""
    a = np.ascontiguousarray(actions, np.int32)
    n, P = a.shape
    legal = np.zeros((n, P + 1), np.uint32)
    status = np.zeros((n, P + 1), np.uint8)
    xs = np.zeros((n, P + 1), np.uint64)
    os_ = np.zeros((n, P + 1), np.uint64)
    rc = np.zeros((n, P + 1), np.int32)
    lib().or_c4_replay(n, P, _i32(a), legal.ctypes.data, status.ctypes.data, xs.ctypes.data, os_.ctypes.data,
                       _i32(rc))
    return dict(legal=legal, status=status, x=xs, o=os_, rc=rc)


# ---------------------------------------------------------------- net
def num_params(game, blocks, hidden):
    return lib().or_net_num_params(game, blocks, hidden)


def init_params(game, blocks, hidden, seed):
    p = np.zeros(num_params(game, blocks, hidden), np.float32)
    lib().or_net_init_params(game, blocks, hidden, seed, _f(p))
    return p


class Net:
    def __init__(self, game, blocks, hidden, params):
        params = np.ascontiguousarray(params, np.float32)
        self.game, self.blocks, self.hidden = game, blocks, hidden
        self.h = lib().or_net_create(game, blocks, hidden, _f(params), params.size)
        if not self.h:
            raise ValueError("bad net params")

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_net_destroy(self.h)
            self.h = None

    def forward(self, x):
        C_, H, W, A = GAME_DIMS[self.game]
        x = np.ascontiguousarray(x, np.float32).reshape(-1, C_ * H * W)
        n = x.shape[0]
        lg = np.zeros((n, A), np.float32)
        v = np.zeros(n, np.float32)
        lib().or_net_forward(self.h, n, _f(x), _f(lg), _f(v))
        return lg, v


# ---------------------------------------------------------------- search / self-play
def search_c4(states, num_searches, eval_kind=EVAL_HASH, net=None, c=2.0, trees=None):
    """Run Mcts::search over fresh trees rooted at `states` (or given tree handles)."""
    L = lib()
    own = trees is None
    if own:
        trees = [L.or_tree_with_root(GAME_CONNECT4, C.byref(s.st)) for s in states]
    n = len(trees)
    arr = (C.c_void_p * n)(*trees)
    pol = np.zeros((n, 7), np.float32)
    ids = np.zeros((n, 7), np.int32)
    vis = np.zeros((n, 7), np.float32)
    nc = np.zeros(n, np.int32)
    rc = L.or_search(arr, n, num_searches, c, eval_kind, net.h if net else None, EVAL_FN(), None,
                     _f(pol), _i(ids), _f(vis), _i(nc))
    if own:
        for t in trees:
            L.or_tree_destroy(t)
    return rc, pol, ids, vis, nc


def self_play(game, n_games, num_searches, seed, eval_kind=EVAL_HASH, net=None, c=2.0, temperature=1.25,
              game_id_base=0, cap=None, max_plies=64, eval_fn=None):
    L = lib()
    C_, H, W, A = GAME_DIMS[game]
    cap = cap if cap is not None else n_games * max_plies
    enc = np.zeros((cap, C_ * H * W), np.float32)
    pol = np.zeros((cap, A), np.float32)
    val = np.zeros(cap, np.float32)
    gid = np.zeros(cap, np.int32)
    ply = np.zeros(cap, np.int32)
    moves = np.full((n_games, max_plies), -1, np.int32)
    nmv = np.zeros(n_games, np.int32)
    stats = np.zeros(2, np.float64)
    cb = EVAL_FN(eval_fn) if eval_fn is not None else EVAL_FN()
    n = L.or_self_play(game, n_games, num_searches, c, temperature, seed, game_id_base, eval_kind,
                       net.h if net else None, cb, None, cap, _f(enc), _f(pol), _f(val), _i32(gid), _i32(ply),
                       max_plies, _i32(moves), _i32(nmv), stats.ctypes.data_as(C.POINTER(C.c_double)))
    if n < 0:
        raise RuntimeError(f"or_self_play failed rc={n}")
    n = min(n, cap)
    return dict(enc=enc[:n], policy=pol[:n], value=val[:n], game=gid[:n], ply=ply[:n], moves=moves,
                n_moves=nmv, sims=stats[0], evals=stats[1])

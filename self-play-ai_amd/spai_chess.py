"""ctypes binding of the chess section of libspai.so (include/spai.h).

Mirrors the reference's chess surface (joshua16266261/self-play-ai):
  State (game/chess.rs)            -> ChessEngine.games_* / legal_moves / apply / status / encode / mask_invalid
  Policy::get_channel / get_action -> move_index / index_move
  Net (model/chess.rs)             -> ChessNet.forward
  Tree + Mcts::search (mcts.rs)    -> ChessEngine.trees_create / search / use_subtree
  SelfPlayWorker::self_play        -> ChessEngine.self_play
Every call goes through the HIP library; there is no CPU fallback.
"""
import ctypes as C

import numpy as np

import spai
from spai import EVAL_HASH, EVAL_NET, EVAL_UNIFORM, Config, SelfPlayStats, SpaiError  # noqa: F401

POLICY, ENC, MAX_MOVES = 4672, 1216, 256

STATE_DTYPE = np.dtype([("pieces", "<u8", 6), ("colors", "<u8", 2), ("side", "u1"), ("castle", "u1"),
                        ("ep", "u1"), ("status", "u1"), ("fifty", "<u2"), ("made", "<u2"), ("reps", "<u4"),
                        ("pad", "<u4")])
assert STATE_DTYPE.itemsize == 80

SINK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                   C.POINTER(C.c_float), C.POINTER(C.c_uint16))

_ready = False


def lib():
    global _ready
    L = spai.lib()
    if not _ready:
        vp, u32, u64, i32, P = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.POINTER
        L.spai_chess_config_default.argtypes = [P(Config)]
        L.spai_chess_create.argtypes = [P(Config), i32, P(vp)]
        L.spai_chess_destroy.argtypes = [vp]
        L.spai_chess_sync.argtypes = [vp]
        L.spai_chess_games_resize.argtypes = [vp, u32]
        L.spai_chess_games_write.argtypes = [vp, u32, u32, vp]
        L.spai_chess_games_read.argtypes = [vp, u32, u32, vp]
        L.spai_chess_legal_moves.argtypes = [vp, u32, u32, vp, vp]
        L.spai_chess_apply.argtypes = [vp, u32, u32, vp, vp]
        L.spai_chess_status.argtypes = [vp, u32, u32, vp, vp, vp, vp]
        L.spai_chess_encode.argtypes = [vp, u32, u32, vp]
        L.spai_chess_mask_invalid.argtypes = [vp, u32, u32, vp, u32, vp]
        L.spai_chess_move_index.argtypes = [i32, C.c_uint16, P(C.c_int32)]
        L.spai_chess_index_move.argtypes = [i32, C.c_int32, P(C.c_uint16)]
        L.spai_chess_net_num_params.argtypes = [i32, P(C.c_size_t)]
        L.spai_chess_net_init_params.argtypes = [i32, u64, vp]
        L.spai_chess_net_create.argtypes = [vp, i32, vp, C.c_size_t, P(vp)]
        L.spai_chess_net_destroy.argtypes = [vp]
        L.spai_chess_net_forward.argtypes = [vp, u32, vp, vp, vp]
        L.spai_chess_predict.argtypes = [vp, u32, u32, vp, vp]
        L.spai_chess_rules_bench.argtypes = [vp, u32, u32, u32, vp]
        L.spai_chess_perft.argtypes = [vp, u32, C.c_int, vp]
        L.spai_chess_tree_reset.argtypes = [vp, u32, u32]
        L.spai_chess_set_net.argtypes = [vp, vp]
        L.spai_chess_trees_create.argtypes = [vp, u32]
        L.spai_chess_search.argtypes = [vp, u32, vp, u32, vp, vp, vp, vp, vp]
        L.spai_chess_tree_use_subtree.argtypes = [vp, u32, u32]
        L.spai_chess_tree_root.argtypes = [vp, u32, vp, vp, vp]
        L.spai_chess_trees_advance.argtypes = [vp, u32, vp, vp, vp, vp]
        L.spai_chess_selfplay_run.argtypes = [vp, u32, u64, SINK, vp, P(SelfPlayStats)]
        L.spai_chess_selfplay_stream.argtypes = [vp, u32, u32, u64, SINK, vp, P(SelfPlayStats)]
        L.spai_chess_set_timing.argtypes = [vp, i32]
        L.spai_chess_timing.argtypes = [vp, vp, vp, vp]
        _ready = True
    return L


def _check(rc):
    if rc != 0:
        raise SpaiError(rc, lib().spai_last_error().decode())


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def move_index(side, mv):
    """Policy::get_prob / set_prob index (get_channel, chess.rs:311-393)"""
    out = C.c_int32()
    _check(lib().spai_chess_move_index(side, mv, C.byref(out)))
    return out.value


def index_move(side, index):
    """Policy::get_action (chess.rs:395-493), knight-underpromotion bug kept"""
    out = C.c_uint16()
    _check(lib().spai_chess_index_move(side, index, C.byref(out)))
    return out.value


def num_params(blocks):
    n = C.c_size_t()
    _check(lib().spai_chess_net_num_params(blocks, C.byref(n)))
    return n.value


def init_params(blocks, seed=0):
    p = np.zeros(num_params(blocks), np.float32)
    _check(lib().spai_chess_net_init_params(blocks, seed, _p(p)))
    return p


def states_from(boards):
    """oracle-style boards (pieces[6], color[2], side, castle[2], ep) -> STATE_DTYPE array"""
    a = np.zeros(len(boards), STATE_DTYPE)
    for i, b in enumerate(boards):
        a[i]["pieces"] = b["pieces"]
        a[i]["colors"] = b["colors"]
        a[i]["side"] = b["side"]
        a[i]["castle"] = b["castle"]
        a[i]["ep"] = b["ep"]
        a[i]["fifty"] = b.get("fifty", 0)
        a[i]["made"] = b.get("made", 0)
    return a


class ChessEngine:
    def __init__(self, num_searches=400, max_trees=1024, eval_kind=EVAL_NET, device=0, c=2.0, temperature=1.25,
                 seed=0, max_moves=None):
        cfg = Config()
        _check(lib().spai_chess_config_default(C.byref(cfg)))
        cfg.c, cfg.num_searches, cfg.temperature = c, num_searches, temperature
        cfg.max_trees, cfg.eval, cfg.seed = max_trees, eval_kind, seed
        if max_moves is not None:
            cfg.max_moves = max_moves
        self.cfg = cfg
        h = C.c_void_p()
        _check(lib().spai_chess_create(C.byref(cfg), device, C.byref(h)))
        self.h = h
        self.net = None

    def close(self):
        if getattr(self, "h", None):
            if self.net is not None:
                self.net.close()
                self.net = None
            lib().spai_chess_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- rules
    def games_resize(self, n):
        _check(lib().spai_chess_games_resize(self.h, n))

    def games_write(self, states, first=0):
        a = np.ascontiguousarray(states, STATE_DTYPE)
        _check(lib().spai_chess_games_write(self.h, first, len(a), _p(a)))

    def games_read(self, n, first=0):
        a = np.zeros(n, STATE_DTYPE)
        _check(lib().spai_chess_games_read(self.h, first, n, _p(a)))
        return a

    def legal_moves(self, n, first=0):
        mv = np.zeros((n, MAX_MOVES), np.uint16)
        cnt = np.zeros(n, np.uint32)
        _check(lib().spai_chess_legal_moves(self.h, first, n, _p(mv), _p(cnt)))
        return mv, cnt

    def apply(self, moves, first=0, check=True):
        m = np.ascontiguousarray(moves, np.uint16)
        rc = np.zeros(len(m), np.int32)
        r = lib().spai_chess_apply(self.h, first, len(m), _p(m), _p(rc))
        if check:
            _check(r)
        return rc

    def status(self, n, first=0):
        st = np.zeros(n, np.uint8)
        reps = np.zeros(n, np.uint32)
        v = np.zeros(n, np.float32)
        term = np.zeros(n, np.uint8)
        _check(lib().spai_chess_status(self.h, first, n, _p(st), _p(reps), _p(v), _p(term)))
        return st, reps, v, term

    def rules_bench(self, n, first=0, iters=10):
        """device ms per launch: [legal moves + status, encoding] over slots [first, first+n)"""
        ms = np.zeros(2, np.float64)
        _check(lib().spai_chess_rules_bench(self.h, first, n, iters, _p(ms)))
        return ms

    def perft(self, depth, slot=0):
        """[perft(1), ..., perft(depth)] of slot `slot`'s position, on the device"""
        out = np.zeros(depth, np.uint64)
        _check(lib().spai_chess_perft(self.h, slot, depth, _p(out)))
        return [int(v) for v in out]

    def encode(self, n, first=0):
        out = np.zeros((n, 19, 8, 8), np.float32)
        _check(lib().spai_chess_encode(self.h, first, n, _p(out)))
        return out

    def mask_invalid(self, policy, first=0):
        p = np.ascontiguousarray(policy, np.float32)
        p2 = p.reshape(p.shape[0], -1)
        out = np.zeros((p2.shape[0], POLICY), np.float32)
        _check(lib().spai_chess_mask_invalid(self.h, first, p2.shape[0], _p(p2), p2.shape[1], _p(out)))
        return out

    # ---- net / search
    def set_net(self, net):
        _check(lib().spai_chess_set_net(self.h, net.h if net else None))
        self.net = net

    def trees_create(self, n):
        _check(lib().spai_chess_trees_create(self.h, n))

    def search(self, trees, num_searches=None):
        idx = np.ascontiguousarray(trees, np.uint32)
        n = len(idx)
        pol = np.zeros((n, POLICY), np.float32)
        ids = np.zeros((n, MAX_MOVES), np.uint32)
        vis = np.zeros((n, MAX_MOVES), np.float32)
        mv = np.zeros((n, MAX_MOVES), np.uint16)
        nc = np.zeros(n, np.uint32)
        ns = self.cfg.num_searches if num_searches is None else num_searches
        _check(lib().spai_chess_search(self.h, n, _p(idx), ns, _p(pol), _p(ids), _p(vis), _p(mv), _p(nc)))
        return pol, ids, vis, mv, nc

    def tree_reset(self, tree, slot):
        """Tree::with_root_state(state of game slot `slot`)"""
        _check(lib().spai_chess_tree_reset(self.h, tree, slot))

    def use_subtree(self, tree, child_index):
        _check(lib().spai_chess_tree_use_subtree(self.h, tree, child_index))

    def advance(self, trees, child_index):
        t = np.ascontiguousarray(trees, np.uint32)
        k = np.ascontiguousarray(child_index, np.uint32)
        st = np.zeros(len(t), np.uint8)
        reps = np.zeros(len(t), np.uint32)
        _check(lib().spai_chess_trees_advance(self.h, len(t), _p(t), _p(k), _p(st), _p(reps)))
        return st, reps

    def tree_root(self, tree):
        st = np.zeros(1, STATE_DTYPE)
        n = C.c_uint32()
        w = C.c_float()
        _check(lib().spai_chess_tree_root(self.h, tree, _p(st), C.byref(n), C.byref(w)))
        return st[0], n.value, w.value

    def self_play(self, n_games, game_id_base=0, keep=True, keep_policy=True, window=None):
        """SelfPlayWorker::self_play over n_games games; window: play them through
        that many tree slots (spai_chess_selfplay_stream), games in finishing order"""
        games = []

        def sink(user, gid, n, enc, pol, val, moves):
            if keep:
                g = dict(game=gid, n=n,
                         enc=np.ctypeslib.as_array(enc, (n, ENC)).copy(),
                         value=np.ctypeslib.as_array(val, (n,)).copy(),
                         moves=np.ctypeslib.as_array(moves, (n,)).copy())
                if keep_policy:
                    g["policy"] = np.ctypeslib.as_array(pol, (n, POLICY)).copy()
                games.append(g)

        cb = SINK(sink)
        st = SelfPlayStats()
        if window is None:
            _check(lib().spai_chess_selfplay_run(self.h, n_games, game_id_base, cb, None, C.byref(st)))
        else:
            _check(lib().spai_chess_selfplay_stream(self.h, n_games, int(window), game_id_base, cb, None, C.byref(st)))
        return games, {k: getattr(st, k) for k, _ in SelfPlayStats._fields_}

    def set_timing(self, on=True):
        _check(lib().spai_chess_set_timing(self.h, 1 if on else 0))

    def timing(self):
        ms = np.zeros(3)
        launches = np.zeros(3)
        items = np.zeros(3)
        _check(lib().spai_chess_timing(self.h, _p(ms), _p(launches), _p(items)))
        return ms, launches, items


class ChessNet:
    def __init__(self, eng, blocks, params):
        p = np.ascontiguousarray(params, np.float32)
        h = C.c_void_p()
        _check(lib().spai_chess_net_create(eng.h, blocks, _p(p), p.size, C.byref(h)))
        self.h = h
        self.eng = eng
        self.blocks = blocks

    def close(self):
        if getattr(self, "h", None):
            lib().spai_chess_net_destroy(self.h)
            self.h = None

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 19 * 64)
        n = x.shape[0]
        lg = np.zeros((n, POLICY), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_chess_net_forward(self.h, n, _p(x), _p(lg), _p(v)))
        return lg, v

    def predict(self, n, first=0):
        """Model::predict over the engine's game slots [first, first+n)"""
        pr = np.zeros((n, POLICY), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_chess_predict(self.h, first, n, _p(pr), _p(v)))
        return pr, v

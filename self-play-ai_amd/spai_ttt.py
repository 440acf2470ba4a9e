"""ctypes binding of the TicTacToe section of libspai.so (include/spai.h):
game/tictactoe.rs + model/tictactoe.rs on the device (BASELINE config 1).
Every call goes through the HIP library; there is no CPU fallback."""
import ctypes as C

import numpy as np

import spai
from spai import EVAL_HASH, EVAL_NET, EVAL_UNIFORM, SINK, Config, SelfPlayStats, SpaiError  # noqa: F401

STATE_DTYPE = np.dtype([("x", "<u2"), ("o", "<u2"), ("n", "u1"), ("status", "u1"), ("pad", "u1", 2)])
assert STATE_DTYPE.itemsize == 8

_ready = False


def lib():
    global _ready
    L = spai.lib()
    if not _ready:
        vp, u32, u64, i32, P = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.POINTER
        L.spai_ttt_create.argtypes = [P(Config), i32, P(vp)]
        L.spai_ttt_destroy.argtypes = [vp]
        L.spai_ttt_games_resize.argtypes = [vp, u32]
        L.spai_ttt_games_write.argtypes = [vp, u32, u32, vp]
        L.spai_ttt_games_read.argtypes = [vp, u32, u32, vp]
        L.spai_ttt_legal_mask.argtypes = [vp, u32, u32, vp]
        L.spai_ttt_apply.argtypes = [vp, u32, u32, vp, vp]
        L.spai_ttt_encode.argtypes = [vp, u32, u32, vp]
        L.spai_ttt_mask_invalid.argtypes = [vp, u32, u32, vp, u32, vp]
        L.spai_ttt_net_num_params.argtypes = [i32, P(C.c_size_t)]
        L.spai_ttt_net_init_params.argtypes = [i32, u64, vp]
        L.spai_ttt_net_create.argtypes = [vp, i32, vp, C.c_size_t, P(vp)]
        L.spai_ttt_net_destroy.argtypes = [vp]
        L.spai_ttt_net_forward.argtypes = [vp, u32, vp, vp, vp]
        L.spai_ttt_predict.argtypes = [vp, u32, u32, vp, vp]
        L.spai_ttt_set_net.argtypes = [vp, vp]
        L.spai_ttt_trees_create.argtypes = [vp, u32]
        L.spai_ttt_search.argtypes = [vp, u32, vp, u32, vp, vp, vp, vp]
        L.spai_ttt_tree_use_subtree.argtypes = [vp, u32, u32]
        L.spai_ttt_tree_reset.argtypes = [vp, u32, vp]
        L.spai_ttt_selfplay_run.argtypes = [vp, u32, u64, SINK, vp, P(SelfPlayStats)]
        L.spai_ttt_selfplay_stream.argtypes = [vp, u32, u32, u64, SINK, vp, P(SelfPlayStats)]
        _ready = True
    return L


def _check(rc):
    if rc != 0:
        raise SpaiError(rc, lib().spai_last_error().decode())


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def num_params(blocks):
    n = C.c_size_t()
    _check(lib().spai_ttt_net_num_params(blocks, C.byref(n)))
    return n.value


def init_params(blocks, seed=0):
    p = np.zeros(num_params(blocks), np.float32)
    _check(lib().spai_ttt_net_init_params(blocks, seed, _p(p)))
    return p


class TTTEngine:
    def __init__(self, num_searches=64, max_trees=1, eval_kind=EVAL_NET, device=0, c=2.0, temperature=1.25, seed=0):
        cfg = Config()
        cfg.c, cfg.num_searches, cfg.temperature = c, num_searches, temperature
        cfg.max_trees, cfg.max_moves, cfg.eval, cfg.seed = max_trees, 9, eval_kind, seed
        self.cfg = cfg
        h = C.c_void_p()
        _check(lib().spai_ttt_create(C.byref(cfg), device, C.byref(h)))
        self.h = h
        self.net = None

    def close(self):
        if getattr(self, "h", None):
            if self.net is not None:
                self.net.close()
                self.net = None
            lib().spai_ttt_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def games_resize(self, n):
        _check(lib().spai_ttt_games_resize(self.h, n))

    def games_write(self, states, first=0):
        a = np.ascontiguousarray(states, STATE_DTYPE)
        _check(lib().spai_ttt_games_write(self.h, first, len(a), _p(a)))

    def games_read(self, n, first=0):
        a = np.zeros(n, STATE_DTYPE)
        _check(lib().spai_ttt_games_read(self.h, first, n, _p(a)))
        return a

    def legal_mask(self, n, first=0):
        m = np.zeros(n, np.uint32)
        _check(lib().spai_ttt_legal_mask(self.h, first, n, _p(m)))
        return m

    def apply(self, actions, first=0, check=True):
        a = np.ascontiguousarray(actions, np.int32)
        rc = np.zeros(len(a), np.int32)
        r = lib().spai_ttt_apply(self.h, first, len(a), _p(a), _p(rc))
        if check:
            _check(r)
        return rc

    def encode(self, n, first=0):
        out = np.zeros((n, 3, 3, 3), np.float32)
        _check(lib().spai_ttt_encode(self.h, first, n, _p(out)))
        return out

    def mask_invalid(self, policy, first=0):
        p = np.ascontiguousarray(policy, np.float32)
        p2 = p.reshape(p.shape[0], -1)
        out = np.zeros((p2.shape[0], 9), np.float32)
        _check(lib().spai_ttt_mask_invalid(self.h, first, p2.shape[0], _p(p2), p2.shape[1], _p(out)))
        return out

    def set_net(self, net):
        _check(lib().spai_ttt_set_net(self.h, net.h if net else None))
        self.net = net

    def trees_create(self, n):
        _check(lib().spai_ttt_trees_create(self.h, n))

    def search(self, trees, num_searches=None):
        idx = np.ascontiguousarray(trees, np.uint32)
        n = len(idx)
        pol = np.zeros((n, 9), np.float32)
        ids = np.zeros((n, 9), np.uint32)
        vis = np.zeros((n, 9), np.float32)
        nc = np.zeros(n, np.uint32)
        ns = self.cfg.num_searches if num_searches is None else num_searches
        _check(lib().spai_ttt_search(self.h, n, _p(idx), ns, _p(pol), _p(ids), _p(vis), _p(nc)))
        return pol, ids, vis, nc

    def tree_reset(self, tree, state):
        """Tree::with_root_state(state); state = one STATE_DTYPE record"""
        a = np.ascontiguousarray(np.asarray(state, STATE_DTYPE).reshape(1))
        _check(lib().spai_ttt_tree_reset(self.h, tree, _p(a)))

    def use_subtree(self, tree, child_index):
        _check(lib().spai_ttt_tree_use_subtree(self.h, tree, child_index))

    def self_play(self, n_games, game_id_base=0, window=None):
        """SelfPlayWorker::self_play; window: through that many tree slots
        (spai_ttt_selfplay_stream), games in finishing order"""
        games = []

        def sink(user, gid, n, enc, pol, val, moves):
            games.append(dict(game=gid, n=n, enc=np.ctypeslib.as_array(enc, (n, 27)).copy(),
                              policy=np.ctypeslib.as_array(pol, (n, 9)).copy(),
                              value=np.ctypeslib.as_array(val, (n,)).copy(),
                              moves=np.ctypeslib.as_array(moves, (n,)).copy()))

        cb = SINK(sink)
        st = SelfPlayStats()
        if window is None:
            _check(lib().spai_ttt_selfplay_run(self.h, n_games, game_id_base, cb, None, C.byref(st)))
        else:
            _check(lib().spai_ttt_selfplay_stream(self.h, n_games, int(window), game_id_base, cb, None, C.byref(st)))
        return games, {k: getattr(st, k) for k, _ in SelfPlayStats._fields_}


class TTTNet:
    def __init__(self, eng, blocks, params):
        p = np.ascontiguousarray(params, np.float32)
        h = C.c_void_p()
        _check(lib().spai_ttt_net_create(eng.h, blocks, _p(p), p.size, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().spai_ttt_net_destroy(self.h)
            self.h = None

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 27)
        n = x.shape[0]
        lg = np.zeros((n, 9), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_ttt_net_forward(self.h, n, _p(x), _p(lg), _p(v)))
        return lg, v

    def predict(self, n, first=0):
        """Model::predict over the engine's game slots [first, first+n)"""
        pr = np.zeros((n, 9), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_ttt_predict(self.h, first, n, _p(pr), _p(v)))
        return pr, v

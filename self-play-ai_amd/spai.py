"""ctypes binding of libspai.so (include/spai.h) — the Python face of the engine.

Mirrors the reference's hot-path surface (joshua16266261/self-play-ai):
  State (game/connect_four.rs)     -> Engine.games_* / legal_mask / apply / encode / mask_invalid
  Net + Model::predict (model/)    -> Net.forward / Net.predict
  Tree + Mcts::search (mcts.rs)    -> Engine.trees_create / search / use_subtree
  SelfPlayWorker::self_play        -> Engine.self_play
Every call goes through the HIP library; there is no CPU fallback.  Importing
this module on a machine without the built library raises immediately.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SPAI_LIB") or os.path.join(HERE, "libspai.so")

GAME_TICTACTOE, GAME_CONNECT4, GAME_CHESS = 0, 1, 2
EVAL_NET, EVAL_UNIFORM, EVAL_HASH = 0, 1, 2
DTYPE_BF16, DTYPE_F32 = 0, 1   # spai_dtype
ONGOING, TIED, WON = 0, 1, 2
OK = 0
ERRORS = {-1: "INVALID", -2: "ILLEGAL_MOVE", -3: "GAME_OVER", -4: "DEVICE", -5: "NAN", -6: "CAPACITY",
          -7: "UNSUPPORTED"}

# every symbol declared in include/spai.h
SYMBOLS = [
    "spai_last_error", "spai_version", "spai_device_count", "spai_config_default", "spai_engine_create",
    "spai_engine_destroy", "spai_engine_sync", "spai_games_resize", "spai_games_reset", "spai_games_write",
    "spai_games_read", "spai_legal_mask", "spai_apply", "spai_value_terminated", "spai_encode",
    "spai_mask_invalid", "spai_rules_bench", "spai_net_num_params", "spai_net_init_params", "spai_net_create",
    "spai_net_destroy", "spai_net_forward", "spai_predict", "spai_engine_set_net", "spai_trees_create",
    "spai_tree_reset", "spai_search", "spai_tree_use_subtree", "spai_tree_node", "spai_tree_size",
    "spai_selfplay_run", "spai_selfplay_stream", "spai_engine_set_timing", "spai_engine_timing", "spai_engine_timing_items",
    "spai_net_phase_cycles", "spai_net_bench", "spai_net_bench_conc", "spai_adam_config_default", "spai_learner_create", "spai_learner_destroy",
    "spai_learner_train_batch", "spai_learner_train_batches", "spai_learner_params", "spai_learner_grads", "spai_learner_activation", "spai_comm_unique_id",
    "spai_learner_set_comm", "spai_learner_broadcast", "spai_learner_set_host_comm", "spai_learner_last_batch",
    "spai_comm_create", "spai_comm_allreduce_f64", "spai_comm_info", "spai_comm_destroy",
    "spai_params_save_safetensors", "spai_params_load_safetensors",
    "spai_replay_create", "spai_replay_destroy", "spai_replay_push", "spai_replay_pop", "spai_replay_size",
    "spai_choose_multiple", "spai_pipeline_config_default", "spai_pipeline_run", "spai_learner_train",
    "spai_policy_normalize", "spai_policy_best_action", "spai_policy_sample",
    # chess (spai_chess.py)
    "spai_chess_config_default", "spai_chess_create", "spai_chess_destroy", "spai_chess_sync",
    "spai_chess_games_resize", "spai_chess_games_write", "spai_chess_games_read", "spai_chess_legal_moves",
    "spai_chess_apply", "spai_chess_status", "spai_chess_encode", "spai_chess_rules_bench", "spai_chess_perft", "spai_chess_mask_invalid",
    "spai_chess_move_index", "spai_chess_index_move", "spai_chess_net_num_params", "spai_chess_net_init_params",
    "spai_chess_net_create", "spai_chess_net_destroy", "spai_chess_net_forward", "spai_chess_predict", "spai_chess_set_net",
    "spai_chess_trees_create", "spai_chess_search", "spai_chess_tree_reset", "spai_chess_tree_use_subtree", "spai_chess_tree_root", "spai_chess_trees_advance",
    "spai_chess_selfplay_run", "spai_chess_selfplay_stream", "spai_chess_set_timing", "spai_chess_timing",
    # tictactoe (spai_ttt.py)
    "spai_ttt_create", "spai_ttt_destroy", "spai_ttt_games_resize", "spai_ttt_games_write", "spai_ttt_games_read",
    "spai_ttt_legal_mask", "spai_ttt_apply", "spai_ttt_encode", "spai_ttt_mask_invalid", "spai_ttt_net_num_params",
    "spai_ttt_net_init_params", "spai_ttt_net_create", "spai_ttt_net_destroy", "spai_ttt_net_forward",
    "spai_ttt_predict",
    "spai_ttt_set_net", "spai_ttt_trees_create", "spai_ttt_search", "spai_ttt_tree_reset", "spai_ttt_tree_use_subtree",
    "spai_ttt_selfplay_run", "spai_ttt_selfplay_stream",
]
COMM_ID_BYTES = 128


class SpaiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"spai error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class C4State(C.Structure):
    _fields_ = [("x", C.c_uint64), ("o", C.c_uint64), ("num_actions_played", C.c_uint8), ("status", C.c_uint8),
                ("pad", C.c_uint8 * 6)]


class Config(C.Structure):
    _fields_ = [("c", C.c_float), ("num_searches", C.c_uint32), ("temperature", C.c_float),
                ("max_trees", C.c_uint32), ("max_moves", C.c_uint32), ("eval", C.c_uint32), ("seed", C.c_uint64)]


class SelfPlayStats(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("sims", "evals", "games", "positions", "moves", "seconds")]


class AdamConfig(C.Structure):
    _fields_ = [(k, C.c_float) for k in ("lr", "beta1", "beta2", "eps", "bn_momentum", "bn_eps")]


class PipelineConfig(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("n_selfplay", C.c_uint32), ("selfplay_devices", C.POINTER(C.c_int)), ("learner_device", C.c_int),
                ("games_per_batch", C.c_uint32), ("num_searches", C.c_uint32), ("c", C.c_float),
                ("temperature", C.c_float), ("batch_size", C.c_uint32), ("batches_per_iter", C.c_uint32),
                ("train_iters", C.c_uint32), ("replay_capacity", C.c_uint32), ("sample_fraction", C.c_float),
                ("blocks", C.c_int), ("seed", C.c_uint64), ("checkpoint_dir", C.c_char_p),
                ("observer", C.c_void_p), ("observer_user", C.c_void_p)]


class PipelineEvent(C.Structure):
    _fields_ = [("kind", C.c_int32), ("worker", C.c_uint32), ("batch", C.c_uint64), ("version", C.c_uint64),
                ("n", C.c_uint32), ("positions", C.c_uint32), ("ring_size", C.c_uint32), ("pad", C.c_uint32),
                ("states", C.POINTER(C.c_float)), ("policies", C.POINTER(C.c_float)),
                ("values", C.POINTER(C.c_float))]


PIPE_PUSH, PIPE_POP = 0, 1
OBSERVER = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(PipelineEvent))


class PipelineStats(C.Structure):
    _fields_ = [(k, C.c_double) for k in ("games", "positions", "samples_pushed", "samples_overwritten",
                                          "batches_trained")] + \
               [("last_loss", C.c_double * 3)] + \
               [(k, C.c_double) for k in ("weight_version_published", "weight_version_used_max", "seconds")]


HOST_ALLREDUCE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_size_t)

SINK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                   C.POINTER(C.c_float), C.POINTER(C.c_int32))

C4_STATE_DTYPE = np.dtype([("x", "<u8"), ("o", "<u8"), ("n", "u1"), ("status", "u1"), ("pad", "u1", 6)])

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C self-play-ai_amd` (hipcc, gfx950)")
        L = C.CDLL(LIB_PATH)
        vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        P = C.POINTER
        for name in SYMBOLS:
            getattr(L, name).restype = C.c_int
        L.spai_last_error.restype = C.c_char_p
        L.spai_version.restype = C.c_char_p
        L.spai_device_count.argtypes = [P(C.c_int)]
        L.spai_config_default.argtypes = [i32, P(Config)]
        L.spai_engine_create.argtypes = [i32, P(Config), i32, P(vp)]
        L.spai_engine_destroy.argtypes = [vp]
        L.spai_engine_sync.argtypes = [vp]
        L.spai_games_resize.argtypes = [vp, u32]
        L.spai_games_reset.argtypes = [vp, u32, u32]
        L.spai_games_write.argtypes = [vp, u32, u32, vp]
        L.spai_games_read.argtypes = [vp, u32, u32, vp]
        L.spai_legal_mask.argtypes = [vp, u32, u32, vp]
        L.spai_apply.argtypes = [vp, u32, u32, vp, vp]
        L.spai_value_terminated.argtypes = [vp, u32, u32, vp, vp]
        L.spai_encode.argtypes = [vp, u32, u32, vp]
        L.spai_mask_invalid.argtypes = [vp, u32, u32, vp, u32, vp]
        L.spai_rules_bench.argtypes = [vp, u32, u32, vp]
        L.spai_net_num_params.argtypes = [i32, i32, i32, P(C.c_size_t)]
        L.spai_net_init_params.argtypes = [i32, i32, i32, u64, vp]
        L.spai_net_create.argtypes = [vp, i32, i32, vp, C.c_size_t, i32, P(vp)]
        L.spai_net_destroy.argtypes = [vp]
        L.spai_net_forward.argtypes = [vp, u32, vp, vp, vp]
        L.spai_predict.argtypes = [vp, u32, vp, vp, vp]
        L.spai_engine_set_net.argtypes = [vp, vp]
        L.spai_trees_create.argtypes = [vp, u32]
        L.spai_tree_reset.argtypes = [vp, u32, vp]
        L.spai_search.argtypes = [vp, u32, vp, u32, vp, vp, vp, vp]
        L.spai_tree_use_subtree.argtypes = [vp, u32, u32]
        L.spai_tree_node.argtypes = [vp, u32, u32, vp, vp, vp]
        L.spai_tree_size.argtypes = [vp, u32, vp]
        L.spai_selfplay_run.argtypes = [vp, u32, u64, SINK, vp, P(SelfPlayStats)]
        L.spai_selfplay_stream.argtypes = [vp, u32, u32, u64, SINK, vp, P(SelfPlayStats)]
        L.spai_engine_set_timing.argtypes = [vp, i32]
        L.spai_engine_timing.argtypes = [vp, vp, vp]
        L.spai_engine_timing_items.argtypes = [vp, vp, vp]
        L.spai_net_phase_cycles.argtypes = [vp, u32, vp]
        L.spai_net_bench.argtypes = [vp, u32, u32, vp]
        L.spai_net_bench_conc.argtypes = [vp, u32, u32, i32, vp]
        L.spai_adam_config_default.argtypes = [P(AdamConfig)]
        L.spai_learner_create.argtypes = [vp, i32, i32, vp, C.c_size_t, P(AdamConfig), P(vp)]
        L.spai_learner_destroy.argtypes = [vp]
        L.spai_learner_train_batch.argtypes = [vp, u32, vp, vp, vp, vp]
        L.spai_learner_train_batches.argtypes = [vp, u32, u32, vp, vp, vp, vp]
        L.spai_learner_params.argtypes = [vp, vp, C.c_size_t]
        L.spai_learner_grads.argtypes = [vp, vp, C.c_size_t]
        L.spai_learner_activation.argtypes = [vp, C.c_int, vp, C.c_size_t]
        L.spai_learner_train.argtypes = [vp, u32, vp, vp, vp, u32, u32, u64, vp]
        L.spai_comm_unique_id.argtypes = [vp]
        L.spai_learner_set_comm.argtypes = [vp, i32, i32, vp]
        L.spai_learner_broadcast.argtypes = [vp, i32]
        L.spai_learner_set_host_comm.argtypes = [vp, i32, i32, HOST_ALLREDUCE, vp]
        L.spai_learner_last_batch.argtypes = [vp, P(u32)]
        L.spai_comm_create.argtypes = [i32, i32, i32, vp, P(vp)]
        L.spai_comm_allreduce_f64.argtypes = [vp, vp, C.c_size_t, i32]
        L.spai_comm_info.argtypes = [vp, P(i32), P(i32), P(i32)]
        L.spai_comm_destroy.argtypes = [vp]
        L.spai_params_save_safetensors.argtypes = [i32, i32, i32, vp, C.c_size_t, C.c_char_p]
        L.spai_params_load_safetensors.argtypes = [i32, i32, i32, C.c_char_p, vp, C.c_size_t]
        L.spai_replay_create.argtypes = [u32, P(vp)]
        L.spai_replay_destroy.argtypes = [vp]
        L.spai_replay_push.argtypes = [vp, u32, vp, vp, vp]
        L.spai_replay_pop.argtypes = [vp, u32, vp, vp, vp]
        L.spai_replay_size.argtypes = [vp, P(u32)]
        L.spai_choose_multiple.argtypes = [u32, u32, u64, u64, vp]
        L.spai_pipeline_config_default.argtypes = [P(PipelineConfig)]
        L.spai_pipeline_run.argtypes = [P(PipelineConfig), vp, C.c_size_t, P(PipelineStats)]
        L.spai_policy_normalize.argtypes = [vp, u32]
        L.spai_policy_best_action.argtypes = [vp, u32, P(u32)]
        L.spai_policy_sample.argtypes = [vp, u32, C.c_float, C.c_float, P(u32)]
        _lib = L
    return _lib


def _check(rc):
    if rc != OK:
        raise SpaiError(rc, lib().spai_last_error().decode())
    return rc


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def device_count():
    n = C.c_int()
    _check(lib().spai_device_count(C.byref(n)))
    return n.value


def num_params(blocks, hidden=64, game=GAME_CONNECT4):
    n = C.c_size_t()
    _check(lib().spai_net_num_params(game, blocks, hidden, C.byref(n)))
    return n.value


def init_params(blocks, hidden=64, seed=0, game=GAME_CONNECT4):
    p = np.zeros(num_params(blocks, hidden, game), np.float32)
    _check(lib().spai_net_init_params(game, blocks, hidden, seed, _p(p)))
    return p


def states_array(states):
    """list of (x, o, n, status) or an existing structured array -> C4_STATE_DTYPE array"""
    if isinstance(states, np.ndarray) and states.dtype == C4_STATE_DTYPE:
        return np.ascontiguousarray(states)
    a = np.zeros(len(states), C4_STATE_DTYPE)
    for i, s in enumerate(states):
        a[i]["x"], a[i]["o"], a[i]["n"], a[i]["status"] = s[0], s[1], s[2], s[3]
    return a


class Net:
    """Net (model/mod.rs:22-28) on the device; Model::predict as .predict()."""

    def __init__(self, engine, blocks, params, hidden=64, dtype=None):
        params = np.ascontiguousarray(params, np.float32)
        self.engine, self.blocks, self.hidden = engine, blocks, hidden
        self.dtype = DTYPE_BF16 if dtype is None else dtype
        h = C.c_void_p()
        _check(lib().spai_net_create(engine.h, blocks, hidden, _p(params), params.size, self.dtype, C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().spai_net_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def forward(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, 126)
        n = x.shape[0]
        lg = np.zeros((n, 7), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_net_forward(self.h, n, _p(x), _p(lg), _p(v)))
        return lg, v

    def phase_cycles(self, count=4096):
        c = np.zeros(48, np.float64)   # 24 stamps; 48 in the k-step diagnostic build (-DSPAI_DIAG_KSTEP)
        _check(lib().spai_net_phase_cycles(self.h, count, _p(c)))
        return c

    def bench(self, count, iters=50, conc=1):
        """ms per forward launch alone on `count` random positions (spai_net_bench); conc > 1:
        at the group size the search picks for conc concurrent chains (spai_net_bench_conc)"""
        ms = np.zeros(1, np.float64)
        _check(lib().spai_net_bench_conc(self.h, count, iters, conc, _p(ms)))
        return float(ms[0])

    def predict(self, states):
        a = states_array(states)
        n = len(a)
        pr = np.zeros((n, 7), np.float32)
        v = np.zeros(n, np.float32)
        _check(lib().spai_predict(self.h, n, _p(a), _p(pr), _p(v)))
        return pr, v


class Engine:
    def __init__(self, num_searches=800, max_trees=4096, eval_kind=EVAL_NET, device=0, c=2.0, temperature=1.25,
                 seed=0, max_moves=42, game=GAME_CONNECT4):
        cfg = Config()
        _check(lib().spai_config_default(game, C.byref(cfg)))
        cfg.c, cfg.num_searches, cfg.temperature = c, num_searches, temperature
        cfg.max_trees, cfg.max_moves, cfg.eval, cfg.seed = max_trees, max_moves, eval_kind, seed
        self.cfg = cfg
        h = C.c_void_p()
        _check(lib().spai_engine_create(game, C.byref(cfg), device, C.byref(h)))
        self.h = h
        self.net = None

    def close(self):
        if getattr(self, "h", None):
            if self.net is not None:
                self.net.close()
                self.net = None
            lib().spai_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def sync(self):
        _check(lib().spai_engine_sync(self.h))

    # ---- rules
    def games_resize(self, n):
        _check(lib().spai_games_resize(self.h, n))

    def games_write(self, states, first=0):
        a = states_array(states)
        _check(lib().spai_games_write(self.h, first, len(a), _p(a)))

    def games_read(self, n, first=0):
        a = np.zeros(n, C4_STATE_DTYPE)
        _check(lib().spai_games_read(self.h, first, n, _p(a)))
        return a

    def legal_mask(self, n, first=0):
        m = np.zeros(n, np.uint32)
        _check(lib().spai_legal_mask(self.h, first, n, _p(m)))
        return m

    def apply(self, actions, first=0, check=True):
        a = np.ascontiguousarray(actions, np.int32)
        rc = np.zeros(len(a), np.int32)
        r = lib().spai_apply(self.h, first, len(a), _p(a), _p(rc))
        if check:
            _check(r)
        return rc

    def value_terminated(self, n, first=0):
        v = np.zeros(n, np.float32)
        t = np.zeros(n, np.uint8)
        _check(lib().spai_value_terminated(self.h, first, n, _p(v), _p(t)))
        return v, t

    def encode(self, n, first=0):
        e = np.zeros((n, 3, 6, 7), np.float32)
        _check(lib().spai_encode(self.h, first, n, _p(e)))
        return e

    def mask_invalid(self, policy, first=0):
        p = np.ascontiguousarray(policy, np.float32)
        n, ln = p.shape
        out = np.zeros((n, 7), np.float32)
        _check(lib().spai_mask_invalid(self.h, first, n, _p(p), ln, _p(out)))
        return out

    def rules_bench(self, n, iters=20):
        ms = np.zeros(3, np.float64)
        _check(lib().spai_rules_bench(self.h, n, iters, _p(ms)))
        return ms

    # ---- net
    def set_net(self, net):
        _check(lib().spai_engine_set_net(self.h, net.h if net is not None else None))
        self.net = net

    # ---- search
    def trees_create(self, n):
        _check(lib().spai_trees_create(self.h, n))

    def tree_reset(self, t, root=None):
        if root is None:
            _check(lib().spai_tree_reset(self.h, t, None))
        else:
            a = states_array([root])
            _check(lib().spai_tree_reset(self.h, t, _p(a)))

    def search(self, tree_idx, num_searches=None):
        idx = np.ascontiguousarray(tree_idx, np.uint32)
        n = len(idx)
        ns = self.cfg.num_searches if num_searches is None else num_searches
        pol = np.zeros((n, 7), np.float32)
        ids = np.zeros((n, 7), np.uint32)
        vis = np.zeros((n, 7), np.float32)
        nc = np.zeros(n, np.uint32)
        _check(lib().spai_search(self.h, n, _p(idx), ns, _p(pol), _p(ids), _p(vis), _p(nc)))
        return pol, ids, vis, nc

    def use_subtree(self, t, child_id):
        _check(lib().spai_tree_use_subtree(self.h, t, int(child_id)))

    def tree_node(self, t, node):
        a = np.zeros(1, C4_STATE_DTYPE)
        vis = C.c_uint32()
        w = C.c_float()
        _check(lib().spai_tree_node(self.h, t, int(node), _p(a), C.byref(vis), C.byref(w)))
        return a[0], vis.value, w.value

    def tree_size(self, t):
        n = C.c_uint32()
        _check(lib().spai_tree_size(self.h, t, C.byref(n)))
        return n.value

    # ---- self-play
    def self_play(self, n_games, game_id_base=0, collect=True, window=None):
        """SelfPlayWorker::self_play over n_games games (spai_selfplay_run); window:
        play them through that many tree slots, refilled as games end
        (spai_selfplay_stream)"""
        games = []

        def sink(user, gid, n, enc, pol, val, moves):
            if collect:
                games.append(dict(game=gid,
                                  enc=np.ctypeslib.as_array(enc, (n, 126)).copy(),
                                  policy=np.ctypeslib.as_array(pol, (n, 7)).copy(),
                                  value=np.ctypeslib.as_array(val, (n,)).copy(),
                                  moves=np.ctypeslib.as_array(moves, (n,)).copy()))

        cb = SINK(sink)
        st = SelfPlayStats()
        if window is None:
            _check(lib().spai_selfplay_run(self.h, n_games, game_id_base, cb, None, C.byref(st)))
        else:
            _check(lib().spai_selfplay_stream(self.h, n_games, window, game_id_base, cb, None, C.byref(st)))
        return games, {k: getattr(st, k) for k, _ in SelfPlayStats._fields_}

    # ---- profiling
    def set_timing(self, on, stride=None):
        """on: enable the sampled HIP events; stride: sample every stride-th iteration (default 4)"""
        _check(lib().spai_engine_set_timing(self.h, (int(stride) if stride and stride > 1 else 1) if on else 0))

    def timing(self):
        avg = np.zeros(3, np.float64)
        launches = np.zeros(3, np.float64)
        tot = np.zeros(3, np.float64)
        items = np.zeros(3, np.float64)
        _check(lib().spai_engine_timing(self.h, _p(avg), _p(launches)))
        _check(lib().spai_engine_timing_items(self.h, _p(tot), _p(items)))
        names = ("select", "evaluate", "expand")
        return {nm: dict(avg_ms=avg[i], launches=launches[i], total_ms=tot[i], items=items[i])
                for i, nm in enumerate(names)}


class Learner:
    """Device training step (ModelTrainerWorker::train_batch, learner_concurrent.rs:72-85):
    train-mode forward, policy NLL + value MSE, backward, one Adam step."""

    def __init__(self, engine, blocks, params, hidden=64, **adam):
        cfg = AdamConfig()
        _check(lib().spai_adam_config_default(C.byref(cfg)))
        for k, v in adam.items():
            setattr(cfg, k, float(v))
        self.params0 = np.ascontiguousarray(params, np.float32)
        self.n = len(self.params0)
        self.blocks, self.hidden = blocks, hidden
        self._host_ar = None
        self.h = C.c_void_p()
        _check(lib().spai_learner_create(engine.h, blocks, hidden, _p(self.params0), self.n, C.byref(cfg),
                                         C.byref(self.h)))

    def train_batch(self, states, policies, values):
        x = np.ascontiguousarray(states, np.float32).reshape(-1, 126)
        pi = np.ascontiguousarray(policies, np.float32).reshape(-1, 7)
        z = np.ascontiguousarray(values, np.float32).reshape(-1)
        assert len(x) == len(pi) == len(z)
        loss = np.zeros(3, np.float32)
        _check(lib().spai_learner_train_batch(self.h, len(x), _p(x), _p(pi), _p(z), _p(loss)))
        return loss   # total, policy, value

    def train_batches(self, states, policies, values, k):
        """k consecutive train_batch steps over equal slices of the arrays, one host
        sync at the end; returns the k x 3 losses (total, policy, value)"""
        x = np.ascontiguousarray(states, np.float32).reshape(-1, 126)
        pi = np.ascontiguousarray(policies, np.float32).reshape(-1, 7)
        z = np.ascontiguousarray(values, np.float32).reshape(-1)
        assert len(x) == len(pi) == len(z) and k >= 1 and len(z) % k == 0
        loss = np.zeros((k, 3), np.float32)
        _check(lib().spai_learner_train_batches(self.h, k, len(z) // k, _p(x), _p(pi), _p(z), _p(loss)))
        return loss

    def train(self, states, policies, values, epochs=1, batch=128, seed=0):
        """Model::train (model/mod.rs:100-149): fresh Adam, one permutation, epochs x batches"""
        x = np.ascontiguousarray(states, np.float32).reshape(-1, 126)
        pi = np.ascontiguousarray(policies, np.float32).reshape(-1, 7)
        z = np.ascontiguousarray(values, np.float32).reshape(-1)
        loss = np.zeros(3, np.float32)
        _check(lib().spai_learner_train(self.h, len(z), _p(x), _p(pi), _p(z), epochs, batch, seed, _p(loss)))
        return loss

    @property
    def last_batch(self):
        """the batch size of the latest train step (the C side's, so it follows train() too)"""
        n = C.c_uint32()
        _check(lib().spai_learner_last_batch(self.h, C.byref(n)))
        return n.value

    def params(self):
        out = np.zeros(self.n, np.float32)
        _check(lib().spai_learner_params(self.h, _p(out), self.n))
        return out

    def grads(self):
        out = np.zeros(self.n, np.float32)
        _check(lib().spai_learner_grads(self.h, _p(out), self.n))
        return out

    def activation(self, layer):
        """the last train step's post-ReLU activations of conv `layer` (stem, residual
        convs, policy head, value head), [B][co][6][7]"""
        nl = 2 * self.blocks + 3
        co = 32 if layer == nl - 2 else 3 if layer == nl - 1 else self.hidden
        out = np.zeros((self.last_batch, co, 6, 7), np.float32)
        _check(lib().spai_learner_activation(self.h, layer, _p(out), out.size))
        return out

    def set_comm(self, rank, world, uid=None):
        buf = None if uid is None else np.frombuffer(bytes(uid), np.uint8).copy()
        _check(lib().spai_learner_set_comm(self.h, rank, world, None if buf is None else _p(buf)))
        self._host_ar = None

    def set_host_comm(self, rank, world, allreduce):
        """host collective in place of RCCL: allreduce(buf) sums the float32 array buf
        over the ranks in place (same rank order everywhere); None drops it"""
        if allreduce is None:
            self._host_ar = None
            _check(lib().spai_learner_set_host_comm(self.h, 0, 1, HOST_ALLREDUCE(), None))
            return

        def fn(_user, ptr, n):
            try:
                allreduce(np.ctypeslib.as_array(ptr, shape=(n,)))
                return 0
            except Exception:   # an error must not unwind through C; the step reports it
                import traceback
                traceback.print_exc()
                return 1

        self._host_ar = HOST_ALLREDUCE(fn)   # kept alive while the learner may call it
        _check(lib().spai_learner_set_host_comm(self.h, rank, world, self._host_ar, None))

    def broadcast(self, root=0):
        """RCCL (or host-collective) broadcast of rank `root`'s parameters to every rank"""
        _check(lib().spai_learner_broadcast(self.h, root))

    def close(self):
        if self.h:
            lib().spai_learner_destroy(self.h)
            self.h = C.c_void_p()


def comm_unique_id():
    buf = np.zeros(COMM_ID_BYTES, np.uint8)
    _check(lib().spai_comm_unique_id(_p(buf)))
    return buf.tobytes()


REDUCE_SUM, REDUCE_MAX = 0, 1


class Comm:
    """stand-alone RCCL communicator, one rank per GPU (spai_comm_*): rank 0 makes
    the id (comm_unique_id), the host group hands it to the other ranks"""

    def __init__(self, device, rank, world, uid):
        buf = np.frombuffer(bytes(uid), np.uint8).copy()
        self.h = C.c_void_p()
        _check(lib().spai_comm_create(device, rank, world, _p(buf), C.byref(self.h)))

    def info(self):
        r, w, d = C.c_int(), C.c_int(), C.c_int()
        _check(lib().spai_comm_info(self.h, C.byref(r), C.byref(w), C.byref(d)))
        return r.value, w.value, d.value

    def allreduce(self, values, op="sum"):
        """list of floats reduced over the ranks (float64 ncclAllReduce)"""
        a = np.ascontiguousarray(values, np.float64).copy()
        _check(lib().spai_comm_allreduce_f64(self.h, _p(a), len(a), REDUCE_MAX if op == "max" else REDUCE_SUM))
        return [float(v) for v in a]

    def close(self):
        if self.h:
            lib().spai_comm_destroy(self.h)
            self.h = C.c_void_p()


def save_params(path, params, blocks, hidden=64, game=GAME_CONNECT4):
    """flat parameters -> safetensors with tch VarStore names (VarStore::save)"""
    p = np.ascontiguousarray(params, np.float32)
    _check(lib().spai_params_save_safetensors(game, blocks, hidden, _p(p), len(p), os.fsencode(path)))


def load_params(path, blocks, hidden=64, game=GAME_CONNECT4, n=None):
    """safetensors with tch VarStore names -> flat parameters (VarStore::load).
    n: parameter count for the TicTacToe / chess nets (spai_ttt.num_params, spai_chess.num_params)"""
    out = np.zeros(num_params(blocks, hidden, game) if n is None else n, np.float32)
    _check(lib().spai_params_load_safetensors(game, blocks, hidden, os.fsencode(path), _p(out), len(out)))
    return out


class Replay:
    """replay ring (HeapRb, push_iter_overwrite / pop_iter().take(n))"""

    def __init__(self, capacity):
        self.h = C.c_void_p()
        _check(lib().spai_replay_create(capacity, C.byref(self.h)))

    def push(self, states, policies, values):
        s = np.ascontiguousarray(states, np.float32).reshape(-1, 126)
        p = np.ascontiguousarray(policies, np.float32).reshape(-1, 7)
        v = np.ascontiguousarray(values, np.float32).reshape(-1)
        _check(lib().spai_replay_push(self.h, len(v), _p(s), _p(p), _p(v)))

    def pop(self, n):
        s, p, v = np.zeros((n, 126), np.float32), np.zeros((n, 7), np.float32), np.zeros(n, np.float32)
        _check(lib().spai_replay_pop(self.h, n, _p(s), _p(p), _p(v)))
        return s, p, v

    def __len__(self):
        n = C.c_uint32()
        _check(lib().spai_replay_size(self.h, C.byref(n)))
        return n.value

    def close(self):
        if self.h:
            lib().spai_replay_destroy(self.h)
            self.h = C.c_void_p()


def choose_multiple(n, k, seed=0, stream=0):
    out = np.zeros(min(n, k), np.uint32)
    _check(lib().spai_choose_multiple(n, k, seed, stream, _p(out)))
    return out


def policy_normalize(p):
    """Policy::normalize (game/mod.rs:40) of a flat f32 policy; returns a new array"""
    a = np.array(p, np.float32, copy=True).ravel()
    _check(lib().spai_policy_normalize(_p(a), a.size))
    return a


def policy_best_action(p):
    """Policy::get_best_action: last index of the f32::total_cmp maximum"""
    a = np.ascontiguousarray(p, np.float32).ravel()
    out = C.c_uint32()
    _check(lib().spai_policy_best_action(_p(a), a.size, C.byref(out)))
    return out.value


def policy_sample(p, temperature, u01):
    """Policy::sample: WeightedIndex over p^temperature at the uniform draw u01 in [0, 1)"""
    a = np.ascontiguousarray(p, np.float32).ravel()
    out = C.c_uint32()
    _check(lib().spai_policy_sample(_p(a), a.size, temperature, u01, C.byref(out)))
    return out.value


def pipeline_run(init_params, selfplay_devices=(0,), learner_device=0, checkpoint_dir=None, events=None, **kw):
    """train_concurrent (main.rs:137-235) on the device; kw: PipelineConfig fields.
    events: a list that receives every ring event in ring order as a dict (kind,
    worker, batch, version, n, positions, ring_size, and copies of the samples)"""
    cfg = PipelineConfig()
    cfg.struct_size = C.sizeof(PipelineConfig)
    _check(lib().spai_pipeline_config_default(C.byref(cfg)))
    devs = (C.c_int * len(selfplay_devices))(*selfplay_devices)
    cfg.n_selfplay = len(selfplay_devices)
    cfg.selfplay_devices = devs
    cfg.learner_device = learner_device
    cfg.checkpoint_dir = os.fsencode(checkpoint_dir) if checkpoint_dir else None
    for k, v in kw.items():
        setattr(cfg, k, v)
    cb = None
    if events is not None:
        def on_event(_user, evp):
            ev = evp.contents
            n = int(ev.n)
            d = {k: int(getattr(ev, k)) for k in ("kind", "worker", "batch", "version", "n", "positions", "ring_size")}
            d["states"] = np.ctypeslib.as_array(ev.states, (n, 126)).copy() if n else np.zeros((0, 126), np.float32)
            d["policies"] = np.ctypeslib.as_array(ev.policies, (n, 7)).copy() if n else np.zeros((0, 7), np.float32)
            d["values"] = np.ctypeslib.as_array(ev.values, (n,)).copy() if n else np.zeros(0, np.float32)
            events.append(d)
        cb = OBSERVER(on_event)
        cfg.observer = C.cast(cb, C.c_void_p)
    p = np.ascontiguousarray(init_params, np.float32)
    st = PipelineStats()
    _check(lib().spai_pipeline_run(C.byref(cfg), _p(p), len(p), C.byref(st)))
    out = {k: getattr(st, k) for k, _ in PipelineStats._fields_ if k != "last_loss"}
    out["last_loss"] = list(st.last_loss)
    return out

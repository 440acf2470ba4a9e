"""TicTacToe (game/tictactoe.rs, model/tictactoe.rs; BASELINE config 1) on the
MI355X through the C ABI, checked against the CPU oracle (oracle/spai_oracle.c)
and the libtorch CPU golden.  Rules, search and self-play with the hash
evaluator: bit-exact.  Net (fp32 on the device): |dlogit| <= 1e-4 max(1,|l|max)."""
import ctypes as C
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def st():
    import spai_ttt
    return spai_ttt


def _bits(s):
    x = o = 0
    for r in range(3):
        for c in range(3):
            if s.st.board[r][c] == 1:
                x |= 1 << (r * 3 + c)
            elif s.st.board[r][c] == 2:
                o |= 1 << (r * 3 + c)
    return x, o


def test_ttt_rules_lockstep(oracle, st):
    rng = random.Random(3)
    n = 256
    games = [oracle.TTT() for _ in range(n)]
    eng = st.TTTEngine(num_searches=4, max_trees=1, eval_kind=st.EVAL_HASH)
    eng.games_resize(n)
    for ply in range(10):
        mask = eng.legal_mask(n)
        enc = eng.encode(n)
        rd = eng.games_read(n)
        acts = np.zeros(n, np.int32)
        for i, g in enumerate(games):
            empty = [r * 3 + c for r in range(3) for c in range(3) if g.st.board[r][c] == 0]
            legal = empty if g.status == 0 else []
            assert mask[i] == sum(1 << a for a in legal), (i, ply)
            x, o = _bits(g)
            assert (rd[i]["x"], rd[i]["o"], rd[i]["n"], rd[i]["status"]) == (x, o, g.st.num_actions_played, g.status)
            e = np.zeros(27, np.float32)
            oracle.lib().or_encode_states(oracle.GAME_TICTACTOE, 1, (C.c_void_p * 1)(C.addressof(g.st)),
                                          e.ctypes.data_as(C.POINTER(C.c_float)))
            assert np.array_equal(enc[i].ravel(), e), (i, ply)
            acts[i] = rng.choice(legal) if legal else 0
        rc = eng.apply(acts, check=False)
        for i, g in enumerate(games):
            if g.status == 0:
                assert rc[i] == 0
                games[i] = g.next_state(int(acts[i]))
            else:
                assert rc[i] == -3   # "Game has already ended"
    assert all(g.status != 0 for g in games)
    # illegal move: occupied cell
    eng.games_resize(1)
    eng.apply([4])
    assert list(eng.apply([4], check=False)) == [-2]
    # mask_invalid_actions: p * mask / ndarray sum, bit-exact
    pol = np.random.default_rng(0).random((1, 9)).astype(np.float32)
    m = eng.mask_invalid(pol)
    msk = pol[0] * np.array([0.0 if i == 4 else 1.0 for i in range(9)], np.float32)
    ref = msk / np.float32(oracle.lib().or_nd_sum(msk.ctypes.data_as(C.POINTER(C.c_float)), 9))
    assert np.array_equal(m[0], ref)
    eng.close()


def test_ttt_net_vs_torch_golden(st):
    g = np.load(os.path.join(GOLDEN, "net_ttt_2x64.npz"))
    blocks = int(g["meta"][0])
    eng = st.TTTEngine()
    net = st.TTTNet(eng, blocks, g["params"])
    lg, v = net.forward(g["x"])
    assert np.abs(lg - g["logits"]).max() <= 1e-4 * max(1.0, np.abs(g["logits"]).max())
    assert np.abs(v - g["value"]).max() <= 1e-5
    net.close()
    eng.close()


def test_ttt_predict_matches_forward_softmax_mask(oracle, st):
    # Model::predict over slots: encode -> forward -> softmax -> mask (fp32 device)
    rng = random.Random(4)
    n = 64
    eng = st.TTTEngine()
    eng.games_resize(n)
    for ply in range(rng.randrange(0, 4) + 2):
        mask = eng.legal_mask(n)
        acts = [rng.choice([a for a in range(9) if (m >> a) & 1]) if m else 0 for m in mask]
        eng.apply(acts, check=False)
    st_arr = eng.games_read(n)
    live = [i for i in range(n) if st_arr[i]["status"] == 0]
    net = st.TTTNet(eng, 2, st.init_params(2, 5))
    pr, v = net.predict(n)
    lg, vf = net.forward(eng.encode(n))
    assert np.array_equal(v, vf)
    mask = eng.legal_mask(n)
    for i in live:
        z = lg[i].astype(np.float64)
        sm = np.exp(z - z.max())
        sm /= sm.sum()
        m = sm * np.array([(mask[i] >> a) & 1 for a in range(9)])
        assert np.abs(pr[i] - m / m.sum()).max() <= 1e-6, i
        assert np.array_equal(pr[i] > 0, m > 0)
    net.close()
    eng.close()


def _oracle_search(oracle, n, sims):
    L = oracle.lib()
    trees = [L.or_tree_create(oracle.GAME_TICTACTOE) for _ in range(n)]
    arr = (C.c_void_p * n)(*trees)
    pol = np.zeros((n, 9), np.float32)
    ids = np.zeros((n, 9), np.int32)
    vis = np.zeros((n, 9), np.float32)
    nc = np.zeros(n, np.int32)
    rc = L.or_search(arr, n, sims, 2.0, oracle.EVAL_HASH, None, oracle.EVAL_FN(), None, oracle._f(pol),
                     oracle._i(ids), oracle._f(vis), oracle._i(nc))
    for t in trees:
        L.or_tree_destroy(t)
    return rc, pol, vis, nc


@pytest.mark.parametrize("sims", [1, 9, 64, 200])
def test_ttt_search_hash_matches_oracle(oracle, st, sims):
    eng = st.TTTEngine(num_searches=sims, max_trees=3, eval_kind=st.EVAL_HASH)
    eng.trees_create(3)
    pol, ids, vis, nc = eng.search(np.arange(3))
    rc, rpol, rvis, rnc = _oracle_search(oracle, 3, sims)
    assert rc >= 0
    assert np.array_equal(nc, rnc) and np.array_equal(vis, rvis)
    assert np.array_equal(pol, rpol, equal_nan=True)   # 1 sim: zero visits -> 0/0 = NaN, as the reference
    eng.close()


def test_ttt_self_play_hash_matches_oracle(oracle, st):
    n, sims, seed = 24, 32, 7
    eng = st.TTTEngine(num_searches=sims, max_trees=n, eval_kind=st.EVAL_HASH, seed=seed)
    games, stats = eng.self_play(n)
    ref = oracle.self_play(oracle.GAME_TICTACTOE, n, sims, seed, eval_kind=oracle.EVAL_HASH, max_plies=9)
    assert np.array_equal(np.concatenate([g["enc"] for g in games]), ref["enc"])
    assert np.array_equal(np.concatenate([g["policy"] for g in games]), ref["policy"])
    assert np.array_equal(np.concatenate([g["value"] for g in games]), ref["value"])
    for g in games:
        k = ref["n_moves"][g["game"]]
        assert np.array_equal(g["moves"], ref["moves"][g["game"], :k])
    assert stats["games"] == n and stats["sims"] == ref["sims"] and stats["evals"] == ref["evals"]
    eng.close()


@pytest.mark.parametrize("window", [5, 11])
def test_ttt_self_play_stream_matches_oracle_per_game(oracle, st, window):
    """spai_ttt_selfplay_stream: the 24 games through `window` tree slots; every
    game (positions, visit policies, signed values, moves) equals the oracle's
    lockstep game of the same id, only the finishing order differs"""
    n, sims, seed = 24, 32, 7
    eng = st.TTTEngine(num_searches=sims, max_trees=n, eval_kind=st.EVAL_HASH, seed=seed)
    games, stats = eng.self_play(n, window=window)
    ref = oracle.self_play(oracle.GAME_TICTACTOE, n, sims, seed, eval_kind=oracle.EVAL_HASH, max_plies=9)
    assert sorted(g["game"] for g in games) == list(range(n))
    for g in games:
        rows = np.nonzero(ref["game"] == g["game"])[0]
        k, m = int(rows[0]), len(rows)
        assert m == g["n"] and np.all(np.diff(rows) == 1)
        assert np.array_equal(g["enc"], ref["enc"][k:k + m])
        assert np.array_equal(g["policy"], ref["policy"][k:k + m])
        assert np.array_equal(g["value"], ref["value"][k:k + m])
        assert np.array_equal(g["moves"], ref["moves"][g["game"], :ref["n_moves"][g["game"]]])
    assert stats["games"] == n and stats["sims"] == ref["sims"] and stats["evals"] == ref["evals"]
    eng.close()


def test_ttt_config1_self_play_with_net(oracle, st):
    # BASELINE config 1: one game, 64 sims/move, random-init 2-block net
    eng = st.TTTEngine(num_searches=64, max_trees=1, eval_kind=st.EVAL_NET, seed=1)
    net = st.TTTNet(eng, 2, st.init_params(2, 0))
    eng.set_net(net)
    games, stats = eng.self_play(1)
    assert stats["games"] == 1 and len(games) == 1
    g = games[0]
    s = oracle.TTT()
    for a in g["moves"]:
        s = s.next_state(int(a))
    assert s.status != 0
    v = -1.0 if s.status == 2 else 0.0
    last_x = s.st.num_actions_played % 2 == 0
    exp = [v if ((i % 2 == 0) == last_x) else -v for i in range(g["n"])]
    assert np.array_equal(g["value"], np.array(exp, np.float32))
    assert np.allclose(g["policy"].sum(1), 1.0, atol=1e-6)
    eng.close()


def test_ttt_tree_reset_matches_oracle(oracle, st):
    """Tree::with_root_state from arbitrary positions, hash-stub search bit-exact vs the oracle"""
    rng = random.Random(8)
    roots = []
    for _ in range(12):
        g = oracle.TTT()
        for _ in range(rng.randrange(0, 6)):
            empty = [r * 3 + c for r in range(3) for c in range(3) if g.st.board[r][c] == 0]
            if g.status or not empty:
                break
            g = g.next_state(rng.choice(empty))
        if g.status == 0:
            roots.append(g)
    n, sims = len(roots), 40
    eng = st.TTTEngine(num_searches=sims, max_trees=n, eval_kind=st.EVAL_HASH)
    eng.trees_create(n)
    for i, g in enumerate(roots):
        x, o = _bits(g)
        rec = np.zeros(1, st.STATE_DTYPE)
        rec["x"], rec["o"], rec["n"], rec["status"] = x, o, g.st.num_actions_played, g.status
        eng.tree_reset(i, rec)
    pol, ids, vis, nc = eng.search(np.arange(n))
    L = oracle.lib()
    trees = [L.or_tree_with_root(oracle.GAME_TICTACTOE, C.byref(g.st)) for g in roots]
    arr = (C.c_void_p * n)(*trees)
    rpol = np.zeros((n, 9), np.float32)
    rids = np.zeros((n, 9), np.int32)
    rvis = np.zeros((n, 9), np.float32)
    rnc = np.zeros(n, np.int32)
    rc = L.or_search(arr, n, sims, 2.0, oracle.EVAL_HASH, None, oracle.EVAL_FN(), None, oracle._f(rpol),
                     oracle._i(rids), oracle._f(rvis), oracle._i(rnc))
    for t in trees:
        L.or_tree_destroy(t)
    assert rc >= 0
    assert np.array_equal(nc, rnc) and np.array_equal(vis, rvis) and np.array_equal(pol, rpol)
    bad = np.zeros(1, st.STATE_DTYPE)
    bad["x"], bad["o"] = 1, 1
    with pytest.raises(st.SpaiError):
        eng.tree_reset(0, bad)
    eng.close()

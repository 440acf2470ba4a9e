"""Pin the CPU oracle against the committed golden fixtures (CPU only).

The fixtures come from an independent pure-Python transliteration of the
reference (rules, MCTS, self-play) and from libtorch CPU for the net; see
tests/golden/gen_golden.py.  No reference outputs exist (no tests, not
buildable), so these pins are restatement-vs-restatement for rules/search and
libtorch-anchored for the net.
"""
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def rules_c4():
    return _load("rules_c4.json")


def test_nd_sum_order(oracle):
    # ndarray unrolled_fold: 9 elements sum as ((x0+x4)+(x1+x5)+(x2+x6)+(x3+x7))+x8
    x = np.array([1e8, 1, 1, 1, -1e8, 1, 1, 1, 1], np.float32)
    got = oracle.lib().or_nd_sum(oracle._f(x), 9)
    p = np.float32(0)
    for a, b in [(0, 4), (1, 5), (2, 6), (3, 7)]:
        p = np.float32(p + np.float32(x[a] + x[b]))
    assert got == np.float32(p + x[8])


def test_c4_rules_traces(oracle, rules_c4):
    rng = np.random.default_rng(0)
    for g in rules_c4["traces"]:
        s = oracle.C4()
        plies = g["plies"]
        for i, p in enumerate(plies):
            assert s.legal_mask() == p["legal"]
            assert s.status == p["status"] and s.n == p["n"] and s.current_player == p["cur"]
            x, o = s.bitboards()
            assert (str(x), str(o)) == (p["x"], p["o"])
            v, t = s.value_terminated()
            assert (v, t) == (p["value"], p["term"])
            enc = s.encoding()
            assert float(enc.ravel() @ np.arange(enc.size)) == p["enc_sum"]
            if i + 1 < len(plies):
                # find the move that produced the next ply from the bitboards
                nx = int(plies[i + 1]["x"]) | int(plies[i + 1]["o"])
                diff = nx ^ (x | o)
                col = (diff.bit_length() - 1) // 7
                s = s.next_state(col)


def test_c4_kats(oracle, rules_c4):
    for k in rules_c4["kats"]:
        s = oracle.C4()
        for a in k["moves"]:
            s = s.next_state(a)
        if "illegal" in k:
            with pytest.raises(ValueError):
                s.next_state(k["illegal"])
            assert s.legal_mask() == k["legal"]
        else:
            assert s.status == k["status"], k["name"]
            assert s.n == k["n"]
    # quirk Q1 explicitly: the anti-diagonal four stays Ongoing
    kat = [k for k in rules_c4["kats"] if k["name"] == "anti_diagonal_ignored"][0]
    assert kat["status"] == oracle.ONGOING


def test_c4_game_over_errors(oracle):
    s = oracle.C4()
    for a in [0, 1, 0, 1, 0, 1, 0]:
        s = s.next_state(a)
    assert s.status == oracle.WON and s.valid_actions() == []
    with pytest.raises(ValueError):
        s.next_state(2)


def test_c4_mask_invalid(oracle):
    s = oracle.C4()
    for a in [0] * 6:
        s = s.next_state(a)
    p = np.array([0.3, 0.1, 0.1, 0.1, 0.1, 0.1, 0.2], np.float32)
    m = s.mask_invalid(p)
    assert m[0] == 0.0
    mp = p * np.array([0, 1, 1, 1, 1, 1, 1], np.float32)
    ssum = np.float32(0)
    for v in mp:
        ssum = np.float32(ssum + v)
    np.testing.assert_array_equal(m, mp / ssum)
    with pytest.raises(ValueError):
        s.mask_invalid(np.ones(6, np.float32))


def test_ttt_traces(oracle):
    d = _load("rules_ttt.json")
    for g in d["traces"]:
        s = oracle.TTT()
        plies = g["plies"]
        for i, p in enumerate(plies):
            assert s.status == p["status"]
            if i + 1 < len(plies):
                nx = int(plies[i + 1]["x"]) | int(plies[i + 1]["o"])
                cur = int(p["x"]) | int(p["o"])
                a = (nx ^ cur).bit_length() - 1
                s = s.next_state(a)


def test_sampler_matches_python(oracle):
    # Philox uniform + weighted index vs the Python transliteration in gen_golden
    import importlib.util
    spec = importlib.util.spec_from_file_location("gg", os.path.join(GOLDEN, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    L = oracle.lib()
    for seed, gid, mv in [(0, 0, 0), (7, 3, 11), (2**40 + 5, 123456, 2**33 + 1)]:
        u = L.or_u01_f32(seed, gid, mv)
        assert u == gg.u01_f32(seed, gid, mv) and 0.0 <= u < 1.0
    vis = np.array([3, 0, 10, 1, 7], np.float32)
    for u in [0.0, 0.1, 0.5, 0.77, 0.99999994]:
        assert L.or_weighted_index(oracle._f(vis), 5, np.float32(1.25), u) == gg.weighted_index(vis, 1.25, u)
    # a zero-weight child is never drawn, whatever the uniform (rand's WeightedIndex)
    rng = np.random.default_rng(0)
    for _ in range(2000):
        u = float(np.float32(rng.random()))
        i = L.or_weighted_index(oracle._f(vis), 5, np.float32(1.25), u)
        assert vis[i] > 0 and i == gg.weighted_index(vis, 1.25, u)


def test_mcts_search_hash(oracle):
    d = _load("mcts_hash.json")
    assert d["search"], "fixture has no cases"
    for case in d["search"]:
        # rebuild the root from bitboards by replaying stones (order does not matter for the tree)
        x, o = int(case["x"]), int(case["o"])
        s = _c4_from_bitboards(oracle, x, o)
        assert s.n == case["n"]
        rc, pol, ids, vis, nc = oracle.search_c4([s], case["sims"])
        k = nc[0]
        assert [int(v) for v in vis[0, :k]] == case["visits"]
        exp = np.array(case["policy"], np.float32)
        np.testing.assert_array_equal(pol[0], exp)


def test_mcts_uniform_first_select(oracle):
    # ties go to the LAST child (mcts.rs:110-113) -> column 6
    d = _load("mcts_hash.json")
    assert d["uniform_first_select"] == 6
    rc, pol, ids, vis, nc = oracle.search_c4([oracle.C4()], 2, eval_kind=oracle.EVAL_UNIFORM)
    assert list(vis[0, :nc[0]]) == [0, 0, 0, 0, 0, 0, 1]


@pytest.mark.parametrize("game", ["c4", "ttt"])
def test_self_play_hash(oracle, game):
    d = _load("mcts_hash.json")["selfplay"][game]
    g = oracle.GAME_CONNECT4 if game == "c4" else oracle.GAME_TICTACTOE
    r = oracle.self_play(g, d["n_games"], d["sims"], d["seed"], eval_kind=oracle.EVAL_HASH)
    exp = d["samples"]
    assert len(r["value"]) == len(exp)
    for i, e in enumerate(exp):
        assert (int(r["game"][i]), int(r["ply"][i])) == (e["game"], e["ply"])
        assert float(r["value"][i]) == e["value"]
        np.testing.assert_array_equal(r["policy"][i], np.array(e["policy"], np.float32))
        assert float(r["enc"][i] @ np.arange(r["enc"].shape[1])) == e["enc_sum"]
    for gi, mv in enumerate(d["moves"]):
        assert list(r["moves"][gi, :r["n_moves"][gi]]) == mv


@pytest.mark.parametrize("name,game", [("net_c4_2x64.npz", 1), ("net_ttt_2x64.npz", 0)])
def test_net_forward_vs_libtorch(oracle, name, game):
    z = np.load(os.path.join(GOLDEN, name))
    blocks, hidden, seed = [int(v) for v in z["meta"]]
    p = oracle.init_params(game, blocks, hidden, seed)
    np.testing.assert_array_equal(p, z["params"])  # init restatement is bitwise
    net = oracle.Net(game, blocks, hidden, p)
    lg, v = net.forward(z["x"])
    # fp32 vs libtorch fp32 (different summation order): tight tolerance
    np.testing.assert_allclose(lg, z["logits"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(v, z["value"], rtol=1e-4, atol=1e-5)


def _c4_from_bitboards(oracle, x, o):
    st = oracle.C4State()
    oracle.lib().or_c4_init(oracle.C.byref(st))
    n = 0
    for col in range(7):
        for row in range(6):
            b = 1 << (col * 7 + row)
            if x & b:
                st.board[row][col] = oracle.X
                n += 1
            elif o & b:
                st.board[row][col] = oracle.O
                n += 1
    st.num_actions_played = n
    st.current_player = oracle.X if n % 2 == 0 else oracle.O
    return oracle.C4(st)


# ------------------------------------------------------------------ learner
def learner_masks(blocks, hidden, g_refs, rel=3e-3):
    """params whose Adam updates are well conditioned at every step given (|grad| above
    rel * max|grad|, ten times the gradient tolerance of the tests, so its sign is
    certain; far above fp32 noise and eps=1e-8) vs the rest.  Conv biases feeding a BatchNorm have a
    mathematically zero gradient (BN removes the batch mean): in fp32 it is rounding
    noise that Adam's g/(|g|+eps) turns into steps of up to lr, so those entries (and
    any entry whose gradient is that small at some step) are only bounded by lr."""
    import learner_ref as LR
    convs, lin, n = LR._layout(blocks, hidden)
    running = np.zeros(n, bool)
    for c in convs:
        running[c["mu"]:c["mu"] + c["co"]] = True
        running[c["var"]:c["var"] + c["co"]] = True
    well = ~running
    for g in g_refs:
        well &= np.abs(g) > rel * np.abs(g).max()
    return well, running


def check_learner_params(P, P_ref, g_refs, blocks, hidden, steps, lr=1e-3, tol=2e-5):
    """g_refs: reference gradients of every step, or of step 1 only (then, for steps > 1,
    the bound holds for 99.9 % of the step-1 well-conditioned entries)"""
    well, running = learner_masks(blocks, hidden, g_refs)
    # BN running stats: exact functions of the batch statistics at step 1; later steps
    # inherit the pre-BN bias noise (a bias shifts the batch mean one-for-one)
    np.testing.assert_allclose(P[running], P_ref[running], rtol=1e-4, atol=1e-5 if steps == 1 else lr * steps)
    err = np.abs(P[well] - P_ref[well])
    if len(g_refs) >= steps:
        assert err.max() <= tol * steps
    else:
        assert np.quantile(err, 0.999) <= tol * steps
    assert np.abs(P - P_ref).max() <= 2 * lr * steps + 1e-5                          # Adam step bound


def test_learner_oracle_vs_torch_golden(oracle):
    """numpy float64 train-step restatement vs PyTorch CPU fp32 (gen_golden.learner_golden)"""
    import learner_ref as LR
    z = np.load(os.path.join(GOLDEN, "learner_c4_1x64.npz"))
    blocks, hidden, seed, B, K = [int(v) for v in z["meta"]]
    p0 = oracle.init_params(oracle.GAME_CONNECT4, blocks, hidden, seed)
    batches = [(z["states"][k], z["policies"][k], z["values"][k]) for k in range(K)]
    P3, losses, grads = LR.train(p0, batches, blocks, hidden)
    np.testing.assert_allclose(losses, z["loss"], rtol=1e-5, atol=1e-6)
    g_ref = z["grads1"]
    assert np.abs(grads[0] - g_ref).max() <= 1e-5 * np.abs(g_ref).max()
    P1, _, _ = LR.train(p0, batches[:1], blocks, hidden)
    check_learner_params(P1, z["params1"], [g_ref], blocks, hidden, 1)
    check_learner_params(P3, z["params3"], [g_ref], blocks, hidden, 3, tol=1e-4)


def test_learner_oracle_dp_restatement(oracle):
    """the float64 DDP restatement (train_step_dp) that pins the world > 1 learner:
    one rank is train_step; two ranks holding the same batch are train_step on it
    (weights 1/2 + 1/2, running statistics the mean of equal values); unequal
    batches weight each rank's mean gradient by B_r / sum B"""
    import learner_ref as LR
    z = np.load(os.path.join(GOLDEN, "learner_c4_1x64.npz"))
    blocks, hidden, seed, B, K = [int(v) for v in z["meta"]]
    p0 = oracle.init_params(oracle.GAME_CONNECT4, blocks, hidden, seed)
    n = len(p0)
    b = (z["states"][0], z["policies"][0], z["values"][0])
    P1, m1, v1, l1, g1 = LR.train_step(p0, np.zeros(n), np.zeros(n), 0, *b, blocks, hidden)
    Pd, md, vd, ld, gd, _ = LR.train_step_dp(p0, np.zeros(n), np.zeros(n), 0, [b], blocks, hidden)
    np.testing.assert_array_equal(Pd, P1)
    np.testing.assert_array_equal(gd, g1)
    Pd, _, _, ld, gd, _ = LR.train_step_dp(p0, np.zeros(n), np.zeros(n), 0, [b, b], blocks, hidden)
    np.testing.assert_allclose(Pd, P1, rtol=0, atol=1e-12)
    np.testing.assert_allclose(gd, g1, rtol=0, atol=1e-12 * np.abs(g1).max())
    s_ = np.concatenate(list(z["states"]))
    p_ = np.concatenate(list(z["policies"]))
    v_ = np.concatenate(list(z["values"]))
    ra, rb = (s_[:12], p_[:12], v_[:12]), (s_[12:32], p_[12:32], v_[12:32])
    _, _, _, _, gd, parts = LR.train_step_dp(p0, np.zeros(n), np.zeros(n), 0, [ra, rb], blocks, hidden)
    _, ga, _ = LR.forward_backward(p0, *ra, blocks, hidden)
    _, gb, _ = LR.forward_backward(p0, *rb, blocks, hidden)
    np.testing.assert_allclose(gd, (12 * ga + 20 * gb) / 32, rtol=0, atol=1e-12 * np.abs(gd).max())


@pytest.mark.parametrize("fixture,k", [("mcts_f32net.npz", 6), ("mcts_f32net_6x64.npz", 1)])
def test_mcts_f32net_fixture(oracle, fixture, k):
    """tests/golden/mcts_f32net*.npz (search with the fp32 net, gen_f32net_golden.py)
    is reproducible by the oracle: the first k roots"""
    z = np.load(os.path.join(GOLDEN, fixture))
    blocks, seed, sims = int(z["blocks"]), int(z["seed"]), int(z["sims"])
    net = oracle.Net(oracle.GAME_CONNECT4, blocks, 64, oracle.init_params(oracle.GAME_CONNECT4, blocks, 64, seed))
    L = oracle.lib()
    roots = []
    for x, o, n in z["roots"][:k]:
        st = oracle.C4State()
        L.or_c4_init(oracle.C.byref(st))
        for col in range(7):
            for row in range(6):
                b = 1 << (col * 7 + row)
                if int(x) & b:
                    st.board[row][col] = oracle.X
                elif int(o) & b:
                    st.board[row][col] = oracle.O
        st.num_actions_played = int(n)
        st.current_player = oracle.X if int(n) % 2 == 0 else oracle.O
        roots.append(oracle.C4(st))
    rc, pol, ids, vis, nc = oracle.search_c4(roots, sims, eval_kind=oracle.EVAL_NET, net=net)
    assert rc >= 0
    np.testing.assert_array_equal(vis, z["visits"][:k])
    np.testing.assert_array_equal(pol, z["policy"][:k])


def test_learner_ref_mask_override_is_identity_with_own_masks():
    """learner_ref.train_step(masks=...) with the restatement's own (pre > 0) masks
    reproduces the plain step exactly (the GPU gradient test forces the device's
    masks through this path)"""
    import learner_ref as LR
    import oracle as O
    blocks, B = 1, 6
    rng = np.random.default_rng(0)
    p0 = O.init_params(O.GAME_CONNECT4, blocks, 64, 3)
    x = (rng.random((B, 126)) < 0.3).astype(np.float32)
    pi = rng.random((B, 7))
    pi /= pi.sum(1, keepdims=True)
    z = rng.choice([-1.0, 0.0, 1.0], B)
    n = len(p0)
    diag = {}
    P1, _, _, l1, g1 = LR.train_step(p0, np.zeros(n), np.zeros(n), 0, x, pi, z, blocks, 64, diag=diag)
    masks = [pre > 0 for pre in diag["pre"]]
    P2, _, _, l2, g2 = LR.train_step(p0, np.zeros(n), np.zeros(n), 0, x, pi, z, blocks, 64, masks=masks)
    np.testing.assert_array_equal(g1, g2)
    np.testing.assert_array_equal(P1, P2)
    np.testing.assert_array_equal(l1, l2)
    flipped = [m.copy() for m in masks]
    flipped[1].flat[0] = ~flipped[1].flat[0]          # one forced flip changes the gradient
    _, _, _, _, g3 = LR.train_step(p0, np.zeros(n), np.zeros(n), 0, x, pi, z, blocks, 64, masks=flipped)
    assert not np.array_equal(g1, g3)

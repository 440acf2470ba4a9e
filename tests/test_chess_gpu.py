"""Chess path on the MI355X through the C ABI, checked against the CPU oracle
(oracle/chess_oracle.c) and the PyTorch CPU net golden.

Bit-exact: ordered legal-move lists, statuses, repetition counts, encodings,
boards, mask_invalid_actions, search visit counts and whole self-play sample
streams with the deterministic hash evaluator.  Tolerance: the bf16 MFMA net
against fp32/fp64 references (stated per test)."""
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ch():
    import chessref
    chessref.lib()
    return chessref


@pytest.fixture(scope="module")
def sc():
    import spai_chess
    return spai_chess


def _abi_state(st):
    """oracle State (ctypes) -> spai_chess_state record"""
    import spai_chess
    a = np.zeros(1, spai_chess.STATE_DTYPE)
    b = st.b
    a["pieces"] = [b.pieces[i] for i in range(6)]
    a["colors"] = [b.color[0], b.color[1]]
    a["side"] = b.side
    a["castle"] = b.castle[0] | (b.castle[1] << 2)
    a["ep"] = b.ep
    a["fifty"] = st.fifty
    a["made"] = st.made
    return a[0]


FENS = [
    "r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1",
    "r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1",
    "rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8",
    "8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1",
    "4k3/8/8/3pP3/8/8/P7/4K3 w - d6 0 1",
]


def test_chess_rules_lockstep(ch, sc):
    rng = random.Random(11)
    games = []
    for g in range(40):
        games.append(ch.ChessState())
    for f in FENS:
        games.append(ch.ChessState(fen=f, made=0, fifty=0))
    n = len(games)
    eng = sc.ChessEngine(num_searches=4, max_trees=4, eval_kind=sc.EVAL_HASH, max_moves=1024)
    eng.games_resize(n)
    eng.games_write(np.array([_abi_state(s.st) for s in games], sc.STATE_DTYPE))
    # scripted knight shuffles in two games to reach threefold repetition
    script = {0: ["g1f3", "g8f6", "f3g1", "f6g8"] * 3}
    alive = [True] * n
    checked = 0
    for ply in range(400):
        mv, cnt = eng.legal_moves(n)
        st, reps, val, term = eng.status(n)
        enc = eng.encode(n)
        moves = np.zeros(n, np.uint16)
        for i, s in enumerate(games):
            ref = s.valid_actions()
            assert list(mv[i, :cnt[i]]) == ref, (i, ply)
            assert st[i] == s.status and reps[i] == s.repetitions(), (i, ply, st[i], reps[i])
            assert val[i] == s.value_terminated()[0]
            assert np.array_equal(enc[i], s.encoding()), (i, ply)
            checked += 1
            if s.status != 0:
                alive[i] = False
                moves[i] = ref[0] if ref else 1 | (2 << 6)
                continue
            sc_ = script.get(i)
            if sc_ and ply < len(sc_):
                m = sc_[ply]
                moves[i] = ch.move(ch.sq(m[:2]), ch.sq(m[2:4]))
            else:
                moves[i] = rng.choice(ref)
        rc = eng.apply(moves, check=False)
        for i, s in enumerate(games):
            if alive[i]:
                assert rc[i] == 0, (i, ply, rc[i])
                games[i] = s.next_state(int(moves[i]))
            else:
                assert rc[i] == -3   # "Game is already over"
        if not any(alive):
            break
        # boards identical
        if ply % 25 == 0:
            rd = eng.games_read(n)
            for i, s in enumerate(games):
                ref = _abi_state(s.st)
                assert np.array_equal(rd[i]["pieces"], ref["pieces"]) and rd[i]["side"] == ref["side"]
                assert rd[i]["castle"] == ref["castle"] and rd[i]["ep"] == ref["ep"]
                assert rd[i]["fifty"] == ref["fifty"] and rd[i]["made"] == ref["made"]
    assert checked > 5000
    assert not alive[0] and games[0].status == 1   # the shuffle ended in a threefold draw
    ch.arena_reset()
    eng.close()


def test_chess_apply_errors(ch, sc):
    eng = sc.ChessEngine(num_searches=4, max_trees=4, eval_kind=sc.EVAL_HASH)
    eng.games_resize(2)
    before = eng.games_read(2)
    rc = eng.apply(np.array([ch.move(ch.sq("e2"), ch.sq("e5")), ch.move(ch.sq("e2"), ch.sq("e4"))], np.uint16),
                   check=False)
    assert list(rc) == [-2, 0]   # "Failed to make move" leaves the slot unchanged
    after = eng.games_read(2)
    assert after[0].tobytes() == before[0].tobytes()
    with pytest.raises(sc.SpaiError):
        eng.mask_invalid(np.ones((1, 7), np.float32))
    eng.close()


def test_chess_mask_invalid_bit_exact(ch, sc):
    rng = random.Random(5)
    states = []
    for g in range(24):
        s = ch.ChessState()
        for _ in range(rng.randrange(0, 80)):
            mv = s.valid_actions()
            if not mv or s.status:
                break
            s = s.next_state(rng.choice(mv))
        states.append(s)
    eng = sc.ChessEngine(num_searches=4, max_trees=4, eval_kind=sc.EVAL_HASH)
    eng.games_resize(len(states))
    eng.games_write(np.array([_abi_state(s.st) for s in states], sc.STATE_DTYPE))
    pol = np.random.default_rng(2).random((len(states), 4672)).astype(np.float32)
    got = eng.mask_invalid(pol)
    for i, s in enumerate(states):
        assert np.array_equal(got[i], s.mask_invalid(pol[i])), i
    ch.arena_reset()
    eng.close()


def test_chess_predict_matches_forward_softmax_mask(ch, sc):
    # Model::predict (model/mod.rs:36-98) on the device = encode -> forward ->
    # softmax -> mask_invalid_actions; checked against the same device forward
    # on the device encoding, softmax in fp64 and the oracle's mask: |dp| <= 1e-6,
    # support == the legal moves exactly, values bit-identical to forward.
    rng = random.Random(9)
    states = []
    for g in range(20):
        s = ch.ChessState()
        for _ in range(rng.randrange(0, 60)):
            mv = s.valid_actions()
            if not mv or s.status:
                break
            s = s.next_state(rng.choice(mv))
        if not s.status:
            states.append(s)
    eng = sc.ChessEngine(num_searches=4, max_trees=4)
    eng.games_resize(len(states) + 2)
    eng.games_write(np.array([_abi_state(s.st) for s in states], sc.STATE_DTYPE), first=2)
    net = sc.ChessNet(eng, 2, sc.init_params(2, 3))
    pr, v = net.predict(len(states), first=2)
    x = eng.encode(len(states), first=2)
    lg, vf = net.forward(x)
    assert np.array_equal(v, vf)
    for i, s in enumerate(states):
        z = lg[i].astype(np.float64)
        sm = np.exp(z - z.max())
        sm = (sm / sm.sum()).astype(np.float32)
        ref = s.mask_invalid(sm)
        assert np.abs(pr[i] - ref).max() <= 1e-6, i
        legal = s.mask_invalid(np.ones(4672, np.float32)) > 0
        assert np.array_equal(pr[i] > 0, legal), i
        assert abs(float(pr[i].sum(dtype=np.float64)) - 1.0) <= 1e-5
    pr0, _ = net.predict(1)   # slot 0: the start position
    assert (pr0[0] > 0).sum() == 20
    with pytest.raises(sc.SpaiError):
        net.predict(len(states) + 3)
    ch.arena_reset()
    net.close()
    eng.close()


def test_chess_net_vs_torch_golden(ch, sc):
    g = np.load(os.path.join(GOLDEN, "chess_net_b1.npz"))
    blocks = int(g["blocks"])
    eng = sc.ChessEngine(num_searches=4, max_trees=8)
    net = sc.ChessNet(eng, blocks, sc.init_params(blocks, int(g["seed"])))
    lg, v = net.forward(g["x"])
    ref_l, ref_v = g["logits"], g["value"]
    # bf16 weights/activations, fp32 accumulate: |dlogit| <= 3e-2 * max(1, |logit|max), |dv| <= 2e-2
    assert np.abs(lg - ref_l).max() <= 3e-2 * max(1.0, np.abs(ref_l).max()), np.abs(lg - ref_l).max()
    assert np.abs(v - ref_v).max() <= 2e-2, (v, ref_v)
    # an odd batch and a single position give the same rows (batch-composition independence)
    lg1, v1 = net.forward(g["x"][3:4])
    assert np.array_equal(lg1[0], lg[3]) and v1[0] == v[3]
    net.close()
    eng.close()


def test_chess_net_positions_per_workgroup_invariance(ch, sc):
    # > #CUs positions run 2 per workgroup, <= #CUs run 1 per workgroup: a
    # position's logits and value must not depend on which
    rng = np.random.default_rng(4)
    x = (rng.random((300, 19, 8, 8)) < 0.2).astype(np.float32)
    eng = sc.ChessEngine(num_searches=4, max_trees=8)
    net = sc.ChessNet(eng, 2, sc.init_params(2, 1))
    lg2, v2 = net.forward(x)
    lg1, v1 = net.forward(x[:37])
    assert np.array_equal(lg1, lg2[:37]) and np.array_equal(v1, v2[:37])
    lg3, v3 = net.forward(x[250:300])
    assert np.array_equal(lg3, lg2[250:300]) and np.array_equal(v3, v2[250:300])
    net.close()
    eng.close()


def test_chess_net_work_split_invariance(ch, sc):
    """more positions than CUs: m = ceil(count / #CUs) positions on the busiest
    CU; even m runs P = 2 passes, odd m an even split as P = 2 passes plus one
    P = 1 pass (k_chess_forward).  Every count must give the one-position-per-
    workgroup results bit for bit."""
    rng = np.random.default_rng(5)
    x = (rng.random((1300, 19, 8, 8)) < 0.2).astype(np.float32)
    eng = sc.ChessEngine(num_searches=4, max_trees=8)
    net = sc.ChessNet(eng, 2, sc.init_params(2, 3))
    ref_l, ref_v = zip(*(net.forward(x[i:i + 200]) for i in range(0, 1300, 200)))   # <= #CUs: P = 1
    ref_l, ref_v = np.concatenate(ref_l), np.concatenate(ref_v)
    for n in (600, 700, 1000, 1100, 1300):   # m = 3, 3, 4, 5, 6 on 256 CUs
        lg, v = net.forward(x[:n])
        assert np.array_equal(lg, ref_l[:n]) and np.array_equal(v, ref_v[:n]), n
    net.close()
    eng.close()


def test_chess_net_20_blocks_vs_fp64(ch, sc):
    rng = random.Random(9)
    xs = []
    for _ in range(3):
        s = ch.ChessState()
        for _ in range(rng.randrange(0, 40)):
            mv = s.valid_actions()
            if not mv or s.status:
                break
            s = s.next_state(rng.choice(mv))
        xs.append(s.encoding())
    x = np.stack(xs)
    eng = sc.ChessEngine(num_searches=4, max_trees=8)
    p = sc.init_params(20, 3)
    net = sc.ChessNet(eng, 20, p)
    lg, v = net.forward(x)
    ref_l, ref_v = ch.net_forward(p, 20, x)
    scale = max(1.0, np.abs(ref_l).max())
    # 41 bf16 layers: |dlogit| <= 5e-2 * max(1, |logit|max); values within 5e-2
    assert np.abs(lg - ref_l).max() <= 5e-2 * scale, (np.abs(lg - ref_l).max(), scale)
    assert np.abs(v - ref_v).max() <= 5e-2, (v, ref_v)
    net.close()
    eng.close()
    ch.arena_reset()


@pytest.mark.parametrize("n_trees,sims", [(1, 64), (9, 40)])
def test_chess_search_hash_matches_oracle(ch, sc, n_trees, sims):
    eng = sc.ChessEngine(num_searches=sims, max_trees=n_trees, eval_kind=sc.EVAL_HASH)
    eng.trees_create(n_trees)
    pol, ids, vis, mv, nc = eng.search(np.arange(n_trees))
    rc, rpol, rids, rvis, rmv, rnc = ch.search(n_trees, sims)
    assert rc >= 0
    assert np.array_equal(nc, rnc)
    for i in range(n_trees):
        k = nc[i]
        assert np.array_equal(vis[i, :k], rvis[i, :k]), i
        assert np.array_equal(mv[i, :k], rmv[i, :k].astype(np.uint16)), i
    assert np.array_equal(pol, rpol)
    ch.arena_reset()
    eng.close()


def test_chess_self_play_hash_matches_oracle(ch, sc):
    n, sims, seed = 6, 8, 21
    eng = sc.ChessEngine(num_searches=sims, max_trees=n, eval_kind=sc.EVAL_HASH, seed=seed, max_moves=2048)
    games, stats = eng.self_play(n)
    ref = ch.self_play(n, sims, seed=seed, max_plies=2048, with_policy=True)
    got_enc = np.concatenate([g["enc"] for g in games])
    got_pol = np.concatenate([g["policy"] for g in games])
    got_val = np.concatenate([g["value"] for g in games])
    got_gid = np.concatenate([np.full(g["n"], g["game"]) for g in games])
    assert np.array_equal(got_gid, ref["game"])
    assert np.array_equal(got_val, ref["value"])
    assert np.array_equal(got_enc, ref["enc"])
    assert np.array_equal(got_pol, ref["policy"])
    for g in games:
        nm = ref["n_moves"][g["game"]]
        assert np.array_equal(g["moves"], ref["moves"][g["game"], :nm].astype(np.uint16))
    assert stats["games"] == n and stats["sims"] == ref["sims"] and stats["evals"] == ref["evals"]
    ch.arena_reset()
    eng.close()


@pytest.mark.parametrize("window", [2, 4])
def test_chess_self_play_stream_matches_oracle_per_game(ch, sc, window):
    """spai_chess_selfplay_stream: the 6 games through `window` tree slots, a slot
    taking the next game (a fresh start-position tree) when its game ends.  Every
    game -- positions, visit policies, signed values, moves -- equals the oracle's
    lockstep game of the same id; only the order in which games finish differs"""
    n, sims, seed = 6, 8, 21
    eng = sc.ChessEngine(num_searches=sims, max_trees=n, eval_kind=sc.EVAL_HASH, seed=seed, max_moves=2048)
    games, stats = eng.self_play(n, game_id_base=0, window=window)
    ref = ch.self_play(n, sims, seed=seed, max_plies=2048, with_policy=True)
    assert sorted(g["game"] for g in games) == list(range(n))
    for g in games:
        rows = np.nonzero(ref["game"] == g["game"])[0]
        assert len(rows) == g["n"] and np.all(np.diff(rows) == 1)
        k, m = rows[0], g["n"]
        assert np.array_equal(g["value"], ref["value"][k:k + m])
        assert np.array_equal(g["enc"], ref["enc"][k:k + m])
        assert np.array_equal(g["policy"], ref["policy"][k:k + m])
        assert np.array_equal(g["moves"], ref["moves"][g["game"], :ref["n_moves"][g["game"]]].astype(np.uint16))
    assert stats["games"] == n and stats["sims"] == ref["sims"] and stats["evals"] == ref["evals"]
    ch.arena_reset()
    eng.close()


def test_chess_self_play_net_legal(ch, sc):
    n = 4
    eng = sc.ChessEngine(num_searches=6, max_trees=n, eval_kind=sc.EVAL_NET, seed=2, max_moves=2048)
    net = sc.ChessNet(eng, 1, sc.init_params(1, 4))
    eng.set_net(net)
    games, stats = eng.self_play(n)
    assert stats["games"] == n and len(games) == n
    for g in games:
        s = ch.ChessState()
        for m in g["moves"]:
            assert int(m) in s.valid_actions()
            s = s.next_state(int(m))
        v, term = s.value_terminated()
        assert term
        final_side = s.side
        exp = np.array([v if (0 if i % 2 == 0 else 1) == final_side else -v for i in range(g["n"])], np.float32)
        assert np.array_equal(g["value"], exp)
        assert np.allclose(g["policy"].sum(1), 1.0, atol=1e-5)
    ch.arena_reset()
    eng.close()


def test_chess_tree_reset_from_slot_matches_oracle(ch, sc):
    """Tree::with_root_state from game slots: random games and a knight shuffle
    whose root has already occurred once (the search meets threefold repetition
    through the copied history); visit counts bit-exact vs the oracle (hash stub)."""
    rng = random.Random(17)
    shuffle = [ch.move(ch.sq(a), ch.sq(b)) for a, b in
               [("g1", "f3"), ("g8", "f6"), ("f3", "g1"), ("f6", "g8"), ("g1", "f3"), ("g8", "f6")]]
    seqs = [shuffle]
    for g in range(5):
        s, seq = ch.ChessState(), []
        for _ in range(rng.randrange(1, 40)):
            mv = s.valid_actions()
            if not mv or s.status:
                break
            m = rng.choice(mv)
            seq.append(m)
            s = s.next_state(m)
        seqs.append(seq)
    n, sims = len(seqs), 48
    states = []
    eng = sc.ChessEngine(num_searches=sims, max_trees=n, eval_kind=sc.EVAL_HASH)
    eng.games_resize(n)
    for p in range(max(len(q) for q in seqs)):
        eng.apply(np.array([q[p] if p < len(q) else 0 for q in seqs], np.uint16), check=False)
    for q in seqs:
        s = ch.ChessState()
        for m in q:
            s = s.next_state(m)
        states.append(s)
    live = [i for i, s in enumerate(states) if not s.status]
    eng.trees_create(n)
    for t, i in enumerate(live):
        eng.tree_reset(t, i)
    pol, ids, vis, mv, nc = eng.search(np.arange(len(live)))
    rc, rpol, rids, rvis, rmv, rnc = ch.search(0, sims, states=[states[i] for i in live])
    assert rc >= 0
    assert np.array_equal(nc, rnc)
    for t in range(len(live)):
        k = nc[t]
        assert np.array_equal(vis[t, :k], rvis[t, :k]), t
        assert np.array_equal(mv[t, :k], rmv[t, :k].astype(np.uint16)), t
    assert np.array_equal(pol, rpol)
    with pytest.raises(sc.SpaiError):
        eng.tree_reset(0, n)          # slot out of range
    ch.arena_reset()
    eng.close()


def test_device_perft_public_counts(ch, sc):
    """the device move generator and make-move (wave_movegen / apply_move, the code
    the search runs) against the public perft counts (chessprogramming.org): the
    start position to depth 6 (119,060,324), Kiwipete to 5 (193,690,690) and
    positions 3-6 to depth 5-6 -- breadth-first on the device, every ply's
    positions in HBM (spai_chess_perft)"""
    from test_chess_oracle import PERFT
    eng = sc.ChessEngine(num_searches=4, max_trees=4, eval_kind=sc.EVAL_HASH, max_moves=64)
    eng.games_resize(len(PERFT))
    eng.games_write(np.array([_abi_state(ch.ChessState(fen=f, made=0, fifty=0).st) for f, _ in PERFT],
                             sc.STATE_DTYPE))
    for i, (fen, counts) in enumerate(PERFT):
        assert eng.perft(len(counts), slot=i) == counts, fen
    with pytest.raises(sc.SpaiError):
        eng.perft(9)
    eng.close()

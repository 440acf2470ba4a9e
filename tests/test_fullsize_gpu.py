"""BASELINE configs at full size on the GPU, checked through size-independent
properties against the CPU oracle's rules (the oracle is far too slow to
replay 4096 searches at 800 sims with a 6x64 net; the bit-exact search and
self-play checks are in test_gpu_parity.py / test_gpu_fp32.py at smaller
sizes).

* C2: one self_play step = 4096 Connect4 games x 800 sims/move with the
  6x64 bf16 net (bench.py's step): every game replays legally in the oracle to
  its recorded outcome, values are signed per player to move
  (learner_concurrent.rs:211-225), visit policies are normalised, zero on
  illegal columns and nonzero on the played move (sampled from N^1.25,
  learner_concurrent.rs:189-193), and the counters add up:
  sims = 800 x positions (every active tree searches every move).
* C4c: chess, 1024 trees x 400 sims for two moves with the 20x256 bf16 net:
  root children in the crate's legal-move order (oracle movegen), visits sum
  to N(root) - 1, and the second search re-rooted by use_subtree keeps N.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spai():
    import spai as s
    s.lib()
    return s


def test_c2_full_step_properties(spai, oracle):
    G, sims = 4096, 800
    e = spai.Engine(num_searches=sims, max_trees=G, eval_kind=spai.EVAL_NET, seed=0)
    net = spai.Net(e, 6, spai.init_params(6, 64, seed=0))
    e.set_net(net)
    games, st = e.self_play(G)
    assert st["games"] == G and sorted(g["game"] for g in games) == list(range(G))
    plies = sum(len(g["moves"]) for g in games)
    assert st["positions"] == plies
    assert st["sims"] == sims * plies
    assert 0 < st["evals"] <= st["sims"]
    assert st["moves"] == max(len(g["moves"]) for g in games) <= 42
    for k, g in enumerate(games):
        s = oracle.C4()
        m = len(g["moves"])
        for j, a in enumerate(g["moves"]):
            p = g["policy"][j]
            legal = np.zeros(7, bool)
            legal[s.valid_actions()] = True
            assert abs(float(p.sum()) - 1.0) < 1e-5, (g["game"], j)
            assert np.all(p[~legal] == 0.0) and p[a] > 0.0, (g["game"], j, p, a)
            if k % 16 == 0:
                np.testing.assert_array_equal(g["enc"][j], s.encoding().ravel())
            s = s.next_state(int(a))
            assert (s.status != 0) == (j == m - 1), (g["game"], j)
        last = 1.0 if s.status == 2 else 0.0   # Won: the last mover won
        exp = np.array([last if (m - 1 - i) % 2 == 0 else -last for i in range(m)], np.float32)
        np.testing.assert_array_equal(g["value"], exp)
    net.close()
    e.close()


def test_c2_full_stream_equals_lockstep_per_game(spai):
    """C2 at full size, the bench's streamed schedule against the lockstep one: 4096
    games x 800 sims with the 6x64 bf16 net, once as one lockstep batch and once
    through 2048 tree slots (a slot taking the next game when its game ends, so
    the leaf batches, group sizes and chain splits all differ).  The forward does
    not depend on its batch, and each game's draws are keyed by its id and its own
    move number, so every game -- moves, visit policies, signed values, encodings
    -- is bit-identical between the two schedules"""
    G, sims = 4096, 800
    e = spai.Engine(num_searches=sims, max_trees=G, eval_kind=spai.EVAL_NET, seed=0)
    net = spai.Net(e, 6, spai.init_params(6, 64, seed=0))
    e.set_net(net)
    lock, st_l = e.self_play(G, game_id_base=7 * G)
    strm, st_s = e.self_play(G, game_id_base=7 * G, window=G // 2)
    for k in ("sims", "evals", "games", "positions"):
        assert st_l[k] == st_s[k], (k, st_l, st_s)
    by_id = {g["game"]: g for g in lock}
    assert sorted(by_id) == sorted(g["game"] for g in strm) == list(range(7 * G, 8 * G))
    for g in strm:
        r = by_id[g["game"]]
        assert list(g["moves"]) == list(r["moves"]), g["game"]
        np.testing.assert_array_equal(g["policy"], r["policy"])
        np.testing.assert_array_equal(g["value"], r["value"])
        np.testing.assert_array_equal(g["enc"], r["enc"])
    net.close()
    e.close()


def test_c4c_chess_two_moves_1024_trees(spai):
    import chessref
    import spai_chess as sc
    n, sims = 1024, 400
    eng = sc.ChessEngine(num_searches=sims, max_trees=n, eval_kind=sc.EVAL_NET, seed=0)
    net = sc.ChessNet(eng, 20, sc.init_params(20, 0))
    eng.set_net(net)
    eng.trees_create(n)
    start = chessref.ChessState()
    roots = [start] * n
    prev_n = np.zeros(n, np.int64)
    for mv_no in range(2):
        pol, ids, vis, mv, nc = eng.search(np.arange(n))
        pick = np.zeros(n, np.uint32)
        for i in range(n):
            k = int(nc[i])
            want = roots[i].valid_actions()
            assert [int(m) for m in mv[i, :k]] == [int(m) for m in want], (mv_no, i)
            _, root_n, _ = eng.tree_root(i) if i < 8 else (None, None, None)
            total = int(vis[i, :k].sum())
            # fresh root: the first iteration expands it, the other sims - 1 descend
            # into a child; a re-rooted tree keeps its N (quirk Q4)
            assert total == prev_n[i] + sims - 1, (mv_no, i, total)
            if root_n is not None:
                assert root_n == total + 1
            assert abs(float(pol[i].sum()) - 1.0) < 1e-5
            j = int(np.flatnonzero(vis[i, :k] == vis[i, :k].max())[-1])
            pick[i] = j
            prev_n[i] = int(vis[i, j])
            roots[i] = roots[i].next_state(int(mv[i, j]))
        if mv_no == 0:
            eng.advance(np.arange(n), pick)
    net.close()
    eng.close()

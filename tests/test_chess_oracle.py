"""CPU checks of the chess oracle (oracle/chess_oracle.c, oracle/chessref.py)
and the host-only chess entry points of the C ABI.

Pinning: move generation by public perft known answers (the `chess` crate 3.2.0
that the reference wraps is not vendored and cannot be run here); the adapter
rules (game/chess.rs) by hand-derived known answers; the net restatement by
PyTorch CPU goldens (tests/golden/gen_chess_golden.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def ch():
    import chessref
    chessref.lib()
    return chessref


# (fen, [perft(1), perft(2), ...]) -- chessprogramming.org perft results: the start
# position to depth 6, Kiwipete and positions 3-6 to depth 5-6 (each run < 2 s in C)
PERFT = [
    ("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", [20, 400, 8902, 197281, 4865609, 119060324]),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", [48, 2039, 97862, 4085603, 193690690]),
    ("8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", [14, 191, 2812, 43238, 674624, 11030083]),
    ("r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", [6, 264, 9467, 422333, 15833292]),
    ("rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", [44, 1486, 62379, 2103487, 89941194]),
    ("r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10", [46, 2079, 89890, 3894594,
                                                                                   164075551]),
]


@pytest.mark.parametrize("fen,counts", PERFT)
def test_perft_known_answers(ch, fen, counts):
    b = ch.board_from_fen(fen)
    assert [ch.perft(b, d) for d in range(1, len(counts) + 1)] == counts


def test_movegen_enumeration_order(ch):
    # chess 3.2.0 MoveGen: pawns (sources ascending, destinations ascending), knights, ..., king
    b = ch.board_from_fen(ch.START_FEN)
    got = [ch.uci(m) for m in ch.legal_moves(b)]
    assert got == ["a2a3", "a2a4", "b2b3", "b2b4", "c2c3", "c2c4", "d2d3", "d2d4", "e2e3", "e2e4", "f2f3", "f2f4",
                   "g2g3", "g2g4", "h2h3", "h2h4", "b1a3", "b1c3", "g1f3", "g1h3"]
    # promotions expand Q, N, R, B; pinned pieces come after unpinned ones of their type;
    # castling destinations sit in the king's ascending destination set
    b = ch.board_from_fen("r3k2r/1P6/8/8/8/8/8/R3K2R w KQkq - 0 1")
    got = [ch.uci(m) for m in ch.legal_moves(b)]
    assert got[:8] == ["b7a8q", "b7a8n", "b7a8r", "b7a8b", "b7b8q", "b7b8n", "b7b8r", "b7b8b"]
    king = [m for m in got if m.startswith("e1")]
    assert king == ["e1c1", "e1d1", "e1f1", "e1g1", "e1d2", "e1e2", "e1f2"]
    b = ch.board_from_fen("4k3/8/8/8/1b6/8/3N4/4K1N1 w - - 0 1")   # Nd2 pinned by Bb4
    got = [ch.uci(m) for m in ch.legal_moves(b)]
    assert not any(m.startswith("d2") for m in got)
    # en passant entries follow every other pawn entry
    b = ch.board_from_fen("4k3/8/8/3pP3/8/8/P7/4K3 w - d6 0 1")
    got = [ch.uci(m) for m in ch.legal_moves(b)]
    assert got[:5] == ["a2a3", "a2a4", "e5e6", "e5d6", "e1d1"]


def test_checkmate_is_won_plus_one(ch):
    # fool's mate; chess.rs:168-174 gives Won -> (+1, true) (quirk Q7; C4/TTT give -1)
    s = ch.ChessState()
    for m in ["f2f3", "e7e5", "g2g4", "d8h4"]:
        s = s.next_state(ch.move(ch.sq(m[:2]), ch.sq(m[2:4])))
    assert s.valid_actions() == []
    assert s.status == 2
    assert s.value_terminated() == (1.0, True)
    with pytest.raises(ValueError):   # "Game is already over"
        s.next_state(ch.move(ch.sq("e2"), ch.sq("e4")))


def test_repetition_by_move_lists(ch):
    s = ch.ChessState()
    seq = ["g1f3", "g8f6", "f3g1", "f6g8"] * 2
    reps = [s.repetitions()]
    for m in seq:
        s = s.next_state(ch.move(ch.sq(m[:2]), ch.sq(m[2:4])))
        reps.append(s.repetitions())
    # the start position's move list recurs at plies 4 and 8 -> 2, then 3 = threefold (Tied)
    assert reps == [1, 1, 1, 1, 2, 2, 2, 2, 3]
    assert s.status == 1 and s.value_terminated() == (0.0, True)
    enc = s.encoding()
    assert np.all(enc[16] == 3.0)


def test_fifty_move_counter(ch):
    s = ch.ChessState(fen="4k3/8/8/8/8/8/8/R3K3 w Q - 0 1", made=10, fifty=98)
    s1 = s.next_state(ch.move(ch.sq("a1"), ch.sq("a2")))   # rook leaves a1: castle right lost -> reset
    assert s1.st.fifty == 0
    s2 = s.next_state(ch.move(ch.sq("e1"), ch.sq("e2")))   # king move: rights lost -> reset
    assert s2.st.fifty == 0
    t = ch.ChessState(fen="4k3/8/8/8/8/8/8/R3K3 w - - 0 1", made=10, fifty=99)
    t1 = t.next_state(ch.move(ch.sq("a1"), ch.sq("a5")))
    assert t1.st.fifty == 100 and t1.status == 1
    e = t1.encoding()
    assert np.all(e[17] == np.float32(100) / np.float32(100.0)) and np.all(e[18] == np.float32(11 // 2) / 50.0)


def test_encoding_black_view_flips_ranks(ch):
    s = ch.ChessState().next_state(ch.move(ch.sq("e2"), ch.sq("e4")))
    e = s.encoding()
    # black to move: row 0 = rank 8; black pawns (own, plane 0) on rank 7 -> row 1
    assert e[0, 1].sum() == 8 and e[6, 4, 4] == 1.0   # white pawn e4 -> row 7-3 = 4, col 4
    assert np.all(e[12:16] == 1.0)                     # all castling rights
    assert np.all(e[18] == 0.0)                        # 1 MakeMove // 2 = 0


def test_channels_and_get_action_bug(ch):
    W, B = ch.WHITE, ch.BLACK
    e2e4 = ch.move(ch.sq("e2"), ch.sq("e4"))
    assert ch.get_channel(W, e2e4) == 23 + 7 + 2 - 1                   # vertical, 2 forward
    assert ch.policy_index(W, e2e4) == (23 + 8) * 64 + 1 * 8 + 4
    e7e5 = ch.move(ch.sq("e7"), ch.sq("e5"))
    assert ch.policy_index(B, e7e5) == ch.policy_index(W, e2e4)        # mirrored for Black
    g1f3 = ch.move(ch.sq("g1"), ch.sq("f3"))
    assert ch.get_channel(W, g1f3) == 65                               # knight NW, |rank| > |file|
    b7a8n = ch.move(ch.sq("b7"), ch.sq("a8"), ch.KNIGHT)
    assert ch.get_channel(W, b7a8n) == 6 + 0
    # get_action round trip holds except for knight underpromotions (chess.rs:442 bug)
    for idx in [ch.policy_index(W, e2e4), ch.policy_index(W, g1f3)]:
        assert ch.get_action(W, idx) in (e2e4, g1f3)
    bad = ch.get_action(W, ch.policy_index(W, b7a8n))
    assert bad != b7a8n and (bad >> 12) == ch.KNIGHT and ((bad >> 6) & 7) == (1 + 6 - 4) % 8


def test_mask_invalid_renormalizes(ch):
    s = ch.ChessState()
    p = np.random.default_rng(0).random(ch.POLICY).astype(np.float32)
    out = s.mask_invalid(p)
    idx = sorted(ch.policy_index(0, m) for m in s.valid_actions())
    assert np.count_nonzero(out) == 20 and sorted(np.flatnonzero(out).tolist()) == idx
    assert abs(out.sum() - 1.0) < 1e-6
    with pytest.raises(ValueError):
        s.mask_invalid(np.ones(7, np.float32))


def test_search_and_self_play_with_hash_stub(ch):
    rc, pol, ids, vis, mv, nc = ch.search(2, 64)
    assert rc >= 0 and list(nc) == [20, 20] and vis[0].sum() == 63.0
    assert np.isclose(pol[0].sum(), 1.0)
    r = ch.self_play(2, 8, seed=3, max_plies=2048, with_policy=False)
    assert len(r["value"]) == int(r["n_moves"].sum())
    ch.arena_reset()


def test_net_restatement_vs_torch_golden(ch):
    import spai_chess
    g = np.load(os.path.join(GOLDEN, "chess_net_b1.npz"))
    p = spai_chess.init_params(int(g["blocks"]), int(g["seed"]))
    lg, v = ch.net_forward(p, int(g["blocks"]), g["x"])
    assert np.abs(lg - g["logits"]).max() < 1e-4 * max(1.0, np.abs(g["logits"]).max())
    assert np.abs(v - g["value"]).max() < 1e-5


def test_capi_move_index_matches_oracle(ch):
    import spai_chess
    rng = np.random.default_rng(1)
    for _ in range(400):
        src, dst = rng.integers(0, 64, 2)
        if src == dst:
            continue
        promo = int(rng.choice([0, 0, 0, 1, 2, 3, 4]))
        m = ch.move(int(src), int(dst), promo)
        for side in (0, 1):
            if promo == 0 or (abs((dst & 7) - (src & 7)) <= 1 and (dst >> 3) - (src >> 3) == (1 if side == 0 else -1)):
                if ch.get_channel(side, m) >= 0 and (promo or _is_queen_or_knight_move(src, dst)):
                    assert spai_chess.move_index(side, m) == ch.policy_index(side, m)
    for side in (0, 1):
        for idx in range(ch.POLICY):
            assert spai_chess.index_move(side, idx) == ch.get_action(side, idx), (side, idx)


def _is_queen_or_knight_move(src, dst):
    dr, df = (dst >> 3) - (src >> 3), (dst & 7) - (src & 7)
    return dr == 0 or df == 0 or abs(dr) == abs(df) or {abs(dr), abs(df)} == {1, 2}


def test_capi_chess_params_and_no_gpu_fallback():
    import spai_chess
    # model/chess.rs at 20 blocks x 256: stem + 40 convs (+BN) + heads
    assert spai_chess.num_params(20) == 23790923
    a, b = spai_chess.init_params(1, 5), spai_chess.init_params(1, 5)
    assert np.array_equal(a, b) and spai_chess.num_params(1) == a.size
    import ctypes
    import spai
    n_dev = ctypes.c_int()
    spai.lib().spai_device_count(ctypes.byref(n_dev))
    if n_dev.value == 0:   # no GPU: the device path fails loudly (no CPU fallback)
        with pytest.raises(spai_chess.SpaiError):
            spai_chess.ChessEngine(num_searches=4, max_trees=4)

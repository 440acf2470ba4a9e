#!/usr/bin/env python3
"""Generate tests/golden/mcts_f32net.npz: MCTS and self-play driven by the
fp32 Connect4 net, computed by the CPU oracle (oracle/spai_oracle.c).

The oracle's net forward is pinned to libtorch CPU fp32 by net_c4_2x64.npz
(tests/test_oracle_golden.py::test_net_forward_vs_libtorch) and its search /
self-play to the Python transliteration of mcts.rs by mcts_hash.json; this
fixture joins the two: Mcts::search (mcts.rs:196-332) and
SelfPlayWorker::self_play (learner_concurrent.rs:169-242) with Model::predict
(model/mod.rs:36-98) as the evaluator.  The oracle takes ~12 ms per 2-block
forward, too slow to run at these sizes inside the GPU suite, hence a fixture.

Two fixtures: mcts_f32net.npz (2 blocks, 48 roots x 64 sims, 6 games x 16 sims)
and mcts_f32net_6x64.npz (the benchmarked 6x64 net, 24 roots x 128 sims, 4 games
x 32 sims):  python gen_f32net_golden.py [--six]

Contents:
  blocks, seed           blocks x 64 net from the shared init stream (spai_net_init_params)
  roots [R][3]           (x, o, n) ongoing positions after 0..13 random plies
  sims                   simulations per search
  visits [R][7], policy [R][7], n_children [R]
  sp_*                   self-play of sp_games games at sp_sims sims/move, seed sp_seed:
                         encodings, policies, values, game ids and move lists
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

SETS = {
    "mcts_f32net.npz": dict(blocks=2, seed=7, roots=48, sims=64, sp_games=6, sp_sims=16, sp_seed=21),
    "mcts_f32net_6x64.npz": dict(blocks=6, seed=0, roots=24, sims=128, sp_games=4, sp_sims=32, sp_seed=5),
}


def roots(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        s = oracle.C4()
        for _ in range(int(rng.integers(0, 14))):
            va = s.valid_actions()
            nx = s.next_state(int(rng.choice(va)))
            if nx.status != 0:
                break
            s = nx
        out.append(s)
    return out


def make(name, blocks, seed, roots_n, sims, sp_games, sp_sims, sp_seed):
    params = oracle.init_params(oracle.GAME_CONNECT4, blocks, 64, seed)
    net = oracle.Net(oracle.GAME_CONNECT4, blocks, 64, params)
    rs = roots(roots_n, 3)
    rc, pol, ids, vis, nc = oracle.search_c4(rs, sims, eval_kind=oracle.EVAL_NET, net=net)
    assert rc >= 0, rc   # number of leaves evaluated
    sp = oracle.self_play(oracle.GAME_CONNECT4, sp_games, sp_sims, sp_seed, eval_kind=oracle.EVAL_NET, net=net,
                          max_plies=42)
    np.savez_compressed(
        os.path.join(HERE, name), blocks=blocks, seed=seed,
        roots=np.array([[*s.bitboards(), s.n] for s in rs], np.uint64), sims=sims, visits=vis, policy=pol,
        n_children=nc, sp_games=sp_games, sp_sims=sp_sims, sp_seed=sp_seed, sp_enc=sp["enc"], sp_policy=sp["policy"],
        sp_value=sp["value"], sp_game=sp["game"], sp_moves=sp["moves"], sp_n_moves=sp["n_moves"])
    print("wrote", name, ":", roots_n, "roots,", len(sp["value"]), "self-play samples")


def main():
    names = ["mcts_f32net_6x64.npz"] if "--six" in sys.argv else list(SETS)
    for name in names:
        c = SETS[name]
        make(name, c["blocks"], c["seed"], c["roots"], c["sims"], c["sp_games"], c["sp_sims"], c["sp_seed"])


if __name__ == "__main__":
    main()

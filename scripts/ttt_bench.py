#!/usr/bin/env python3
"""TicTacToe, BASELINE.json config 1: one self-play game, 64 MCTS sims/move,
random-init 2-block x 64 ResNet.  The reference runs it on the CPU via tch; here
the whole game (rules, search, fp32 net) runs on the GPU through spai_ttt_*.

GPU leg: --games sequential single-game self-play runs (config 1 repeated), each
a full game of <= 9 moves x 64 search iterations; value = games/s and sims/s.
One game is 3 launches per search iteration, so this is a launch-latency
measurement, not a throughput one.  CPU leg: the oracle's self-play of the same
game (scalar C tree loop + scalar fp32 net, one core) over the same count."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "self-play-ai_amd"), os.path.join(REPO, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=20)
    ap.add_argument("--sims", type=int, default=64)
    ap.add_argument("--blocks", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    import spai_ttt as st
    params = st.init_params(args.blocks, 0)
    eng = st.TTTEngine(num_searches=args.sims, max_trees=1, eval_kind=st.EVAL_NET, seed=1)
    net = st.TTTNet(eng, args.blocks, params)
    eng.set_net(net)
    eng.self_play(1, game_id_base=10_000)   # warm-up
    sims = moves = 0
    t0 = time.perf_counter()
    for g in range(args.games):
        games, stats = eng.self_play(1, game_id_base=g)
        sims += stats["sims"]
        moves += stats["moves"]
    dt = time.perf_counter() - t0
    out = {"metric": "TicTacToe self-play, 1 game x 64 sims/move (BASELINE.json config 1)",
           "value": args.games / dt, "unit": "games/s", "sims_per_s": sims / dt, "games": args.games,
           "moves": moves, "seconds": dt, "dtype": "f32",
           "config": {"workload": "TicTacToe, 1 game at a time, %d sims/move, %dx64 ResNet fp32" % (args.sims,
                                                                                                   args.blocks)}}
    eng.close()
    if not args.no_cpu_baseline:
        import oracle
        onet = oracle.Net(oracle.GAME_TICTACTOE, args.blocks, 64, params)
        csims = 0
        t0 = time.perf_counter()
        for g in range(args.games):
            r = oracle.self_play(oracle.GAME_TICTACTOE, 1, args.sims, 1, eval_kind=oracle.EVAL_NET, net=onet,
                                 game_id_base=g, max_plies=9)
            csims += r["sims"]
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": args.games / cdt, "unit": "games/s", "sims_per_s": csims / cdt, "cores": 1,
                               "kind": "port", "sample": "%d single games: oracle tree loop + scalar fp32 net "
                                                         "(oracle/spai_oracle.c), one thread" % args.games}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

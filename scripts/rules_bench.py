#!/usr/bin/env python3
"""Batched bitboard rules kernels on one MI355X (north_star: "rocprof HBM GB/s on
the bitboard kernels").

Connect4 (HBM-bound byte kernels, rules.hip): 2^24 random reachable positions,
legal mask / apply / bf16 encoding, algorithmic bytes per game 18 / 33 / 269
(rules.hip header) -> GB/s and fraction of the 8 TB/s HBM peak.

Chess (chess_rules.hip): N random reachable positions (random legal play on the
device through the batched API), one wave per position: ordered legal-move list +
count + status (k_slots_status) and the f32 encoding (k_slots_encode).  Move
generation is ALU work (bitboard fills, a packed prefix scan), so it is reported as
positions/s and generated moves/s next to its bytes/s.
Times are HIP events around each launch (mean of --iters)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "self-play-ai_amd")]
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4-games", type=int, default=1 << 24)
    ap.add_argument("--chess-positions", type=int, default=1 << 16)
    ap.add_argument("--chess-plies", type=int, default=60, help="random plies per position (uniform 0..N)")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import spai
    import spai_chess as sc

    out = {"c4": {}, "chess": {}}
    e = spai.Engine(num_searches=1, max_trees=1)
    n = args.c4_games
    ms = e.rules_bench(n, iters=args.iters)
    for name, m, b in zip(("k_legal", "k_apply", "k_encode_bf16"), ms, (18, 33, 269)):
        gbs = n * b / (m * 1e-3) / 1e9
        out["c4"][name] = {"games": n, "ms": m, "bytes_per_game": b, "GB/s": gbs, "frac_hbm": gbs / HBM_PEAK_GBS,
                           "games_per_s": n / (m * 1e-3)}
    e.close()
    print("[rules_bench] c4 done", file=sys.stderr, flush=True)

    N = args.chess_positions
    ce = sc.ChessEngine(num_searches=1, max_trees=1, eval_kind=sc.EVAL_HASH, max_moves=256)
    ce.games_resize(N)
    rng = np.random.default_rng(0)
    stop = rng.integers(0, args.chess_plies + 1, N)
    t0 = time.perf_counter()
    for p in range(args.chess_plies):
        mv, cnt = ce.legal_moves(N)
        pick = rng.integers(0, np.maximum(cnt, 1))
        m = mv[np.arange(N), pick].astype(np.uint16)
        m[(p >= stop) | (cnt == 0)] = 0          # an illegal move leaves the slot unchanged
        ce.apply(m, check=False)
    setup_s = time.perf_counter() - t0
    mv, cnt = ce.legal_moves(N)
    st, _, _, _ = ce.status(N)
    ms = ce.rules_bench(N, iters=args.iters)
    moves = float(cnt.sum())
    hist_avg = float(np.minimum(stop, args.chess_plies).mean())
    # bytes per position: Board 72 + n_hist 4 + repetition scan of the history
    # (8 B per earlier position) in; move list 2 B per move + count 4 + status 1 out
    b_legal = 72 + 4 + 8 * hist_avg + 2 * moves / N + 5
    b_enc = 72 + 4 + 8 * hist_avg + 19 * 64 * 4
    for name, m, b in (("k_slots_status", ms[0], b_legal), ("k_slots_encode", ms[1], b_enc)):
        gbs = N * b / (m * 1e-3) / 1e9
        out["chess"][name] = {"positions": N, "ms": m, "bytes_per_position": b, "GB/s": gbs,
                              "frac_hbm": gbs / HBM_PEAK_GBS, "positions_per_s": N / (m * 1e-3)}
    out["chess"]["k_slots_status"]["moves_per_s"] = moves / (ms[0] * 1e-3)
    out["chess"]["sample"] = {"positions": N, "avg_legal_moves": moves / N, "ongoing": int((st == 0).sum()),
                              "avg_plies_played": hist_avg, "setup_s": setup_s}
    ce.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

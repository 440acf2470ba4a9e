#!/usr/bin/env python3
"""Chess self-play benchmark on one MI355X (BASELINE.json config 4: 1024
parallel games, 400 MCTS simulations per move, 20-block x 256 ResNet, bf16).

GPU leg: the first --moves moves of all games from the start position (each
move = Mcts::search over every live tree + sampling + use_subtree), or with
--full every game to completion through spai_chess_selfplay_run.  value =
simulations/s (trees x search iterations).  roofline = the fused chess forward:
3,036,348,928 algorithmic FLOPs per evaluated leaf x leaves per launch / its
HIP-event time, vs 2.5 PF dense bf16.

CPU leg (subprocess, --cpu-seconds window): the chess oracle's tree loop
(reference layout: AoS arena with a full State per node, sequential descent)
with the same net on libtorch CPU fp32, bounded to whole search iterations.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "self-play-ai_amd"), os.path.join(REPO, "oracle")]
BF16_PEAK_TFLOPS = 2500.0


def flops_per_eval(blocks):
    """2 x MACs of model/chess.rs:48-77 at 256 channels (3,036,348,928 at 20 blocks)"""
    conv = lambda ci, co, k: 2 * 64 * co * ci * k * k
    return (conv(19, 256, 3) + 2 * blocks * conv(256, 256, 3) + conv(256, 256, 1) + conv(256, 73, 1) +
            conv(256, 1, 1) + 2 * 64 * 256 + 2 * 256)


def weight_bytes(blocks):
    """bytes k_chess_forward reads as weights (chess_net.hip packing): bf16 conv fragments
    (stem 32 padded input channels, 2*blocks residual 3x3 convs, policy 1x1 256->256 and
    256->80 padded), fp32 biases and the fp32 value head (1x1 256->1, linear 64->256, 256->1)"""
    bf16 = 32 * 256 * 9 + 2 * blocks * 256 * 256 * 9 + 256 * 256 + 256 * 80
    f32 = 256 + 2 * blocks * 256 + 256 + 80 + (256 + 1) + (64 * 256 + 256) + (256 + 1)
    return 2 * bf16 + 4 * f32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=1024)
    ap.add_argument("--sims", type=int, default=400)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--moves", type=int, default=4)
    ap.add_argument("--full", action="store_true", help="play every game to completion (selfplay_run)")
    ap.add_argument("--batches", type=int, default=1,
                    help="--full: K x games games, as K lockstep batches or (--stream) one stream through the slots")
    ap.add_argument("--stream", action="store_true",
                    help="--full: the K x games games through `games` tree slots (spai_chess_selfplay_stream)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-games", type=int, default=32)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r01", "chess", "forward_traffic.json"),
                    help="PMC summary (scripts/gpu_chess_traffic.sh): HBM bytes per k_chess_forward launch")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def cpu_baseline(args):
    import torch
    import torch.nn.functional as F

    import chessref as ch
    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    L = ch.lib()
    import spai_chess
    P = ch.unpack_params(spai_chess.init_params(args.blocks, args.seed), args.blocks)
    T = [(k, tuple(torch.from_numpy(np.ascontiguousarray(a)) for a in v) if k == "bn" else torch.from_numpy(v))
         for k, v in P]
    enc = np.zeros((args.cpu_games, 19, 8, 8), np.float32)
    pri = np.zeros(ch.POLICY, np.float32)

    def forward(x):
        it = iter(T)

        def nxt():
            return next(it)[1]

        def bn(h):
            g, b, m, v = nxt()
            return F.batch_norm(h, m, v, g, b, training=False, eps=1e-5)

        h = F.relu(bn(F.conv2d(x, nxt(), nxt(), padding=1)))
        for _ in range(args.blocks):
            y = F.relu(bn(F.conv2d(h, nxt(), nxt(), padding=1)))
            h = F.relu(h + bn(F.conv2d(y, nxt(), nxt(), padding=1)))
        p = F.conv2d(F.relu(F.conv2d(h, nxt(), nxt())), nxt(), nxt()).flatten(1)
        v = F.relu(F.conv2d(h, nxt(), nxt())).flatten(1)
        v = torch.tanh(F.linear(F.relu(F.linear(v, nxt(), nxt())), nxt(), nxt()))[:, 0]
        return torch.softmax(p, -1), v

    def evaluate(user, n, states, priors, values):
        # Model::predict (model/mod.rs:36-98): encode, forward, softmax, mask_invalid_actions
        for i in range(n):
            L.orc_encoding(states[i], enc[i].ctypes.data_as(C.POINTER(C.c_float)))
        with torch.no_grad():
            sm, v = forward(torch.from_numpy(enc[:n]))
        sm = np.ascontiguousarray(sm.numpy())
        for i in range(n):
            L.orc_mask_invalid(states[i], sm[i].ctypes.data_as(C.POINTER(C.c_float)), ch.POLICY,
                               C.cast(C.addressof(priors.contents) + 4 * ch.POLICY * i, C.POINTER(C.c_float)))
        np.ctypeslib.as_array(values, (n,))[:] = v.numpy()

    cb = ch.EVAL_FN(evaluate)
    n = args.cpu_games
    trees = [L.orc_tree_create() for _ in range(n)]
    arr = (C.c_void_p * n)(*trees)
    pol = np.zeros((n, ch.POLICY), np.float32)
    ids = np.zeros((n, ch.MAX_MOVES), np.int32)
    vis = np.zeros((n, ch.MAX_MOVES), np.float32)
    nc = np.zeros(n, np.int32)
    ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    t0 = time.perf_counter()
    sims = 0
    while time.perf_counter() - t0 < args.cpu_seconds:
        L.orc_search(arr, n, 1, 2.0, cb, None, fp(pol), ip(ids), fp(vis), None, ip(nc))
        sims += n
    dt = time.perf_counter() - t0
    for t in trees:
        L.orc_tree_destroy(t)
    print(json.dumps({"value": sims / dt, "unit": "sims/s", "cores": threads, "kind": "port",
                      "sample": f"{n} chess games from the start position, {sims // n} search iterations in "
                                f"{dt:.1f}s: chess oracle tree loop (AoS arena, State clones, sequential) + "
                                f"libtorch CPU fp32 {args.blocks}x256 forward on {threads} threads"}))


def run_cpu_baseline(args):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-seconds", str(args.cpu_seconds),
           "--cpu-games", str(args.cpu_games), "--blocks", str(args.blocks), "--seed", str(args.seed)]
    if args.cpu_threads:
        cmd += ["--cpu-threads", str(args.cpu_threads)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.cpu_seconds * 4 + 180)
        return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    except Exception as ex:
        return {"value": None, "unit": "sims/s", "error": repr(ex)[:300]}


def heartbeat(stop, t0):
    while not stop.wait(30.0):
        print("[chess_bench] %.0f s" % (time.perf_counter() - t0), file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline(args)
        return
    import spai_chess as sc
    eng = sc.ChessEngine(num_searches=args.sims, max_trees=args.games, eval_kind=sc.EVAL_NET, seed=args.seed)
    net = sc.ChessNet(eng, args.blocks, sc.init_params(args.blocks, args.seed))
    eng.set_net(net)
    # warm-up: one short search
    eng.trees_create(args.games)
    eng.search(np.arange(args.games), num_searches=4)
    eng.trees_create(args.games)
    eng.set_timing(True)
    stop = threading.Event()
    t_start = time.perf_counter()
    threading.Thread(target=heartbeat, args=(stop, t_start), daemon=True).start()
    rng = np.random.default_rng(args.seed)
    if args.full:
        sims = games = moves = 0
        if args.stream:
            _, st = eng.self_play(args.batches * args.games, keep=False, window=args.games)
            sims, games, moves = st["sims"], st["games"], st["moves"]
        else:
            for k in range(args.batches):
                _, st = eng.self_play(args.games, game_id_base=k * args.games, keep=False)
                sims, games, moves = sims + st["sims"], games + st["games"], moves + st["moves"]
        dt = time.perf_counter() - t_start
    else:
        live = np.arange(args.games, dtype=np.uint32)
        sims = games = moves = 0
        t0 = time.perf_counter()
        for m in range(args.moves):
            pol, ids, vis, mv, nc = eng.search(live)
            sims += len(live) * args.sims
            w = np.power(vis.astype(np.float64), 1.25)          # learner_concurrent.rs:189-193
            w[np.arange(vis.shape[1])[None, :] >= nc[:, None]] = 0
            cum = np.cumsum(w, 1)
            u = rng.random(len(live))[:, None] * cum[:, -1:]
            pick = np.minimum((cum <= u).sum(1), nc - 1).astype(np.uint32)
            status, _ = eng.advance(live, pick)
            games += int((status != 0).sum())
            live = live[status == 0]
            moves += 1
            if len(live) == 0:
                break
        dt = time.perf_counter() - t0
    stop.set()
    ms, launches, items = eng.timing()
    fpe = flops_per_eval(args.blocks)
    leaves = items[1] / max(1.0, launches[1])
    achieved = fpe * leaves / (ms[1] * 1e-3) / 1e12 if ms[1] > 0 else None
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):   # measured by separate rocprofv3 --pmc passes of this workload
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if "k_chess_forward" in tj:
            traffic = tj["k_chess_forward"]["hbm_bytes_per_launch"]
            traffic_src = ("%s: (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch over %d launches (FETCH doubled for "
                           "gfx950)" % (os.path.relpath(args.traffic_json, REPO), tj["k_chess_forward"]["launches"]))
    result = {
        "metric": "MCTS sims/sec, chess 400 sims/move (BASELINE.json config 4)",
        "value": sims / dt, "unit": "sims/s", "n_gpus": 1, "higher_is_better": True, "dtype": "bf16",
        "data": "synthetic: self-play from the start position, random-init net (tch default init, seed %d)" % args.seed,
        "config": {"workload": "chess self-play, %d games x %d sims/move, %dx256 ResNet bf16, %s"
                               % (args.games, args.sims, args.blocks,
                                  ("%d games to completion%s" % (args.batches * args.games,
                                                                 ", streamed through the slots" if args.stream else "")
                                   if args.full else "first %d moves" % moves)),
                   "games": args.games, "sims_per_move": args.sims, "blocks": args.blocks},
        "seconds": dt, "moves": moves, "games_finished": games,
        "games_per_sec": games / dt if args.full else None,
        "kernel_ms": {"select_leaf": ms[0], "forward": ms[1], "expand": ms[2]},
        "roofline": {"bound": "mfma", "kernel": "k_chess_forward (fused %dx256 ResNet)" % args.blocks,
                     "achieved": achieved, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_PEAK_TFLOPS if achieved else None, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "flop_per_eval": fpe, "avg_leaves_per_launch": leaves, "avg_launch_ms": ms[1],
                     # weights once + per leaf the bf16 input planes [64][32] in, 4672 logits + value out
                     "algorithmic_bytes": weight_bytes(args.blocks) + leaves * (64 * 32 * 2 + 4672 * 4 + 4)},
    }
    net.close()
    eng.close()
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = run_cpu_baseline(args)
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()

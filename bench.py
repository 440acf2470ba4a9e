#!/usr/bin/env python3
"""Benchmark: batched self-play MCTS on MI355X (BASELINE.json metric).

One step = one SelfPlayWorker::self_play call (learner_concurrent.rs:169-242):
G games from the empty Connect4 board played to completion with 800 MCTS
simulations per move against a random-init 6-block x 64 ResNet (bf16 MFMA),
all of it on the device (search trees in HBM, fused net forward per search
iteration).  value = MCTS simulations per second summed over all ranks.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): games are
sharded by id across ranks (rank r plays ids [r*G, (r+1)*G) per step), no
collective touches the data path; gloo carries only the timing barrier and the
max/sum reductions.  The GPU process never imports torch at N=1 (torch ships
its own HIP runtime).

Adds to the JSON line:
  roofline      the fused forward kernel (dominant): algorithmic FLOPs of the
                evaluated leaves / HIP-event time of the sampled launches
                (engine stream), vs the 2.5 PF dense bf16 MFMA peak
  cpu_baseline  the CPU restatement (oracle/: reference data layout, AoS
                arena with State clones, sequential tree loop) with the net on
                libtorch CPU fp32, run in a subprocess for a bounded window
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "self-play-ai_amd"))

METRIC = "MCTS sims/sec + self-play games/sec, Connect4 800 sims/move, 1/2/4/8 GPU"
BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def flops_per_eval(blocks, hid=64):
    """algorithmic FLOPs (2 x MACs) of one C4 forward (39,016,572 at 6x64)"""
    cells = 42
    conv = lambda ci, co: 2 * cells * co * ci * 9
    return conv(3, hid) + 2 * blocks * conv(hid, hid) + conv(hid, 32) + conv(hid, 3) + 2 * 1344 * 7 + 2 * 126


def weight_bytes(blocks):
    """bytes the fused C4 forward reads as weights (net_c4.hip packing): residual convs
    [2*blocks][18 k-steps][4 co tiles] x 1 KiB fragments, stem 4 KiB, head [18][3] x 1 KiB,
    fused linear 48 x 1 KiB, fp32 biases (64 + 2*blocks*64 + 48) + 8"""
    return 2 * blocks * 18 * 4 * 1024 + 4096 + 18 * 3 * 1024 + 48 * 1024 + 4 * (64 + 2 * blocks * 64 + 48 + 8)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--games", type=int, default=4096, help="parallel self-play games per GPU")
    ap.add_argument("--sims", type=int, default=800, help="MCTS simulations per move")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-games", type=int, default=256)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--rules-bench", action="store_true", help="also time the batched rules kernels")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events (A/B of their cost)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r01", "forward_traffic.json"),
                    help="PMC summary (scripts/gpu_traffic.sh) of this bench command: HBM bytes per k_forward launch")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


# ---------------------------------------------------------------- CPU baseline (subprocess)
def cpu_baseline(args):
    """Oracle self-play (reference algorithm and data layout) + libtorch CPU fp32
    forward, for a bounded wall-time window; prints one JSON line."""
    import ctypes as C

    import numpy as np
    import torch
    import torch.nn.functional as F

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    threads = args.cpu_threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    L = O.lib()
    p = torch.from_numpy(O.init_params(O.GAME_CONNECT4, args.blocks, 64, args.seed))
    off = [0]

    def take(*shape):
        n = int(np.prod(shape))
        v = p[off[0]:off[0] + n].reshape(shape)
        off[0] += n
        return v

    def cbn(ci, co):
        return [take(co, ci, 3, 3), take(co), take(co), take(co), take(co), take(co)]

    stem = cbn(3, 64)
    blocks = [(cbn(64, 64), cbn(64, 64)) for _ in range(args.blocks)]
    pol = cbn(64, 32)
    pw, pb = take(7, 1344), take(7)
    val = cbn(64, 3)
    vw, vb = take(1, 126), take(1)

    def conv_bn(t, c, relu):
        w, b, g, be, mu, var = c
        t = F.batch_norm(F.conv2d(t, w, b, padding=1), mu, var, g, be, training=False, eps=1e-5)
        return F.relu(t) if relu else t

    enc = np.zeros((args.cpu_games, 126), np.float32)
    deadline = [None]
    iters = [0]

    class Stop(Exception):
        pass

    def evaluate(user, n, states, priors, values):
        # Model::predict on the CPU (model/mod.rs:36-98): encode, forward, softmax, mask
        L.or_encode_states(O.GAME_CONNECT4, n, states, enc.ctypes.data_as(C.POINTER(C.c_float)))
        with torch.no_grad():
            t = torch.from_numpy(enc[:n]).view(-1, 3, 6, 7)
            t = conv_bn(t, stem, True)
            for c1, c2 in blocks:
                t = F.relu(t + conv_bn(conv_bn(t, c1, True), c2, False))
            lg = F.linear(conv_bn(t, pol, True).flatten(1), pw, pb)
            v = torch.tanh(F.linear(conv_bn(t, val, True).flatten(1), vw, vb)).view(-1)
            sm = torch.softmax(lg, -1).numpy()
        legal = enc[:n].reshape(n, 3, 6, 7)[:, 2, 5, :]
        m = sm * legal
        m /= m.sum(1, keepdims=True)
        pr = np.ctypeslib.as_array(priors, (n, 7))
        pr[:] = m
        np.ctypeslib.as_array(values, (n,))[:] = v.numpy()
        iters[0] += 1

    # run whole moves until the window closes; count simulations of completed moves
    trees = [L.or_tree_create(O.GAME_CONNECT4) for _ in range(args.cpu_games)]
    arr = (C.c_void_p * len(trees))(*trees)
    n = len(trees)
    pol_o = np.zeros((n, 7), np.float32)
    ids = np.zeros((n, 7), np.int32)
    vis = np.zeros((n, 7), np.float32)
    nc = np.zeros(n, np.int32)
    cb = O.EVAL_FN(evaluate)
    t0 = time.perf_counter()
    sims = 0
    moves = 0
    chunk = 50   # search iterations per call; the reference runs 800 per move
    while time.perf_counter() - t0 < args.cpu_seconds and moves < 4:
        done = 0
        while done < args.sims and time.perf_counter() - t0 < args.cpu_seconds:
            k = min(chunk, args.sims - done)
            L.or_search(arr, n, k, 2.0, O.EVAL_NET, None, cb, None, O._f(pol_o), O._i(ids), O._f(vis), O._i(nc))
            done += k
            sims += n * k
        if done < args.sims:
            break
        moves += 1
        for i, t in enumerate(trees):   # advance on the most visited child, as a move would
            j = int(np.argmax(vis[i, :nc[i]]))
            L.or_tree_use_subtree(t, int(ids[i, j]))
    dt = time.perf_counter() - t0
    for t in trees:
        L.or_tree_destroy(t)
    sps = sims / dt
    print(json.dumps({"value": sps, "unit": "sims/s", "cores": threads, "kind": "port",
                      "sample": f"{args.cpu_games} C4 games from the empty board, {sims // n} search iterations "
                                f"(800 sims/move) in {dt:.1f}s: oracle tree loop (AoS arena, State clones, "
                                f"sequential) + libtorch CPU fp32 {args.blocks}x64 forward on {threads} threads; "
                                f"games/s estimate = sims/s / (800 x plies per game)",
                      "cpu_model": _cpu_model()}))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run_cpu_baseline(args):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-seconds", str(args.cpu_seconds),
           "--cpu-games", str(args.cpu_games), "--blocks", str(args.blocks), "--sims", str(args.sims),
           "--seed", str(args.seed)]
    if args.cpu_threads:
        cmd += ["--cpu-threads", str(args.cpu_threads)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.cpu_seconds * 4 + 120)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
        return json.loads(line)
    except Exception as ex:  # the baseline must never sink the GPU number
        return {"value": None, "unit": "sims/s", "error": repr(ex)[:300]}


# ---------------------------------------------------------------- GPU bench
class Dist:
    """one process per GPU; host-side barrier and scalar reductions over a socket
    group (hostgroup.py) so no torch (and no second HIP runtime) enters the GPU process"""

    def __init__(self):
        from hostgroup import HostGroup
        self.g = HostGroup()
        self.world, self.rank = self.g.world, self.g.rank
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if "SPAI_BENCH_DEVICE" in os.environ:   # rehearsal: every rank on one device
            self.local = int(os.environ["SPAI_BENCH_DEVICE"])

    def barrier(self):
        self.g.barrier()

    def reduce(self, values, op):
        return self.g.allreduce(values, op)

    def close(self):
        self.g.close()


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline(args)
        return
    dist = Dist()
    import spai

    eng = spai.Engine(num_searches=args.sims, max_trees=args.games, eval_kind=spai.EVAL_NET, device=dist.local,
                      seed=args.seed)
    net = spai.Net(eng, args.blocks, spai.init_params(args.blocks, 64, seed=args.seed))
    eng.set_net(net)
    G = args.games

    def step(i):
        base = (i * dist.world + dist.rank) * G
        _, st = eng.self_play(G, game_id_base=base, collect=False)
        return st

    for i in range(args.warmup):
        step(-1 - i)
    eng.sync()
    dist.barrier()
    # HIP events on every 32nd search iteration of each chain: ~0.6 % overhead (every
    # 4th measured ~5 %: 31.9M vs 33.4M sims/s), ~1000 sampled launches per step
    eng.set_timing(not args.no_timing, stride=32)
    tot = dict(sims=0.0, games=0.0, evals=0.0, positions=0.0, moves=0.0)
    t0 = time.perf_counter()
    for i in range(args.steps):
        st = step(i)
        for k in tot:
            tot[k] += st[k]
    eng.sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    timing = eng.timing()
    (dt_max,) = dist.reduce([dt], "max")
    sims, games, evals, positions = dist.reduce([tot["sims"], tot["games"], tot["evals"], tot["positions"]], "sum")

    fpe = flops_per_eval(args.blocks)
    ev = timing["evaluate"]
    achieved = fpe * ev["items"] / (ev["total_ms"] * 1e-3) / 1e12 if ev["total_ms"] > 0 else None
    per_launch_flop = fpe * ev["items"] / ev["launches"] if ev["launches"] else None
    traffic, traffic_src = None, None
    if os.path.exists(args.traffic_json):   # measured by separate rocprofv3 --pmc passes of this command
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if "k_forward<false>" in tj:
            traffic = tj["k_forward<false>"]["hbm_bytes_per_launch"]
            traffic_src = ("%s: (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch over %d launches "
                           "(FETCH doubled for gfx950)" % (os.path.relpath(args.traffic_json, REPO),
                                                           tj["k_forward<false>"]["launches"]))
    result = {
        "metric": METRIC,
        "value": sims / dt_max,
        "unit": "sims/s",
        "games_per_sec": games / dt_max,
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max * 1e3 / max(1, args.steps),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic: self-play from the empty board, random-init net (tch default init, seed %d)" % args.seed,
        "config": {"workload": "Connect4 self-play, %d games/GPU x %d sims/move, %dx64 ResNet bf16, to completion"
                               % (G, args.sims, args.blocks),
                   "model": "c4-resnet-%dx64" % args.blocks, "games_per_gpu": G, "sims_per_move": args.sims,
                   "global_batch": G * dist.world, "parallelism": "dp%d (games sharded, no collective)" % dist.world},
        "evals_per_sec": evals / dt_max,
        "positions_per_sec": positions / dt_max,
        "kernel_ms": {k: v["avg_ms"] for k, v in timing.items()},
        "roofline": {"bound": "mfma", "kernel": "k_forward (fused 6x64 ResNet)",
                     "achieved": achieved, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_PEAK_TFLOPS if achieved else None, "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     # algorithmic bytes of one launch: the packed bf16 weights + fp32 biases once,
                     # plus per leaf 16 B of bitboards in and 36 B (8 priors + value) out
                     "algorithmic_bytes": weight_bytes(args.blocks) + 52 * (ev["items"] / max(1, ev["launches"])),
                     "flop_per_launch": per_launch_flop, "flop_per_eval": fpe,
                     # whole-GPU view: every forward FLOP of the timed region over its wall time
                     # (the two search chains' forwards overlap, so this is not per launch)
                     "chip_achieved": evals / dt_max * fpe / 1e12 / dist.world,
                     "chip_frac": evals / dt_max * fpe / 1e12 / dist.world / BF16_PEAK_TFLOPS,
                     "avg_launch_ms": ev["avg_ms"], "avg_leaves_per_launch": ev["items"] / max(1, ev["launches"])},
    }
    if args.rules_bench and dist.rank == 0:
        n = 1 << 24
        ms = eng.rules_bench(n, iters=10)
        bytes_per = [18, 33, 269]
        result["rules_kernels"] = {nm: {"ms": m, "GB/s": n * b / (m * 1e-3) / 1e9, "frac": n * b / (m * 1e-3) / 1e9 / HBM_PEAK_GBS}
                                   for nm, m, b in zip(("legal", "apply", "encode_bf16"), ms, bytes_per)}
    net.close()
    eng.close()
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        cb = run_cpu_baseline(args)
        result["cpu_baseline"] = cb
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: batched self-play MCTS on MI355X (BASELINE.json metric).

One step = one SelfPlayWorker::self_play call (learner_concurrent.rs:169-242):
G games from the empty Connect4 board played to completion with 800 MCTS
simulations per move against a random-init 6-block x 64 ResNet (bf16 MFMA),
all of it on the device (search trees in HBM, fused net forward per search
iteration).  value = MCTS simulations per second summed over all ranks.

Multi-GPU: `python bench.py --gpus N` (no launcher) starts N rank processes
itself, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_* on
127.0.0.1), and relays rank 0's line; under `torch.distributed.run
--nproc-per-node N ... bench.py --gpus N` the launcher's ranks are used and
WORLD_SIZE must equal N.  Games are sharded by id across ranks (rank r plays
ids [r*G, (r+1)*G) per step), no collective touches the data path (main.rs:
169-186,220-234: each worker owns its Mcts + Model); a rank-0 TCP star
(hostgroup.py, not torch gloo) carries the timing barrier and the max/sum
reductions, and the same work counters and step times are reduced once more
through an N-rank RCCL communicator over the ranks' devices (`rccl` in the
line: its rank count and whether its sums equal the host group's).  The GPU
process never imports torch (torch ships its own HIP runtime with the same
SONAME).

Adds to the JSON line:
  roofline      the fused forward kernel (dominant) vs the 2.5 PF dense bf16
                MFMA peak.  achieved/frac = job level: the algorithmic FLOPs of
                every leaf evaluated in the timed region over its wall time (the
                two search chains' forwards overlap each other and the tree
                kernels, so per-launch event times overlap and do not add up to
                the step).  per_launch = the same FLOPs over the HIP-event time
                of the sampled launches (engine streams; CUs shared), the figure
                rocprof's kernel average checks.  isolated = the kernel alone.
  rules_kernels the bitboard rules kernels (k_legal4, k_apply4, k_encode bf16)
                on 2^24 game slots: algorithmic bytes / HIP-event time vs 8 TB/s
  chess         BASELINE config 4 window: 1024 chess games x 400 sims, the
                first 2 moves (sims/s, k_chess_forward fraction of peak)
  cpu_baseline  the CPU restatement (oracle/refcpu.py: reference data layout,
                AoS arena with State clones, sequential tree loop) with the net
                on libtorch CPU fp32, run in a subprocess: the reference worker's
                batch of 100 games played to completion in this run (vs_baseline
                divides by it), beside the committed 256-game record (flagged
                with whether it was taken on this host)
"""
import argparse
import json
import os
import resource
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--games", type=int, default=4096, help="parallel self-play games per GPU")
    ap.add_argument("--sims", type=int, default=800, help="MCTS simulations per move")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--lockstep", action="store_true",
                    help="one lockstep batch of G games per step (every game starts together; the batch thins out "
                         "as games end) instead of the default stream: the steps' K x G games played through G tree "
                         "slots, a slot taking the next game when its game ends (spai_selfplay_stream)")
    ap.add_argument("--stream", action="store_true", help=argparse.SUPPRESS)   # the default; kept for old scripts
    ap.add_argument("--no-lockstep-ref", action="store_true",
                    help="skip the one-step lockstep figure reported beside the streamed headline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-games", type=int, default=100,
                    help="games the CPU baseline plays to completion inside this run: the reference worker's batch "
                         "(learner_concurrent.rs:50-59, num_batched_self_play_games = 100), ~2 min on the GPU box's host")
    ap.add_argument("--cpu-timeout", type=float, default=360.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-rules-bench", action="store_true", help="skip the batched rules-kernel timing (HBM GB/s)")
    ap.add_argument("--no-chess", action="store_true", help="skip the chess window (config 4, 2 moves)")
    ap.add_argument("--chess-moves", type=int, default=2)
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events (A/B of their cost)")
    ap.add_argument("--no-isolated", action="store_true", help="skip the isolated-forward measurement")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r05", "final", "forward_traffic.json"),
                    help="PMC summary (scripts/gpu_traffic.sh) of this bench command: HBM bytes per k_forward launch")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "r06", "final_s3", "forward_pmc.json"),
                    help="PMC summary of this bench command (scripts/gpu_roofline_pmc.sh): executed MFMA FLOPs, MFMA "
                         "busy cycles and HBM bytes per k_forward launch; preferred over --traffic-json when present")
    ap.add_argument("--chess-cpu-seconds", type=float, default=15.0,
                    help="the chess window's CPU leg: this many seconds of the chess oracle's tree loop + libtorch "
                         "CPU 20x256 (scripts/chess_bench.py --cpu-baseline-only)")
    ap.add_argument("--chess-cpu-games", type=int, default=16)
    ap.add_argument("--chess-record", default=os.path.join(REPO, "profiles", "r06", "chess_full", "record.json"),
                    help="committed record of BASELINE config 4 played to completion (scripts/chess_bench.py --full)")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


# ---------------------------------------------------------------- CPU baseline (subprocess)
CPU_RECORD = os.path.join(REPO, "profiles", "r02", "cpu_baseline.json")


def cpu_record():
    """the committed CPU record (scripts/cpu_games_baseline.py on the GPU box's host):
    the thread sweep and a run of whole games to completion at 800 sims/move"""
    try:
        with open(CPU_RECORD) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def cpu_baseline(args):
    """SelfPlayWorker::self_play on the CPU, measured in THIS run: args.cpu_games games
    from the empty board played to completion at args.sims sims/move by the oracle
    tree loop (reference algorithm and data layout) + libtorch CPU fp32 forward
    (oracle/refcpu.py).  Whole games, so the rate covers every game phase (an
    early-game window flatters the CPU: its early positions are its best case).
    The default is the reference worker's batch, 100 games
    (learner_concurrent.rs:50-59).  The committed larger run
    (profiles/r02/cpu_baseline.json, 256 games) is reported beside it, flagged by
    whether it was taken on this host.  Prints one JSON line."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import refcpu

    rec = cpu_record()
    model, quota = refcpu.cpu_model(), refcpu.cpu_quota()
    # the record counts only for the same host and the same workload (800 sims, 6x64)
    same_host = (bool(rec) and rec.get("cpu_model") == model and rec.get("cpu_quota") == quota
                 and args.sims == 800 and args.blocks == 6)
    threads = args.cpu_threads or (rec.get("best_threads") if same_host else None) or min(8, quota)
    r = refcpu.games_to_completion(args.cpu_games, args.sims, blocks=args.blocks, seed=args.seed, threads=threads)
    out = {"value": r["sims_per_sec"], "unit": "sims/s", "games_per_sec": r["games_per_sec"], "cores": threads,
           "kind": "port",
           "sample": f"{args.cpu_games} C4 games from the empty board played to completion at {args.sims} sims/move "
                     f"({r['positions']} positions, mean {r['mean_plies']:.1f} plies, {r['sims_done']:.0f} sims) in "
                     f"{r['seconds']:.1f}s: oracle tree loop (AoS arena, State clones, sequential) + libtorch CPU "
                     f"fp32 {args.blocks}x64 forward batched over the live games, {threads} intra-op threads",
           "cpu_model": model, "os_cpu_count": os.cpu_count(), "cpu_quota": quota}
    if rec and "games_run" in rec:
        g = rec["games_run"]
        out["record"] = {
            "games_per_sec": g["games_per_sec"], "sims_per_sec": g["sims_per_sec"], "same_host": same_host,
            "sample": (f"{g['games']} games played to completion at {g.get('sims', 800)} sims/move "
                       f"({g['positions']} positions, "
                       f"mean {g['mean_plies']:.1f} plies, {g['seconds']:.0f}s) on {g['threads']} threads; record "
                       f"{os.path.relpath(CPU_RECORD, REPO)} ({rec.get('cpu_model', '?')}, cpu quota "
                       f"{rec.get('cpu_quota', '?')})")}
    print(json.dumps(out))


def run_cpu_baseline(args):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only",
           "--cpu-games", str(args.cpu_games), "--blocks", str(args.blocks), "--sims", str(args.sims),
           "--seed", str(args.seed)]
    if args.cpu_threads:
        cmd += ["--cpu-threads", str(args.cpu_threads)]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=args.cpu_timeout)
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


def rules_bench(eng):
    """k_legal4 / k_apply4 / k_encode<bf16> over 2^24 C4 game slots (spai_rules_bench:
    HIP events over 10 launches each); algorithmic bytes per slot: legal 16 B of
    bitboards in + 2 B mask out, apply 16 + 1 + 4 (action) in and 8 + 4 out, encode
    16 B in + 126 x 2 B planes + 1 out"""
    n = 1 << 24
    ms = eng.rules_bench(n, iters=10)
    out = {}
    for nm, m, b in zip(("k_legal4", "k_apply4", "k_encode_bf16"), ms, (18, 33, 269)):
        gbs = n * b / (m * 1e-3) / 1e9
        out[nm] = {"ms": m, "slots": n, "bytes_per_slot": b, "GB/s": gbs, "frac": gbs / HBM_PEAK_GBS}
    return out


def chess_window(args, device, dist_world=1):
    """BASELINE config 4 (chess, 1024 games x 400 sims/move, 20x256 bf16) for the first
    --chess-moves moves from the start position: every move searches every live tree,
    samples visits^1.25 and re-roots (scripts/chess_bench.py, windowed).  sims/s and
    k_chess_forward's algorithmic FLOPs over its HIP-event time; ~2 s of GPU time"""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import chess_bench as cb
    import spai_chess as sc
    games, sims, blocks = 1024, 400, 20
    eng = sc.ChessEngine(num_searches=sims, max_trees=games, eval_kind=sc.EVAL_NET, device=device, seed=args.seed)
    net = sc.ChessNet(eng, blocks, sc.init_params(blocks, args.seed))
    eng.set_net(net)
    eng.trees_create(games)
    eng.search(np.arange(games), num_searches=4)   # warm-up
    eng.trees_create(games)
    eng.set_timing(True)
    rng = np.random.default_rng(args.seed)
    live = np.arange(games, dtype=np.uint32)
    done = 0
    t0 = time.perf_counter()
    for _ in range(args.chess_moves):
        _, _, vis, _, nc = eng.search(live)
        done += len(live) * sims
        w = np.power(vis.astype(np.float64), 1.25)   # learner_concurrent.rs:189-193
        w[np.arange(vis.shape[1])[None, :] >= nc[:, None]] = 0
        cum = np.cumsum(w, 1)
        u = rng.random(len(live))[:, None] * cum[:, -1:]
        pick = np.minimum((cum <= u).sum(1), nc - 1).astype(np.uint32)
        status, _ = eng.advance(live, pick)
        live = live[status == 0]
    dt = time.perf_counter() - t0
    ms, launches, items = eng.timing()
    net.close()
    eng.close()
    fpe = cb.flops_per_eval(blocks)
    leaves = items[1] / max(1.0, launches[1])
    tf = fpe * leaves / (ms[1] * 1e-3) / 1e12 if ms[1] > 0 else None
    out = {"workload": "chess self-play, %d games x %d sims/move, %dx256 ResNet bf16, first %d moves from the "
                       "start position" % (games, sims, blocks, args.chess_moves),
           "sims_per_sec": done / dt, "seconds": dt,
           "forward": {"kernel": "k_chess_forward", "avg_launch_ms": ms[1], "avg_leaves_per_launch": leaves,
                       "flop_per_eval": fpe, "achieved_TFLOP/s": tf,
                       "frac": tf / BF16_PEAK_TFLOPS if tf else None},
           "kernel_ms": {"select_leaf": ms[0], "forward": ms[1], "expand": ms[2]}}
    out["record"] = chess_record(args.chess_record)
    if dist_world == 1 and args.chess_cpu_seconds > 0:
        # the CPU reference path on the same window's shape: the chess oracle's tree loop
        # (AoS arena, a full State per node, sequential descent) + libtorch CPU fp32 20x256,
        # from the start position, run in a subprocess (torch never enters this process)
        ns = argparse.Namespace(cpu_seconds=args.chess_cpu_seconds, cpu_games=args.chess_cpu_games, blocks=blocks,
                                seed=args.seed, cpu_threads=0)
        c = cb.run_cpu_baseline(ns)
        out["cpu_baseline"] = c
        if c.get("value"):
            out["vs_cpu"] = out["sims_per_sec"] / c["value"]
    return out


def chess_record(path):
    """the committed full-game record of BASELINE config 4 (scripts/chess_bench.py --full,
    profiles/r06/chess_full): games/s and sims/s of 2 x 1024 games played to completion at
    400 sims/move, lockstep and streamed, flagged with the commit it was taken at"""
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    rec["source"] = os.path.relpath(path, REPO)
    return rec


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`bench.py --gpus N` without a launcher: start N rank processes of this same
    command (rank r on GPU r), rank 0's stdout to ours, the others' to our stderr.
    This process never imports the library or touches a GPU.  If a rank fails the
    others are stopped (a rank blocked in a barrier would otherwise wait forever).
    Returns the worst exit status."""
    port, group_port = _free_port(), _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPAI_GROUP_PORT=str(group_port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):
                break
            time.sleep(0.2)
    finally:
        own = list(rcs)   # exit statuses the ranks reached on their own
        for r, p in enumerate(procs):
            if rcs[r] is None:
                p.terminate()
                try:
                    rcs[r] = p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    rcs[r] = p.wait()
    if all(rc == 0 for rc in rcs):
        return 0
    print("bench.py: rank exit status %s" % rcs, file=sys.stderr)
    failed = [rc for rc in own if rc not in (None, 0)]
    return failed[0] if failed and failed[0] > 0 else 1


class _StdoutToStderr:
    """C-level stdout (fd 1) to stderr for a block: RCCL prints its version banner
    to stdout at communicator creation, and rank 0's stdout must hold exactly one
    JSON line"""

    def __enter__(self):
        import ctypes
        self.libc = ctypes.CDLL(None)
        sys.stdout.flush()
        self.libc.fflush(None)
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        self.libc.fflush(None)
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def rccl_comm(dist, spai):
    """an RCCL communicator over the ranks' devices (rank 0's id through the host
    group); None with a reason when the ranks share a device (RCCL refuses that) or
    when it could not be formed on every rank.  spai_comm_create is non-blocking with
    a bounded wait (SPAI_COMM_TIMEOUT_S), so a rank whose peer failed gets an error
    back instead of hanging in ncclCommInitRank; the ranks then agree over the host
    group, and without a communicator on every rank none uses one (the host group
    carries the reductions either way)."""
    devs = dist.g.allgather(dist.local)
    if len(set(devs)) != len(devs):
        return None, "ranks share device(s) %s: RCCL needs one rank per GPU; host group only" % devs
    comm, err = None, None
    try:
        with _StdoutToStderr():
            uid = dist.g.broadcast_bytes(spai.comm_unique_id() if dist.rank == 0 else None)
            comm = spai.Comm(dist.local, dist.rank, dist.world, uid)
    except Exception as ex:
        err = "rank %d: %r" % (dist.rank, ex)
    errs = [e for e in dist.g.allgather(err)] if dist.world > 1 else [err]
    if any(errs):
        if comm is not None:
            with _StdoutToStderr():
                comm.close()
        return None, "RCCL communicator failed (%s); host group only" % "; ".join(e for e in errs if e)
    return comm, None


def host_cpus():
    """CPUs this process may use: its affinity mask and the cgroup v2 quota"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


# host cores one rank keeps busy (profiles/r06/host_sync): ~1.9 with the HIP runtime
# spinning on its waits, ~1.1 with the waits sleeping (SPAI_BLOCKING_SYNC, -0.3 % sims/s)
SPIN_CORES_PER_RANK = 2.0


def host_sync_mode(local_world, cpus):
    """spin-wait on the device (the faster default) unless the ranks on this node would
    then keep more than 3/4 of the host cores the process may use busy (the rest is
    headroom for the HIP runtime's threads and the host group); an explicit
    SPAI_BLOCKING_SYNC wins"""
    if "SPAI_BLOCKING_SYNC" in os.environ:
        return "blocking" if os.environ["SPAI_BLOCKING_SYNC"] not in ("", "0") else "spin"
    return "blocking" if SPIN_CORES_PER_RANK * local_world > 0.75 * cpus else "spin"


def stream_base(first, k, world, rank, G):
    """first game id of rank `rank`'s stream of k steps' games starting at step
    `first`: the ranks' ranges [(first * world + rank * k) * G, + k * G) tile
    [first * world * G, (first + k) * world * G) without overlap (world 1: the
    ids of lockstep steps first .. first + k - 1)"""
    return (first * world + rank * k) * G


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline(args)
        return
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks"
                 % (args.gpus, os.environ["WORLD_SIZE"]))
    dist = Dist()
    # the host-core budget of a node's ranks: each rank's host loop spins on
    # its device waits (~1.9 cores); when the ranks of this node would need more cores than
    # the process may use, the waits sleep instead (~1.1 cores).  Set before the first
    # device use in this process, which is when the library reads it.
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", dist.world))
    cpus = host_cpus()
    sync_mode = host_sync_mode(local_world, cpus)
    os.environ["SPAI_BLOCKING_SYNC"] = "1" if sync_mode == "blocking" else "0"
    import spai

    eng = spai.Engine(num_searches=args.sims, max_trees=args.games, eval_kind=spai.EVAL_NET, device=dist.local,
                      seed=args.seed)
    net = spai.Net(eng, args.blocks, spai.init_params(args.blocks, 64, seed=args.seed))
    eng.set_net(net)
    comm, comm_note = rccl_comm(dist, spai)
    G = args.games

    def step(i):
        base = (i * dist.world + dist.rank) * G
        _, st = eng.self_play(G, game_id_base=base, collect=False)
        return st

    def stream(first, k):
        """k steps' worth of games through G tree slots (stream_base)"""
        base = stream_base(first, k, dist.world, dist.rank, G)
        _, st = eng.self_play(k * G, game_id_base=base, collect=False, window=G)
        return st

    streaming = not args.lockstep
    if streaming:
        if args.warmup:
            stream(-args.warmup, args.warmup)
    else:
        for i in range(args.warmup):
            step(-1 - i)
    eng.sync()
    dist.barrier()
    # HIP events on every 32nd search iteration of each chain: ~0.6 % overhead (every
    # 4th measured ~5 %: 31.9M vs 33.4M sims/s), ~1000 sampled launches per step
    eng.set_timing(not args.no_timing, stride=32)
    tot = dict(sims=0.0, games=0.0, evals=0.0, positions=0.0, moves=0.0)
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    if streaming:
        st = stream(0, args.steps)
        for k in tot:
            tot[k] += st[k]
    else:
        for i in range(args.steps):
            st = step(i)
            for k in tot:
                tot[k] += st[k]
    eng.sync()
    t_own = time.perf_counter() - t0   # this rank's own work, before it waits for the others
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    dist.barrier()
    dt = time.perf_counter() - t0
    timing = eng.timing()
    # host CPU time of this rank's process (every thread: the self-play host loop, the HIP
    # runtime's) over the timed region: the host-core budget per GPU
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    per_rank = dist.g.allgather({"rank": dist.rank, "device": dist.local, "wall_s": t_own, "sims": tot["sims"],
                                 "games": tot["games"], "sims_per_sec": tot["sims"] / t_own,
                                 "host_cpu_s": cpu_s, "host_cpu_share": cpu_s / t_own})
    (dt_max,) = dist.reduce([dt], "max")
    counters = [tot["sims"], tot["games"], tot["evals"], tot["positions"]]
    sims, games, evals, positions = dist.reduce(counters, "sum")
    rccl = {"ranks": 0, "note": comm_note}
    if comm is not None:   # the same reductions over RCCL (xGMI between GPUs): exact for these integer counts
        r_sum = r_max = err = None
        try:
            with _StdoutToStderr():
                r_sum = comm.allreduce(counters, "sum")
                (r_max,) = comm.allreduce([dt], "max")
        except Exception as ex:   # bounded inside the library: a failed or absent peer returns an error
            err = "rank %d: %r" % (dist.rank, ex)
        errs = dist.g.allgather(err) if dist.world > 1 else [err]
        if any(errs):
            rccl = {"ranks": 0, "note": "RCCL all-reduce failed (%s); host group only" % "; ".join(e for e in errs if e)}
        else:
            rccl = {"ranks": comm.info()[1], "devices": dist.g.allgather(dist.local),
                    "counters_agree": r_sum == [sims, games, evals, positions] and r_max == dt_max}
        with _StdoutToStderr():
            comm.close()

    fpe = flops_per_eval(args.blocks)
    ev = timing["evaluate"]
    achieved = fpe * ev["items"] / (ev["total_ms"] * 1e-3) / 1e12 if ev["total_ms"] > 0 else None
    per_launch_flop = fpe * ev["items"] / ev["launches"] if ev["launches"] else None
    traffic, traffic_src, pmc = None, None, None
    if os.path.exists(args.pmc_json):   # rocprofv3 --pmc passes of this command (scripts/gpu_roofline_pmc.sh)
        with open(args.pmc_json) as f:
            pmc = json.load(f)
        kf = pmc.get("k_forward<false>", {})
        if "hbm_bytes_per_launch" in kf:
            traffic = kf["hbm_bytes_per_launch"]
            traffic_src = ("%s: (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch over %d launches (FETCH doubled for "
                           "gfx950), commit %s" % (os.path.relpath(args.pmc_json, REPO), kf["launches"],
                                                  pmc.get("commit", "?")))
    if traffic is None and os.path.exists(args.traffic_json):   # measured by separate rocprofv3 --pmc passes of this command
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if "k_forward<false>" in tj:
            traffic = tj["k_forward<false>"]["hbm_bytes_per_launch"]
            traffic_src = ("%s: (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch over %d launches "
                           "(FETCH doubled for gfx950)" % (os.path.relpath(args.traffic_json, REPO),
                                                           tj["k_forward<false>"]["launches"]))
    executed = None
    if pmc and "derived" in pmc:
        d = pmc["derived"]
        frac_job = evals / dt_max * fpe / 1e12 / dist.world / BF16_PEAK_TFLOPS
        executed = {
            "executed_over_algorithmic": d["executed_over_algorithmic"],
            # the job-level rate in the FLOPs the MFMA pipe actually executes (tap skipping drops the
            # MFMAs of all-off-board (tile, tap) pairs; padding rows add some)
            "executed_flop_frac": frac_job * d["executed_over_algorithmic"],
            "mfma_busy": d["mfma_busy"],
            "mfma_insts_per_launch": d["mfma_insts_per_launch"],
            "wave_cycles": d.get("wave_cycles"),
            "source": "%s (commit %s): SQ_INSTS_MFMA x 16*16*32*2 per k_forward launch over the launch's "
                      "algorithmic FLOPs (its leaves x flop_per_eval); mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / "
                      "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) per launch under rocprofv3 (kernels serialised)"
                      % (os.path.relpath(args.pmc_json, REPO), pmc.get("commit", "?"))}
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
        "config": {"workload": "Connect4 self-play, %d games/GPU x %d sims/move, %dx64 ResNet bf16, to completion%s"
                               % (G, args.sims, args.blocks,
                                  (", %d games streamed through %d tree slots" % (G * args.steps, G))
                                  if streaming else ", one lockstep batch per step"),
                   "model": "c4-resnet-%dx64" % args.blocks, "games_per_gpu": G, "sims_per_move": args.sims,
                   "global_batch": G * dist.world, "parallelism": "dp%d (games sharded, no collective)" % dist.world},
        "work": {"sims": sims, "games": games, "evals": evals, "positions": positions},   # summed over ranks
        "schedule": "streamed" if streaming else "lockstep",
        "rccl_ranks": rccl["ranks"],
        "rccl": rccl,
        "per_rank": per_rank,
        "host": {"cpu_s_per_rank_max": max(r["host_cpu_s"] for r in per_rank),
                 "cpu_share_per_rank_max": max(r["host_cpu_share"] for r in per_rank),
                 "cores_per_node_at_8_ranks": 8 * max(r["host_cpu_share"] for r in per_rank),
                 "sims_per_sec_rank_spread": (max(r["sims_per_sec"] for r in per_rank) /
                                              min(r["sims_per_sec"] for r in per_rank)),
                 "sync": sync_mode, "cpus_available": cpus, "ranks_on_node": local_world,
                 "note": "host CPU seconds (getrusage of each rank process: user + system, all threads) over the "
                         "timed region; share = CPU seconds / the rank's own wall time, i.e. host cores busy per GPU; "
                         "sync = how the ranks wait on their devices (spin, or sleep when %g cores x ranks exceed "
                         "3/4 of the CPUs the process may use)" % SPIN_CORES_PER_RANK},
        "evals_per_sec": evals / dt_max,
        "positions_per_sec": positions / dt_max,
        "kernel_ms": {k: v["avg_ms"] for k, v in timing.items()},
        "roofline": {"bound": "mfma", "kernel": "k_forward (fused 6x64 ResNet)",
                     # job level: every forward FLOP of the timed region over its wall time
                     "achieved": evals / dt_max * fpe / 1e12 / dist.world, "peak": BF16_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": evals / dt_max * fpe / 1e12 / dist.world / BF16_PEAK_TFLOPS,
                     "basis": "job level: flop_per_eval x leaves evaluated in the timed region / its wall time, "
                              "per GPU (the two search chains' forwards overlap, so per-launch event times "
                              "over-count the step; see per_launch)",
                     "executed": executed,
                     "traffic": traffic,
                     "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     # algorithmic bytes of one launch: the packed bf16 weights + fp32 biases once,
                     # plus per leaf 16 B of bitboards in and 36 B (8 priors + value) out
                     "algorithmic_bytes": weight_bytes(args.blocks) + 52 * (ev["items"] / max(1, ev["launches"])),
                     "flop_per_launch": per_launch_flop, "flop_per_eval": fpe,
                     "avg_launch_ms": ev["avg_ms"], "avg_leaves_per_launch": ev["items"] / max(1, ev["launches"]),
                     # per launch: HIP events on the chain streams (every 32nd iteration); the
                     # CUs are shared with the other chain's kernels while a launch runs
                     "per_launch": {"achieved": achieved,
                                    "frac": achieved / BF16_PEAK_TFLOPS if achieved else None,
                                    "avg_launch_ms": ev["avg_ms"], "launches_sampled": ev["launches"],
                                    "note": "shared CUs: launches x avg_launch_ms exceeds the step time"}},
    }
    # the lockstep schedule beside the streamed headline: one step of G games started
    # together (game ids after the timed region's), rank 0 of a 1-rank run
    if streaming and not args.no_lockstep_ref:   # every rank, its own game ids after the timed region's
        eng.set_timing(False)
        eng.sync()
        dist.barrier()
        t1 = time.perf_counter()
        ls = step(args.steps)
        eng.sync()
        dist.barrier()
        (d1,) = dist.reduce([time.perf_counter() - t1], "max")
        ls_sims, ls_games, ls_evals = dist.reduce([ls["sims"], ls["games"], ls["evals"]], "sum")
        result["lockstep"] = {"value": ls_sims / d1, "games_per_sec": ls_games / d1, "ms_per_step": d1 * 1e3,
                              "frac": ls_evals / d1 * fpe / 1e12 / dist.world / BF16_PEAK_TFLOPS, "steps": 1,
                              "n_gpus": dist.world,
                              "note": "one batch of %d games per GPU started together and played to completion "
                                      "(the reference worker's schedule; bench.py --lockstep times K of these); "
                                      "summed over ranks, max time" % G}
    # the same forward launch ALONE on the GPU (spai_net_bench, HIP events, random reachable
    # positions) at the timed region's mean leaves per launch, at one chain's (x2) and at the
    # full-batch sizes: the isolated-kernel roofline beside the shared-CU per-launch figure above
    if dist.rank == 0 and not args.no_isolated:
        iso = {}
        mean_leaves = int(round(ev["items"] / max(1, ev["launches"])))
        net.bench(G, iters=1500)   # ~0.2 s of launches first: time at the clock the GPU holds under load
        for n in sorted({max(1, mean_leaves), max(1, 2 * mean_leaves), G // 2, G}):
            ms = net.bench(n, iters=300)
            tf = fpe * n / (ms * 1e-3) / 1e12
            iso[str(n)] = {"ms": ms, "TFLOP/s": tf, "frac": tf / BF16_PEAK_TFLOPS}
        # the timed region's configuration: a chain's forward at the mean leaves with the
        # group size the search picks for two chains sharing the CUs (group_size_conc)
        n = max(1, mean_leaves)
        ms = net.bench(n, iters=300, conc=2)
        tf = fpe * n / (ms * 1e-3) / 1e12
        iso["%d@conc2" % n] = {"ms": ms, "TFLOP/s": tf, "frac": tf / BF16_PEAK_TFLOPS}
        result["roofline"]["isolated"] = iso
        result["roofline"]["isolated_note"] = ("k_forward alone on the GPU at N leaves per launch (spai_net_bench: "
                                               "300 back-to-back launches between HIP events, after ~0.2 s of "
                                               "warm-up launches) at the one-chain group size; 'N@conc2' at the "
                                               "group size the timed region's two chains use (spai_net_bench_conc); "
                                               "the timed region's per-launch figure shares the CUs with the other "
                                               "search chain")
    if not args.no_rules_bench and dist.rank == 0:
        result["rules_kernels"] = rules_bench(eng)
    net.close()
    eng.close()
    if not args.no_chess and dist.rank == 0:
        try:
            result["chess"] = chess_window(args, dist.local, dist.world)
        except Exception as ex:   # the window must never sink the headline number
            result["chess"] = {"error": repr(ex)[:300]}
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        cb = run_cpu_baseline(args)
        result["cpu_baseline"] = cb
        # BASELINE.md publishes no number for this metric: the ratio is against the CPU
        # reference path on whole games (same unit, sims/s over games played to
        # completion), measured in this run at the reference worker's batch of 100
        # games; the committed 256-game record is reported beside it, not used
        if cb.get("value"):
            result["vs_baseline"] = result["value"] / cb["value"]
            result["vs_cpu_games_per_sec"] = result["games_per_sec"] / cb["games_per_sec"]
            result["vs_baseline_basis"] = (
                "whole-game sims/s over the CPU reference path's whole-game sims/s measured in this run "
                "(%d games, %.0f sims/s, %.3f games/s)" % (args.cpu_games, cb["value"], cb["games_per_sec"]))
    if dist.rank == 0:
        print(json.dumps(result), flush=True)
    dist.close()


if __name__ == "__main__":
    main()

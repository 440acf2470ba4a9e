"""BASELINE config 3: Connect4 self-play sharded over N GPUs with a data-parallel
device learner whose gradients are all-reduced with RCCL every round of games,
and the refreshed weights broadcast back to every self-play replica.

One process per GPU (python -m torch.distributed.run ... scripts/c3_selfplay_dp.py),
each rank owning one engine, one bf16 self-play net and one fp32 learner.  A
round is learner_concurrent.rs's loop restated for N ranks:

  self-play  SelfPlayWorker::self_play (learner_concurrent.rs:169-242) over this
             rank's G games, ids (round * world + rank) * G ..: no collective;
  sample     a `fraction` subsample of the finished games' positions
             (choose_multiple, learner_concurrent.rs:280-285) into this rank's ring;
  train      K steps of ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85)
             on B samples per rank: RCCL all-reduce of the fp32 gradients (1.9 MB
             for 6x64) inside every step, exact for unequal per-rank batches;
  refresh    RCCL broadcast of rank 0's parameters (the trainer -> self-play
             weight hand-off, learner_concurrent.rs:158-159,260-264), then every
             rank rebuilds its bf16 self-play net from them.

Rank 0 prints one JSON line: self-play sims/s and games/s over all ranks (the
self-play phase only, max over ranks), learner samples/s, the seconds of each
phase and whether the replicas ended bit-identical (sha256 of the parameters).
At N=1 the learner still gets a 1-rank RCCL communicator, so the all-reduce and
the broadcast run through RCCL.  Host-side barrier/reductions: hostgroup.py.
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "self-play-ai_amd"))
import numpy as np  # noqa: E402

import spai  # noqa: E402
from hostgroup import HostGroup  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096, help="self-play games per GPU per round")
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--train-steps", type=int, default=20, help="learner steps per round (TrainingArgs: 20 batches)")
    ap.add_argument("--batch", type=int, default=128, help="samples per rank per step")
    ap.add_argument("--fraction", type=float, default=0.3, help="subsample of each round's positions")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    g = HostGroup()
    rank, world = g.rank, g.world
    local = int(os.environ.get("SPAI_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    eng = spai.Engine(num_searches=a.sims, max_trees=a.games, eval_kind=spai.EVAL_NET, device=local, seed=a.seed)
    params = spai.init_params(a.blocks, 64, seed=a.seed)   # same init on every rank
    learner = spai.Learner(eng, a.blocks, params)
    uid = g.broadcast_bytes(spai.comm_unique_id() if rank == 0 else None) if world > 1 else spai.comm_unique_id()
    learner.set_comm(rank, world, uid)
    rng = np.random.default_rng([a.seed, rank])
    ring_s, ring_p, ring_v = [], [], []
    tot = dict(sims=0.0, games=0.0, positions=0.0, samples=0.0)
    t_sp = t_train = t_refresh = 0.0
    loss = None
    g.barrier()
    t_all = time.perf_counter()
    for r in range(a.rounds):
        net = spai.Net(eng, a.blocks, params)
        eng.set_net(net)
        t0 = time.perf_counter()
        games, st = eng.self_play(a.games, game_id_base=(r * world + rank) * a.games)
        t_sp += time.perf_counter() - t0
        for k in ("sims", "games", "positions"):
            tot[k] += st[k]
        enc = np.concatenate([x["enc"] for x in games])
        pol = np.concatenate([x["policy"] for x in games])
        val = np.concatenate([x["value"] for x in games])
        keep = rng.choice(len(val), max(a.batch, int(a.fraction * len(val))), replace=False)
        ring_s.append(enc[keep])
        ring_p.append(pol[keep])
        ring_v.append(val[keep])
        S, P, V = np.concatenate(ring_s), np.concatenate(ring_p), np.concatenate(ring_v)
        g.barrier()
        t0 = time.perf_counter()
        for _ in range(a.train_steps):
            idx = rng.choice(len(V), a.batch, replace=False)
            loss = learner.train_batch(S[idx], P[idx], V[idx])
        t_train += time.perf_counter() - t0
        tot["samples"] += a.train_steps * a.batch
        t0 = time.perf_counter()
        learner.broadcast(0)
        params = learner.params()
        t_refresh += time.perf_counter() - t0
        net.close()
    g.barrier()
    wall = time.perf_counter() - t_all
    sp_max, tr_max, rf_max, wall_max = g.allreduce([t_sp, t_train, t_refresh, wall], "max")
    sims, ngames, pos, samples = g.allreduce([tot["sims"], tot["games"], tot["positions"], tot["samples"]], "sum")
    digests = g.allgather(hashlib.sha256(params.tobytes()).hexdigest())
    if rank == 0:
        print(json.dumps({
            "config": "C3: Connect4 %d games/GPU x %d sims/move, %dx64 net, %d GPUs, %d rounds" %
                      (a.games, a.sims, a.blocks, world, a.rounds),
            "n_gpus": world, "rounds": a.rounds,
            "selfplay_sims_per_sec": sims / sp_max, "selfplay_games_per_sec": ngames / sp_max,
            "positions": pos, "train_samples_per_sec": samples / tr_max if tr_max > 0 else None,
            "train_steps_per_round": a.train_steps, "batch_per_rank": a.batch,
            "seconds": {"selfplay": sp_max, "train": tr_max, "refresh": rf_max, "wall": wall_max},
            "collectives": "RCCL all-reduce of %d fp32 gradients per train step; RCCL broadcast of the "
                           "parameters per round" % learner.n,
            "last_loss": [float(v) for v in loss] if loss is not None else None,
            "replicas_identical": len(set(digests)) == 1}), flush=True)
    learner.close()
    eng.close()
    g.close()


if __name__ == "__main__":
    main()

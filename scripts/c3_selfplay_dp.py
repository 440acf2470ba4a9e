"""BASELINE config 3: Connect4 self-play sharded over N GPUs with a data-parallel
device learner whose gradients are all-reduced with RCCL every round of games,
and the refreshed weights broadcast back to every self-play replica.

One process per GPU (python -m torch.distributed.run ... scripts/c3_selfplay_dp.py),
each rank owning one engine, one bf16 self-play net and one fp32 learner.  A
round is learner_concurrent.rs's loop restated for N ranks:

  self-play  SelfPlayWorker::self_play (learner_concurrent.rs:169-242) over this
             rank's G games, ids (round * world + rank) * G ..: no collective;
  sample     (positions as f32 * 0.3) as usize of the finished positions
             (choose_multiple, learner_concurrent.rs:278-283) into this rank's
             replay ring (HeapRb of batch * 100, push_iter_overwrite);
  train      K steps of ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85)
             on the ring's oldest B samples per rank (pop_iter().take(B)): RCCL
             all-reduce of the fp32 gradients (1.9 MB for 6x64) inside every step,
             exact for unequal per-rank batches;
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
import spai  # noqa: E402
from hostgroup import HostGroup  # noqa: E402
from selfplay_dp import Config3Rank  # noqa: E402


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
    uid = g.broadcast_bytes(spai.comm_unique_id() if rank == 0 else None) if world > 1 else spai.comm_unique_id()
    R = Config3Rank(rank, world, uid, games=a.games, sims=a.sims, blocks=a.blocks, batch=a.batch,
                    train_steps=a.train_steps, fraction=a.fraction, seed=a.seed, device=local, group=g)
    loss = None
    g.barrier()
    t_all = time.perf_counter()
    for _ in range(a.rounds):
        _, _, loss, _ = R.run_round()
    g.barrier()
    wall = time.perf_counter() - t_all
    t = R.seconds
    sp_max, tr_max, rf_max, wall_max = g.allreduce([t["selfplay"], t["train"], t["refresh"], wall], "max")
    tot = R.totals
    sims, ngames, pos, samples = g.allreduce([tot["sims"], tot["games"], tot["positions"], tot["samples_trained"]],
                                             "sum")
    digests = g.allgather(hashlib.sha256(R.params.tobytes()).hexdigest())
    if rank == 0:
        print(json.dumps({
            "config": "C3: Connect4 %d games/GPU x %d sims/move, %dx64 net, %d GPUs, %d rounds" %
                      (a.games, a.sims, a.blocks, world, a.rounds),
            "n_gpus": world, "rounds": a.rounds,
            "selfplay_sims_per_sec": sims / sp_max, "selfplay_games_per_sec": ngames / sp_max,
            "positions": pos, "train_samples_per_sec": samples / tr_max if tr_max > 0 else None,
            "train_steps_per_round": a.train_steps, "steps_trained": tot["steps_trained"],
            "steps_skipped": tot["steps_skipped"], "batch_per_rank": a.batch,
            "seconds": {"selfplay": sp_max, "train": tr_max, "refresh": rf_max, "wall": wall_max},
            "collectives": "RCCL all-reduce of %d fp32 gradients per train step; RCCL broadcast of the "
                           "parameters per round" % R.learner.n,
            "last_loss": [float(v) for v in loss] if loss is not None else None,
            "replicas_identical": len(set(digests)) == 1}), flush=True)
    R.close()
    g.close()


if __name__ == "__main__":
    main()

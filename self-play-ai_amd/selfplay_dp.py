"""BASELINE config 3, one rank: sharded Connect4 self-play feeding a data-parallel
device learner, its gradients all-reduced with RCCL, its weights broadcast back
to the self-play net.  Shared by scripts/c3_selfplay_dp.py (the N-GPU driver)
and tests/test_configs_gpu.py (the 1-GPU slice).

One round is learner_concurrent.rs's loop restated for N ranks:

  self-play  SelfPlayWorker::self_play (learner_concurrent.rs:169-242) over this
             rank's G games, ids (round * world + rank) * G ..: no collective;
  sample     choose_multiple of (positions as f32 * 0.3) as usize of the
             finished positions (:278-283), pushed into this rank's replay ring
             (HeapRb of batch * 100, main.rs:142; push_iter_overwrite);
  train      K steps of ModelTrainerWorker::train_batch (:72-85) on the oldest
             B samples of the ring (pop_iter().take(B), :94-101): RCCL all-reduce
             of the fp32 gradients inside every step;
  refresh    RCCL broadcast of rank 0's parameters (the trainer -> self-play
             weight hand-off, :158-159,260-264), then the bf16 self-play net is
             rebuilt from them.
"""
import time

import numpy as np

import spai


class Config3Rank:
    def __init__(self, rank, world, uid, games=4096, sims=800, blocks=6, batch=128, train_steps=20, fraction=0.3,
                 capacity=None, seed=0, device=0, group=None):
        self.rank, self.world = rank, world
        # host group (hostgroup.HostGroup): agrees the step count over ranks.  Every
        # train step is a collective, so ranks that counted their own ring sizes
        # could issue different numbers of them and hang: required when world > 1
        if world > 1 and group is None:
            raise ValueError("Config3Rank: world %d needs a host group to agree the train steps" % world)
        self.group = group
        self.games, self.sims, self.blocks = games, sims, blocks
        self.batch, self.train_steps, self.fraction, self.seed = batch, train_steps, fraction, seed
        self.eng = spai.Engine(num_searches=sims, max_trees=games, eval_kind=spai.EVAL_NET, device=device, seed=seed)
        self.params = spai.init_params(blocks, 64, seed=seed)   # same init on every rank
        self.learner = spai.Learner(self.eng, blocks, self.params)
        self.learner.set_comm(rank, world, uid)
        self.ring = spai.Replay(capacity or batch * 100)
        self.round_no = 0
        self.net = None
        self.totals = dict(sims=0.0, games=0.0, positions=0.0, samples_pushed=0.0, samples_trained=0.0,
                           steps_trained=0.0, steps_skipped=0.0)
        self.seconds = dict(selfplay=0.0, train=0.0, refresh=0.0)

    def run_round(self, collect_games=False):
        """one round; returns (games or None, self-play stats, last loss, pushed)"""
        r = self.round_no
        if self.net is None:
            self.net = spai.Net(self.eng, self.blocks, self.params)
            self.eng.set_net(self.net)
        t0 = time.perf_counter()
        games, st = self.eng.self_play(self.games, game_id_base=(r * self.world + self.rank) * self.games)
        self.seconds["selfplay"] += time.perf_counter() - t0
        for k in ("sims", "games", "positions"):
            self.totals[k] += st[k]
        enc = np.concatenate([x["enc"] for x in games])
        pol = np.concatenate([x["policy"] for x in games])
        val = np.concatenate([x["value"] for x in games])
        k = int(np.float32(len(val)) * np.float32(self.fraction))      # (len as f32 * 0.3) as usize
        keep = spai.choose_multiple(len(val), k, seed=self.seed, stream=(self.rank << 32) | r).astype(np.int64)
        self.ring.push(enc[keep], pol[keep], val[keep])
        self.totals["samples_pushed"] += k
        t0 = time.perf_counter()
        loss = None
        # The reference trainer blocks until a batch is buffered (Condvar::wait_while,
        # learner_concurrent.rs:94-101); a round-synchronous rank cannot wait for samples
        # that only the next round produces, so it trains the steps every rank can fill
        # (the minimum over ranks: each step is a collective) and counts the rest as skipped
        steps = min(self.train_steps, len(self.ring) // self.batch)
        if self.group is not None and self.world > 1:
            steps = int(-self.group.allreduce([-steps], "max")[0])
        for _ in range(steps):
            s, p, v = self.ring.pop(self.batch)
            loss = self.learner.train_batch(s, p, v)
        self.seconds["train"] += time.perf_counter() - t0
        self.totals["samples_trained"] += steps * self.batch
        self.totals["steps_trained"] += steps
        self.totals["steps_skipped"] += self.train_steps - steps
        t0 = time.perf_counter()
        self.learner.broadcast(0)
        self.params = self.learner.params()
        self.net.close()
        self.net = spai.Net(self.eng, self.blocks, self.params)
        self.eng.set_net(self.net)
        self.seconds["refresh"] += time.perf_counter() - t0
        self.round_no += 1
        return (games if collect_games else None), st, loss, k

    def close(self):
        if self.net is not None:
            self.net.close()
        self.ring.close()
        self.learner.close()
        self.eng.close()

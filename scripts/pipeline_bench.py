"""train_concurrent (main.rs:137-235) on the device: self-play workers + learner
over the replay ring (spai_pipeline_run).  Reference defaults (100 games x 600
sims per self-play batch, batch 128, 20 batches x 10 iterations, ring 12,800,
30 % subsample, 4 blocks) unless overridden.  Prints one JSON line.

  python scripts/pipeline_bench.py [--selfplay-devices 0,1,...] [--learner-device 7] [--games 100] ...
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "self-play-ai_amd"))
import spai  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--selfplay-devices", default="0")
    ap.add_argument("--learner-device", type=int, default=0)
    ap.add_argument("--games", type=int, default=100)
    ap.add_argument("--sims", type=int, default=600)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--batches-per-iter", type=int, default=20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--capacity", type=int, default=12800)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--checkpoint-dir", default=None)
    a = ap.parse_args()
    devs = tuple(int(d) for d in a.selfplay_devices.split(","))
    st = spai.pipeline_run(spai.init_params(a.blocks, 64, seed=a.seed), selfplay_devices=devs,
                           learner_device=a.learner_device, checkpoint_dir=a.checkpoint_dir, games_per_batch=a.games,
                           num_searches=a.sims, batch_size=a.batch, batches_per_iter=a.batches_per_iter,
                           train_iters=a.iters, replay_capacity=a.capacity, blocks=a.blocks, seed=a.seed)
    st.update(selfplay_devices=list(devs), learner_device=a.learner_device, games_per_batch=a.games, sims=a.sims,
              batch=a.batch, blocks=a.blocks, games_per_sec=st["games"] / st["seconds"],
              trained_samples_per_sec=st["batches_trained"] * a.batch / st["seconds"],
              # every live tree searches every move: sims = positions x sims per move
              selfplay_sims_per_sec=st["positions"] * a.sims / st["seconds"],
              workers=len(devs))
    print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main()

"""Rehearse bench.py's N>1 process layout on one GPU: torch.distributed (gloo)
imported before libspai, then a small NET self-play and a learner step; print
which HIP runtime copies the process mapped."""
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29517")
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo", rank=0, world_size=1)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np  # noqa: E402

import spai  # noqa: E402

e = spai.Engine(num_searches=32, max_trees=64, eval_kind=spai.EVAL_NET, seed=1)
net = spai.Net(e, 6, spai.init_params(6, 64, seed=0))
e.set_net(net)
games, st = e.self_play(64)
print("self-play ok", st["games"], st["sims"])
L = spai.Learner(e, 6, spai.init_params(6, 64, seed=0))
x = np.concatenate([g["enc"] for g in games])[:128]
pi = np.concatenate([g["policy"] for g in games])[:128]
z = np.concatenate([g["value"] for g in games])[:128]
print("learner loss", L.train_batch(x, pi, z))
maps = {l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l}
print("HIP runtimes mapped:", sorted(maps))
L.close()
net.close()
e.close()
dist.destroy_process_group()

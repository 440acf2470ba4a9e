"""Forward-only workload for counter profiling: Model::predict over N random
reachable positions, repeated."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

import spai

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
rng = np.random.default_rng(0)
e.games_resize(n)
for _ in range(12):   # random reachable positions
    lm = e.legal_mask(n)
    r = rng.random((n, 7)) * ((lm[:, None] >> np.arange(7)) & 1)
    e.apply(np.argmax(r, 1).astype(np.int32), check=False)
st = e.games_read(n)
st = st[st["status"] == 0]
for _ in range(reps):
    pr, v = net.predict(st)
print("forward positions", len(st), "reps", reps, "prior sum", float(pr.sum()))

"""Chess search timing on one GPU: T trees from the start position, one move of
S simulations with a B-block 256-channel net (BASELINE config 4 shape by default)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import spai_chess as sc  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--trees", type=int, default=1024)
ap.add_argument("--sims", type=int, default=400)
ap.add_argument("--blocks", type=int, default=20)
ap.add_argument("--moves", type=int, default=1)
a = ap.parse_args()
eng = sc.ChessEngine(num_searches=a.sims, max_trees=a.trees, eval_kind=sc.EVAL_NET)
net = sc.ChessNet(eng, a.blocks, sc.init_params(a.blocks, 0))
eng.set_net(net)
eng.trees_create(a.trees)
eng.search(np.arange(a.trees), num_searches=8)   # warm-up
eng.trees_create(a.trees)
eng.set_timing(True)
t0 = time.perf_counter()
for m in range(a.moves):
    pol, ids, vis, mv, nc = eng.search(np.arange(a.trees))
    if m + 1 < a.moves:
        for t in range(a.trees):
            eng.use_subtree(t, int(np.argmax(vis[t, :nc[t]])))
dt = time.perf_counter() - t0
ms, launches, items = eng.timing()
flop = {20: 3036348928, 10: 1526399488}.get(a.blocks, 0)
leaves = items[1] / max(1, launches[1])
print(json.dumps({"trees": a.trees, "sims": a.sims, "blocks": a.blocks, "moves": a.moves, "seconds": dt,
                  "sims_per_s": a.trees * a.sims * a.moves / dt, "kernel_ms": list(ms), "launches": list(launches),
                  "leaves_per_forward": leaves,
                  "forward_tflops": flop * leaves / (ms[1] * 1e-3) / 1e12 if ms[1] > 0 else None}))

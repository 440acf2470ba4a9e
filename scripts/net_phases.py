"""Print the fused forward's per-phase cycle breakdown (diagnostic stamps)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
names = ["start", "stem"] + ["res%d" % i for i in range(12)] + ["head_conv", "linear", "end"]
for n in (2048, 4096):
    c = net.phase_cycles(n)
    d = np.diff(c)
    print(f"batch {n}: total {c[16]:.0f} cycles/wave = {c[16] / 2.1e3:.1f} us @2.1GHz")
    print("  " + "  ".join(f"{names[k + 1]}={d[k]:.0f}" for k in range(16)))
net.close()
e.close()

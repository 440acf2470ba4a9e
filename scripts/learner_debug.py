"""Per-tensor step-1 gradient error of the device learner vs the torch golden."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "self-play-ai_amd")); sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import numpy as np
import spai, learner_ref as LR
z = np.load(os.path.join(HERE, "..", "tests", "golden", "learner_c4_1x64.npz"))
blocks, hidden, seed, B, K = [int(v) for v in z["meta"]]
e = spai.Engine(num_searches=1, max_trees=1)
L = spai.Learner(e, blocks, spai.init_params(blocks, hidden, seed=seed), hidden=hidden)
L.train_batch(z["states"][0], z["policies"][0], z["values"][0])
g = L.grads(); gr = z["grads1"]
convs, lin, n = LR._layout(blocks, hidden)
names = ["stem"] + ["res%d" % i for i in range(2 * blocks)] + ["pol", "val"]
for nm, c in zip(names, convs):
    for key, ln in (("w", c["co"] * c["ci"] * 9), ("b", c["co"]), ("g", c["co"]), ("be", c["co"])):
        o = c[key]
        d = np.abs(g[o:o + ln] - gr[o:o + ln])
        print(f"{nm:5s} {key:2s} maxerr {d.max():.3e} ref max {np.abs(gr[o:o+ln]).max():.3e} argmax {d.argmax()}")
for key, ln in (("pw", 7 * 1344), ("pb", 7), ("vw", 126), ("vb", 1)):
    o = lin[key]; d = np.abs(g[o:o + ln] - gr[o:o + ln])
    print(f"lin   {key} maxerr {d.max():.3e} ref max {np.abs(gr[o:o+ln]).max():.3e}")

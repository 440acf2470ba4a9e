"""Where does the device learner's first-step gradient differ most from the numpy
float64 restatement?  Prints the largest differences with the parameter they
belong to (construction order: conv w, b, BN gamma, beta, mean, var; linears w, b)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "self-play-ai_amd"), os.path.join(HERE, "..", "oracle"),
                os.path.join(HERE, "..", "tests")]
import numpy as np

import learner_ref as LR
import spai
from test_gpu_parity import _reachable_positions

blocks, B = int(sys.argv[1]) if len(sys.argv) > 1 else 6, int(sys.argv[2]) if len(sys.argv) > 2 else 128
rng = np.random.default_rng(blocks * 100 + B)
states = _reachable_positions(spai, 4 * B, 10, seed=B)
e = spai.Engine(num_searches=1, max_trees=1)
e.games_resize(len(states))
e.games_write(states)
x = e.encode(len(states)).reshape(len(states), 126)[:B]
pi = rng.random((B, 7)).astype(np.float32) ** 2
pi = (pi / pi.sum(1, keepdims=True)).astype(np.float32)
z = rng.choice(np.array([-1, 0, 1], np.float32), B)
p0 = spai.init_params(blocks, 64, seed=blocks + 7)
L = spai.Learner(e, blocks, p0)
L.train_batch(x, pi, z)
g = L.grads()
_, _, ref = LR.train(p0, [(x, pi, z)], blocks, 64)
ref = ref[0]
names = []
def conv(ci, co, tag):
    names.extend([(tag + ".w", co * ci * 9), (tag + ".b", co), (tag + ".bn_g", co), (tag + ".bn_b", co),
                  (tag + ".bn_mu", co), (tag + ".bn_var", co)])
conv(3, 64, "stem")
for i in range(2 * blocks):
    conv(64, 64, "res%d" % i)
conv(64, 32, "pol")
names += [("pol_lin.w", 7 * 1344), ("pol_lin.b", 7)]
conv(64, 3, "val")
names += [("val_lin.w", 126), ("val_lin.b", 1)]
bounds = np.cumsum([0] + [n for _, n in names])
d = np.abs(g - ref)
print("max |g|", np.abs(ref).max(), "tol", 3e-4 * np.abs(ref).max())
for i in np.argsort(-d)[:8]:
    k = np.searchsorted(bounds, i, side="right") - 1
    print("%8d %-12s dev % .6e ref % .6e diff %.3e" % (i, names[k][0], g[i], ref[i], d[i]))
for (nm, n), lo in zip(names, bounds):
    seg = d[lo:lo + n]
    if seg.max() > 1e-4 * np.abs(ref).max():
        print("  %-12s max diff %.3e  max |ref| %.3e" % (nm, seg.max(), np.abs(ref[lo:lo + n]).max()))

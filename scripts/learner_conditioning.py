"""How sensitive is the first-step gradient to fp32-sized rounding?  Runs the
numpy float64 restatement on the learner test's inputs twice, the second time
with every parameter perturbed by a random relative 2^-24 (one fp32 ulp), and
prints max |g - g'| / max |g| beside the parity test's 3e-4 bound.  Large
values mean the case is ill-conditioned (near-constant BN channels: invstd up
to 1/sqrt(eps) amplifies rounding), so any fp32 summation order lands that far
from the float64 answer."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "self-play-ai_amd"), os.path.join(HERE, "..", "oracle"),
                os.path.join(HERE, "..", "tests")]
import numpy as np

import learner_ref as LR
import spai
from test_gpu_parity import _reachable_positions

for cfg in sys.argv[1:] or ["6:128", "2:128", "2:48"]:
    blocks, B = map(int, cfg.split(":"))
    rng = np.random.default_rng(blocks * 100 + B)
    states = _reachable_positions(spai, 4 * B, 10, seed=B)
    e = spai.Engine(num_searches=1, max_trees=1)
    e.games_resize(len(states))
    e.games_write(states)
    x = e.encode(len(states)).reshape(len(states), 126)[:B]
    e.close()
    pi = rng.random((B, 7)).astype(np.float32) ** 2
    pi = (pi / pi.sum(1, keepdims=True)).astype(np.float32)
    z = rng.choice(np.array([-1, 0, 1], np.float32), B)
    p0 = spai.init_params(blocks, 64, seed=blocks + 7).astype(np.float64)
    g = LR.train(p0, [(x, pi, z)], blocks, 64)[2][0]
    prng = np.random.default_rng(1)
    for k in range(3):
        p1 = p0 * (1 + prng.choice([-1.0, 1.0], p0.shape) * 2.0 ** -24)
        g1 = LR.train(p1, [(x, pi, z)], blocks, 64)[2][0]
        print("blocks %d B %d: perturbation %d -> max|dg| / max|g| = %.2e (parity bound 3e-4)"
              % (blocks, B, k, np.abs(g1 - g).max() / np.abs(g).max()), flush=True)

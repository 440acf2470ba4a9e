#!/usr/bin/env python3
"""Generate tests/golden/chess_net_b1.npz: the chess net (model/chess.rs:48-77,
model/mod.rs:152-184) forward in PyTorch CPU fp32 -- the libtorch conv2d /
batch_norm / linear ops that tch 0.13 wraps -- on encodings of positions from
random games of the chess oracle.

Runs in the build container only (needs torch CPU and libspai.so for the
deterministic parameter init spai_chess_net_init_params, a host-only entry
point).  The fixture stores the init seed, the inputs and the outputs; the
parameters are regenerated from the seed by the tests.
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "self-play-ai_amd")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import chessref  # noqa: E402
import spai_chess  # noqa: E402

BLOCKS, SEED = 1, 7


def torch_forward(params, blocks, x):
    P = chessref.unpack_params(params, blocks)
    it = iter(P)

    def nxt():
        return torch.from_numpy(np.ascontiguousarray(next(it)[1]))

    def bn(h):
        g, b, m, v = (torch.from_numpy(np.ascontiguousarray(a)) for a in next(it)[1])
        return F.batch_norm(h, m, v, g, b, training=False, eps=1e-5)

    h = torch.from_numpy(x)
    h = F.relu(bn(F.conv2d(h, nxt(), nxt(), padding=1)))
    for _ in range(blocks):
        y = F.relu(bn(F.conv2d(h, nxt(), nxt(), padding=1)))
        y = bn(F.conv2d(y, nxt(), nxt(), padding=1))
        h = F.relu(h + y)
    p = F.relu(F.conv2d(h, nxt(), nxt()))
    p = F.conv2d(p, nxt(), nxt()).flatten(1)
    v = F.relu(F.conv2d(h, nxt(), nxt())).flatten(1)
    v = F.relu(F.linear(v, nxt(), nxt()))
    v = torch.tanh(F.linear(v, nxt(), nxt()))[:, 0]
    return p.numpy(), v.numpy()


def positions(n, seed=3):
    rng = random.Random(seed)
    out = []
    for g in range(n):
        s = chessref.ChessState()
        for _ in range(rng.randrange(0, 60)):
            mv = s.valid_actions()
            if not mv or s.status != 0:
                break
            s = s.next_state(rng.choice(mv))
        out.append(s.encoding())
    return np.stack(out).astype(np.float32)


def main():
    torch.set_num_threads(8)
    params = spai_chess.init_params(BLOCKS, SEED)
    x = positions(6)
    lg, v = torch_forward(params, BLOCKS, x)
    np.savez_compressed(os.path.join(HERE, "chess_net_b1.npz"), blocks=BLOCKS, seed=SEED, x=x, logits=lg, value=v)
    print("wrote chess_net_b1.npz", x.shape, lg.shape, v)


if __name__ == "__main__":
    main()

"""CPU reference path for the bench's `cpu_baseline`: the
reference's algorithm and data layout timed on the host cores.

TEST / MEASUREMENT INFRASTRUCTURE ONLY: imported by bench.py's cpu_baseline
subprocess and scripts/cpu_games_baseline.py, never by the product path.

* tree loop: the oracle (spai_oracle.c) — AoS node arena with a full State per
  node, one sequential select/expand/backup pass per tree and iteration
  (mcts.rs:214-285), encoding per state (connect_four.rs:242-259);
* Model::predict (model/mod.rs:36-98): ONE batched libtorch CPU fp32 forward
  per search iteration over the live leaves, softmax, then
  mask_invalid_actions — libtorch is the engine tch wraps (tch 0.13 ->
  libtorch 2.0; here PyTorch 2.10's CPU kernels), on `threads` intra-op threads;
* self-play (learner_concurrent.rs:169-242): oracle or_self_play, games run to
  completion with the same Philox move sampling as the device path.
"""
import ctypes as C
import json
import os
import time

import numpy as np

import oracle as O


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs this process may use: the affinity mask and the cgroup v2 quota"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return n


class TorchEval:
    """Model::predict on libtorch CPU fp32 for the C4 net (model/connect_four.rs:50-81)"""

    def __init__(self, blocks, seed, threads, max_batch):
        import torch
        import torch.nn.functional as F
        self.torch, self.F = torch, F
        torch.set_num_threads(threads)
        self.threads = threads
        self.L = O.lib()
        p = torch.from_numpy(O.init_params(O.GAME_CONNECT4, blocks, 64, seed))
        off = [0]

        def take(*shape):
            n = int(np.prod(shape))
            v = p[off[0]:off[0] + n].reshape(shape)
            off[0] += n
            return v

        def cbn(ci, co):
            return [take(co, ci, 3, 3), take(co), take(co), take(co), take(co), take(co)]

        self.stem = cbn(3, 64)
        self.blocks = [(cbn(64, 64), cbn(64, 64)) for _ in range(blocks)]
        self.pol = cbn(64, 32)
        self.pw, self.pb = take(7, 1344), take(7)
        self.val = cbn(64, 3)
        self.vw, self.vb = take(1, 126), take(1)
        self.enc = np.zeros((max_batch, 126), np.float32)
        self.calls = 0
        self.leaves = 0
        self.cb = O.EVAL_FN(self)

    def _conv_bn(self, t, c, relu):
        w, b, g, be, mu, var = c
        t = self.F.batch_norm(self.F.conv2d(t, w, b, padding=1), mu, var, g, be, training=False, eps=1e-5)
        return self.F.relu(t) if relu else t

    def __call__(self, user, n, states, priors, values):
        F, torch = self.F, self.torch
        self.L.or_encode_states(O.GAME_CONNECT4, n, states, self.enc.ctypes.data_as(C.POINTER(C.c_float)))
        with torch.no_grad():
            t = torch.from_numpy(self.enc[:n]).view(-1, 3, 6, 7)
            t = self._conv_bn(t, self.stem, True)
            for c1, c2 in self.blocks:
                t = F.relu(t + self._conv_bn(self._conv_bn(t, c1, True), c2, False))
            lg = F.linear(self._conv_bn(t, self.pol, True).flatten(1), self.pw, self.pb)
            v = torch.tanh(F.linear(self._conv_bn(t, self.val, True).flatten(1), self.vw, self.vb)).view(-1)
            sm = torch.softmax(lg, -1).numpy()
        legal = self.enc[:n].reshape(n, 3, 6, 7)[:, 2, 5, :]
        m = sm * legal
        m /= m.sum(1, keepdims=True)
        np.ctypeslib.as_array(priors, (n, 7))[:] = m
        np.ctypeslib.as_array(values, (n,))[:] = v.numpy()
        self.calls += 1
        self.leaves += n


def sims_window(games, sims, seconds, blocks=6, seed=0, threads=1, max_moves=4):
    """CPU sims/s over whole search iterations of `games` trees from the empty
    board, advancing each tree on its most visited child after every full move,
    until `seconds` or `max_moves` moves have passed"""
    L = O.lib()
    ev = TorchEval(blocks, seed, threads, games)
    trees = [L.or_tree_create(O.GAME_CONNECT4) for _ in range(games)]
    arr = (C.c_void_p * games)(*trees)
    n = games
    pol = np.zeros((n, 7), np.float32)
    ids = np.zeros((n, 7), np.int32)
    vis = np.zeros((n, 7), np.float32)
    nc = np.zeros(n, np.int32)
    t0 = time.perf_counter()
    done_sims, moves = 0, 0
    chunk = 50
    while time.perf_counter() - t0 < seconds and moves < max_moves:
        done = 0
        while done < sims and time.perf_counter() - t0 < seconds:
            k = min(chunk, sims - done)
            L.or_search(arr, n, k, 2.0, O.EVAL_NET, None, ev.cb, None, O._f(pol), O._i(ids), O._f(vis), O._i(nc))
            done += k
            done_sims += n * k
        if done < sims:
            break
        moves += 1
        for i, t in enumerate(trees):
            j = int(np.argmax(vis[i, :nc[i]]))
            L.or_tree_use_subtree(t, int(ids[i, j]))
    dt = time.perf_counter() - t0
    for t in trees:
        L.or_tree_destroy(t)
    return dict(sims_per_sec=done_sims / dt, seconds=dt, sims_done=done_sims, evals=ev.leaves, moves_completed=moves)


def games_to_completion(games, sims, blocks=6, seed=0, threads=1):
    """SelfPlayWorker::self_play on the CPU: `games` games from the empty board
    played to completion at `sims` simulations per move"""
    ev = TorchEval(blocks, seed, threads, games)
    t0 = time.perf_counter()
    r = O.self_play(O.GAME_CONNECT4, games, sims, seed, eval_kind=O.EVAL_NET, eval_fn=ev, max_plies=42)
    dt = time.perf_counter() - t0
    return dict(games=games, games_per_sec=games / dt, sims_per_sec=r["sims"] / dt, seconds=dt,
                sims_done=r["sims"], evals=r["evals"], positions=int(len(r["value"])),
                mean_plies=float(np.mean(r["n_moves"])), max_plies=int(np.max(r["n_moves"])))


if __name__ == "__main__":   # python oracle/refcpu.py <json args>
    import sys
    a = json.loads(sys.argv[1])
    fn = games_to_completion if a.pop("mode") == "games" else sims_window
    print(json.dumps(fn(**a)))

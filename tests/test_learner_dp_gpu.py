"""The data-parallel learner at world > 1 (BASELINE config 3):
the arithmetic every rank runs around the gradient all-reduce of
ModelTrainerWorker::train_batch (learner_concurrent.rs:72-85) under DDP —
each rank's mean gradient weighted by B_rank / sum B (`k_weight_grad`), the
summed gradient into Adam, the BN running statistics averaged (`k_gather`,
`k_scatter_scaled` with 1/world), and the parameter broadcast of the weight
refresh (learner_concurrent.rs:158-159).

RCCL refuses two ranks on one device, so the ranks here reduce through the
learner's host collective (spai_learner_set_host_comm): the same step and the
same kernels, with each all-reduce staged through pinned host memory and summed
by the test — two threads of one process (a barrier group), and two processes
over bench.py's TCP host group.  The result is checked against the float64 DDP
restatement (oracle/learner_ref.py::train_step_dp) with unequal batches (48 + 80).
"""
import os
import socket
import subprocess
import sys
import textwrap
import threading

import numpy as np
import pytest

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spai():
    import spai as s
    assert s.device_count() > 0, "no GPU visible"
    return s


class ThreadGroup:
    """an in-process host collective for `world` learner threads: float32 sums in
    rank order, so every rank gets the same bits (as RCCL's two-rank sum)"""

    def __init__(self, world):
        self.world = world
        self.bufs = [None] * world
        self.bar = threading.Barrier(world)
        self.calls = [0] * world
        self.sizes = []

    def member(self, rank):
        def allreduce(buf):
            self.bufs[rank] = buf.copy()
            self.bar.wait(timeout=120)
            tot = self.bufs[0].copy()
            for r in range(1, self.world):
                tot += self.bufs[r]
            if rank == 0:
                self.sizes.append(len(buf))
            self.bar.wait(timeout=120)
            buf[:] = tot
            self.calls[rank] += 1
        return allreduce


def _in_threads(fns):
    out, errs = [None] * len(fns), []

    def run(i):
        try:
            out[i] = fns[i]()
        except Exception as ex:   # surfaced after the join
            errs.append(ex)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "learner thread hung"
    if errs:
        raise errs[0]
    return out


def _batches(spai, sizes, steps, seed):
    """per rank and step: encoded reachable positions, random policies, outcomes"""
    from test_gpu_parity import _reachable_positions
    n = sum(sizes) * steps
    states = _reachable_positions(spai, 2 * n, 10, seed=seed)[:n]
    assert len(states) == n
    e = spai.Engine(num_searches=1, max_trees=1)
    e.games_resize(n)
    e.games_write(states)
    x = e.encode(n).reshape(n, 126)
    e.close()
    rng = np.random.default_rng(seed)
    pi = rng.random((n, 7)).astype(np.float32) ** 2
    pi = (pi / pi.sum(1, keepdims=True)).astype(np.float32)
    z = rng.choice(np.array([-1, 0, 1], np.float32), n)
    out, o = [], 0
    for _ in range(steps):
        per = []
        for b in sizes:
            per.append((x[o:o + b], pi[o:o + b], z[o:o + b]))
            o += b
        out.append(per)
    return out


def _run_two_ranks(spai, blocks, p_ranks, batches):
    """two learners on device 0, one thread each, reducing through a ThreadGroup;
    returns the learners (open), the group, per-step grads/activations/losses"""
    grp = ThreadGroup(2)
    engines = [spai.Engine(num_searches=1, max_trees=1) for _ in range(2)]
    Ls = [spai.Learner(engines[r], blocks, p_ranks[r]) for r in range(2)]
    for r in range(2):
        Ls[r].set_host_comm(r, 2, grp.member(r))
    # weight refresh first: rank 1 starts from other parameters and must take rank 0's
    _in_threads([lambda L=L: L.broadcast(0) for L in Ls])
    rec = []
    for step in batches:
        losses = _in_threads([lambda r=r: Ls[r].train_batch(*step[r]) for r in range(2)])
        nl = 2 * blocks + 3
        rec.append(dict(loss=losses, grads=[L.grads() for L in Ls],
                        masks=[[L.activation(l) > 0 for l in range(nl)] for L in Ls]))
    return engines, Ls, grp, rec


def test_learner_two_ranks_vs_ddp_restatement(spai):
    """world 2, batches of 48 and 80: the replicas stay bit-identical, the reduced
    gradient is sum_r (B_r / 128) g_r of the float64 DDP restatement run with each
    rank's own ReLU masks (3e-4 max|g|, the single-rank bound), the running
    statistics are the ranks' averaged, and two steps track the restatement's Adam"""
    import learner_ref as LR
    from test_oracle_golden import check_learner_params
    blocks, sizes, steps = 2, (48, 80), 2
    p0 = spai.init_params(blocks, 64, seed=21)
    p_other = spai.init_params(blocks, 64, seed=22)
    batches = _batches(spai, sizes, steps, seed=5)
    engines, Ls, grp, rec = _run_two_ranks(spai, blocks, (p0, p_other), batches)
    # the broadcast made rank 1 equal rank 0's parameters (checked through the step below:
    # both ranks ran from p0 if their reduced gradients agree with the restatement from p0)
    # all-reduces per step: batch size, gradients, running statistics; plus the broadcast
    n = len(p0)
    nr = sum(2 * c for c in [64] * (2 * blocks + 1) + [32, 3])
    assert grp.sizes == [n] + [1, n, nr] * steps, grp.sizes
    P = [L.params() for L in Ls]
    np.testing.assert_array_equal(P[0], P[1])
    P_ref, m, v = np.asarray(p0, np.float64), np.zeros(n), np.zeros(n)
    ref_grads = []
    for k, step in enumerate(batches):
        g_dev = rec[k]["grads"]
        np.testing.assert_array_equal(g_dev[0], g_dev[1])
        diags = [{}, {}]
        P_ref, m, v, losses, G, parts = LR.train_step_dp(P_ref, m, v, k, step, blocks, 64,
                                                         rank_masks=rec[k]["masks"], rank_diags=diags)
        ref_grads.append(G)
        # step 1 starts from identical parameters: the single-rank bounds.  Step 2 starts
        # from the device's Adam step vs the float64 one, which differ by up to lr in the
        # ill-conditioned entries (check_learner_params), so its bounds are 10x looser
        tol = 1e-4 if k == 0 else 1e-3
        for r in range(2):   # device masks may differ only at pre-activations within rounding of 0
            for l, pre in enumerate(diags[r]["pre"]):
                diff = rec[k]["masks"][r][l] != (pre > 0)
                assert np.all(np.abs(pre[diff]) <= tol * np.abs(pre).max()), (k, r, l)
            np.testing.assert_allclose(rec[k]["loss"][r], losses[r], rtol=1e-3, atol=1e-4)
        d, mx = np.abs(g_dev[0] - G), np.abs(G).max()
        assert d.max() <= 3 * tol * mx, (k, d.max() / mx)
        # the weighting matters: the unweighted mean of the two ranks' gradients is far off
        plain = 0.5 * (parts[0] + parts[1])
        assert np.abs(plain - G).max() > 10 * d.max()
    check_learner_params(P[0], P_ref, ref_grads, blocks, 64, steps, tol=1e-4)
    for L in Ls:
        L.close()
    for e in engines:
        e.close()


def test_learner_two_ranks_one_step_params(spai):
    """one world-2 step from equal parameters: parameters (incl. the averaged BN
    running statistics, k_scatter_scaled with 1/world = 0.5) vs the restatement at
    the single-step bounds"""
    import learner_ref as LR
    from test_oracle_golden import check_learner_params
    blocks, sizes = 1, (48, 80)
    p0 = spai.init_params(blocks, 64, seed=31)
    batches = _batches(spai, sizes, 1, seed=6)
    engines, Ls, grp, rec = _run_two_ranks(spai, blocks, (p0, p0), batches)
    n = len(p0)
    P_ref, _, _, _, G, _ = LR.train_step_dp(p0, np.zeros(n), np.zeros(n), 0, batches[0], blocks, 64,
                                            rank_masks=rec[0]["masks"])
    P = Ls[0].params()
    np.testing.assert_array_equal(P, Ls[1].params())
    check_learner_params(P, P_ref, [G], blocks, 64, 1)
    # the running statistics really are the average of two different batches' updates
    P_a, _, _ = LR.forward_backward(p0, *batches[0][0], blocks, 64)
    P_b, _, _ = LR.forward_backward(p0, *batches[0][1], blocks, 64)
    convs, _, _ = LR._layout(blocks, 64)
    sl = slice(convs[0]["mu"], convs[0]["mu"] + 64)
    assert np.abs(P_a[sl] - P_b[sl]).max() > 1e-4
    np.testing.assert_allclose(P[sl], 0.5 * (P_a[sl] + P_b[sl]), rtol=1e-4, atol=1e-6)
    for L in Ls:
        L.close()
    for e in engines:
        e.close()


RANK_WORKER = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, os.path.join({repo!r}, "self-play-ai_amd"))
    import numpy as np
    import spai
    from hostgroup import HostGroup
    g = HostGroup()
    d = np.load({data!r})
    r = g.rank
    e = spai.Engine(num_searches=1, max_trees=1)
    L = spai.Learner(e, int(d["blocks"]), d["p0"] if r == 0 else d["p_other"])
    L.set_host_comm(r, g.world, g.allreduce_f32)
    L.broadcast(0)
    for k in range(int(d["steps"])):
        L.train_batch(d["x_%d_%d" % (k, r)], d["pi_%d_%d" % (k, r)], d["z_%d_%d" % (k, r)])
    np.savez({out!r} % r, params=L.params(), grads=L.grads())
    L.close(); e.close(); g.close()
""")


def test_learner_two_processes_host_group(spai, tmp_path):
    """two rank processes on the one GPU (launched as torch.distributed.run would:
    RANK / WORLD_SIZE / MASTER_*), reducing over bench.py's TCP host group: both
    end bit-identical to each other and to the in-process two-thread run, which the
    test above pins to the DDP restatement"""
    blocks, sizes, steps = 1, (48, 80), 2
    p0 = spai.init_params(blocks, 64, seed=41)
    p_other = spai.init_params(blocks, 64, seed=42)
    batches = _batches(spai, sizes, steps, seed=7)
    data = {"blocks": blocks, "steps": steps, "p0": p0, "p_other": p_other}
    for k, step in enumerate(batches):
        for r in range(2):
            data["x_%d_%d" % (k, r)], data["pi_%d_%d" % (k, r)], data["z_%d_%d" % (k, r)] = step[r]
    np.savez(tmp_path / "data.npz", **data)
    out = str(tmp_path / "rank%d.npz")
    script = tmp_path / "rank.py"
    script.write_text(RANK_WORKER.format(repo=REPO, data=str(tmp_path / "data.npz"), out=out))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPAI_GROUP_PORT=str(port),
               WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    try:
        outs = [p.communicate(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), outs
    res = [np.load(out % r) for r in range(2)]
    np.testing.assert_array_equal(res[0]["params"], res[1]["params"])
    np.testing.assert_array_equal(res[0]["grads"], res[1]["grads"])
    engines, Ls, grp, rec = _run_two_ranks(spai, blocks, (p0, p_other), batches)
    np.testing.assert_array_equal(res[0]["params"], Ls[0].params())
    np.testing.assert_array_equal(res[0]["grads"], Ls[0].grads())
    for L in Ls:
        L.close()
    for e in engines:
        e.close()


def test_learner_last_batch_after_train(spai):
    """the activations of the last train step are readable after Model::train too
    (the batch size comes from the C side: n % batch for a short last batch)"""
    z = np.load(os.path.join(GOLDEN, "learner_c4_1x64.npz"))
    blocks, hidden, seed, B, K = [int(v) for v in z["meta"]]
    s = np.concatenate(list(z["states"]))[:70]
    p = np.concatenate(list(z["policies"]))[:70]
    v = np.concatenate(list(z["values"]))[:70]
    e = spai.Engine(num_searches=1, max_trees=1)
    L = spai.Learner(e, blocks, spai.init_params(blocks, hidden, seed=seed), hidden=hidden)
    assert L.last_batch == 0
    L.train(s, p, v, epochs=1, batch=32, seed=3)
    assert L.last_batch == 70 % 32
    a = L.activation(0)
    assert a.shape == (70 % 32, 64, 6, 7) and (a >= 0).all() and (a > 0).any()
    L.close()
    e.close()


def test_host_comm_world_one_is_dropped(spai):
    """spai.h: a host collective with world 1 (or a NULL fn) is dropped, so the
    step stays launch-only: the function is never called and the step equals a
    plain learner's bit for bit"""
    blocks = 1
    p0 = spai.init_params(blocks, 64, seed=5)
    (step,) = _batches(spai, [32], 1, seed=11)
    calls = []

    def fn(buf):
        calls.append(len(buf))

    eng = [spai.Engine(num_searches=1, max_trees=1) for _ in range(2)]
    La, Lb = spai.Learner(eng[0], blocks, p0), spai.Learner(eng[1], blocks, p0)
    try:
        La.set_host_comm(0, 1, fn)
        la, lb = La.train_batch(*step[0]), Lb.train_batch(*step[0])
        La.broadcast(0)
        assert calls == []
        assert np.array_equal(np.asarray(la), np.asarray(lb))
        assert np.array_equal(La.params(), Lb.params())
    finally:
        La.close()
        Lb.close()
        for e in eng:
            e.close()

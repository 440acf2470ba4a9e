"""Data-parallel device learner: one process per GPU, each
trains the C4 net on its own batches; rank 0's RCCL unique id goes to every
rank over the host group, gradients are all-reduced with RCCL inside
spai_learner_train_batch.  Prints one JSON line (rank 0): training samples/s
over all ranks, ms per step, and whether the replicas ended bit-identical.

  python scripts/learner_dp.py [--steps K] [--batch B] [--blocks 6]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
      --master-addr 127.0.0.1 --master-port P scripts/learner_dp.py
"""
import argparse
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "self-play-ai_amd"))
import numpy as np  # noqa: E402

import spai  # noqa: E402
from hostgroup import HostGroup  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X vector FP32 (MI355X_MICROARCH.md)


def train_flops_per_sample(blocks, hid=64):
    """forward + backward (data and weight gradients: 2x forward)"""
    cells = 42
    conv = lambda ci, co: 2 * cells * co * ci * 9
    fwd = conv(3, hid) + 2 * blocks * conv(hid, hid) + conv(hid, 32) + conv(hid, 3) + 2 * 1344 * 7 + 2 * 126
    return 3 * fwd


def synthetic_batches(eng, n_batches, B, seed):
    """encoded reachable positions, random normalised policies, values in {-1, 0, 1}"""
    rng = np.random.default_rng(seed)
    n = n_batches * B
    eng.games_resize(n)   # empty boards
    plies = rng.integers(0, 30, n)
    for k in range(30):
        lm = eng.legal_mask(n)
        r = rng.random((n, 7)) * ((lm[:, None] >> np.arange(7)) & 1) * (plies[:, None] > k)
        act = np.where(r.max(1) > 0, np.argmax(r, 1), -1).astype(np.int32)
        if (act < 0).all():
            break
        eng.apply(act, check=False)   # -1 (illegal) leaves a slot unchanged
    x = eng.encode(n).reshape(n_batches, B, 126)
    pi = rng.random((n_batches, B, 7)).astype(np.float32) ** 2
    pi /= pi.sum(2, keepdims=True)
    z = rng.choice(np.array([-1, 0, 1], np.float32), (n_batches, B))
    return x, pi.astype(np.float32), z


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=128)   # TrainingArgs::default (learner_concurrent.rs:61-69)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--group", type=int, default=1,
                    help="steps handed over per call (spai_learner_train_batches; 1: train_batch per step)")
    args = ap.parse_args()
    g = HostGroup()
    local = int(os.environ.get("SPAI_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    eng = spai.Engine(num_searches=1, max_trees=1, device=local)
    L = spai.Learner(eng, args.blocks, spai.init_params(args.blocks, 64, seed=args.seed))   # same init everywhere
    uid = g.broadcast_bytes(spai.comm_unique_id() if g.rank == 0 else None) if g.world > 1 else None
    if uid is not None:
        L.set_comm(g.rank, g.world, uid)
    nb = 8
    x, pi, z = synthetic_batches(eng, nb, args.batch, args.seed * 1000 + g.rank)   # each rank its own data
    for i in range(args.warmup):
        L.train_batch(x[i % nb], pi[i % nb], z[i % nb])
    g.barrier()
    t0 = time.perf_counter()
    loss = None
    if args.group <= 1:
        for i in range(args.steps):
            loss = L.train_batch(x[i % nb], pi[i % nb], z[i % nb])   # returns after the step (loss is read back)
    else:   # the same steps, `group` per call (one host sync per call); the batches are prepared outside the clock
        calls = []
        for c0 in range(0, args.steps, args.group):
            idx = [i % nb for i in range(c0, min(args.steps, c0 + args.group))]
            calls.append((np.concatenate([x[i] for i in idx]), np.concatenate([pi[i] for i in idx]),
                          np.concatenate([z[i] for i in idx]), len(idx)))
        t0 = time.perf_counter()
        for cx, cp, cz, k in calls:
            loss = L.train_batches(cx, cp, cz, k)[-1]
    dt = time.perf_counter() - t0
    g.barrier()
    (dt_max,) = g.allreduce([dt], "max")
    digests = g.allgather(hashlib.sha256(L.params().tobytes()).hexdigest())
    fps = train_flops_per_sample(args.blocks)
    samples = args.steps * args.batch * g.world
    if g.rank == 0:
        ach = fps * samples / g.world / dt_max / 1e12   # per GPU
        print(json.dumps({
            "metric": "learner training samples/s (C4 train_batch: forward+backward+Adam)",
            "value": samples / dt_max, "unit": "samples/s", "n_gpus": g.world, "batch_per_gpu": args.batch,
            "steps": args.steps, "ms_per_step": dt_max * 1e3 / args.steps, "blocks": args.blocks,
            "steps_per_call": max(1, args.group),
            "last_loss": [float(v) for v in loss], "replicas_identical": len(set(digests)) == 1,
            "collective": "RCCL all-reduce of %d fp32 gradients per step" % L.n if g.world > 1 else None,
            "roofline": {"bound": "fp32 vector", "achieved": ach, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": ach / FP32_PEAK_TFLOPS, "flop_per_sample": fps}}), flush=True)
    L.close()
    eng.close()
    g.close()


if __name__ == "__main__":
    main()

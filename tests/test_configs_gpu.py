"""BASELINE configs 3 and 5 at their per-GPU shape on one MI355X, checked by
properties (the oracle cannot replay 4096 x 800 searches; the bit-exact checks
of search, self-play and the train step are in test_gpu_parity.py /
test_gpu_fp32.py at smaller sizes).

* C3 slice (BASELINE config 3, one rank's share): 4096 games x 800 sims with
  the 6x64 bf16 net, the (positions as f32 * 0.3) as usize subsample into the
  replay ring, 20 learner steps of 128 through a 1-rank RCCL communicator, the
  RCCL broadcast refresh, and a second round on the refreshed net
  (self-play-ai_amd/selfplay_dp.py, learner_concurrent.rs:72-85,158-159,169-290).
  The 1-rank DP learner must stay bit-identical to a plain learner fed the same
  batches, and the refreshed self-play net must equal a net built from the
  learner's parameters.
* C5 at SURVEY §8d's per-GPU shape (train_concurrent, main.rs:137-235):
  4096-game self-play workers at 800 sims, 6x64, batch 128, 20 x 10 train
  iterations, ring 12,800; every ring event replayed through the HeapRb model
  (tests/pipeline_model.py).
* C5 with several self-play workers on one device (main.rs:169-186 runs 6):
  three workers' pushes interleave in the ring, checked the same way.
"""
import os

import numpy as np
import pytest

from pipeline_model import check_events, subsample_size

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spai():
    import spai as s
    s.lib()
    return s


def test_c3_slice_full_size(spai, oracle):
    from selfplay_dp import Config3Rank
    G, sims, B, K = 4096, 800, 128, 20
    R = Config3Rank(0, 1, spai.comm_unique_id(), games=G, sims=sims, blocks=6, batch=B, train_steps=K, seed=0)
    plain = spai.Learner(R.eng, 6, spai.init_params(6, 64, seed=0))   # no communicator
    ring_twin = spai.Replay(B * 100)
    for rnd in range(2):
        games, st, loss, k = R.run_round(collect_games=True)
        assert st["games"] == G and len(games) == G
        positions = sum(len(g["moves"]) for g in games)
        assert st["positions"] == positions and st["sims"] == sims * positions
        assert k == subsample_size(positions, 0.3)
        assert np.all(np.isfinite(loss)) and loss[0] > 0
        # outcomes replay legally in the oracle (every 64th game; all of them in test_fullsize_gpu)
        for g in games[::64]:
            s = oracle.C4()
            for a in g["moves"]:
                assert a in s.valid_actions()
                s = s.next_state(int(a))
            assert s.status != 0
        # the plain learner, fed the same FIFO batches, stays bit-identical to the
        # 1-rank RCCL learner (all-reduce weight B/sum(B) = 1, broadcast a no-op)
        enc = np.concatenate([g["enc"] for g in games])
        pol = np.concatenate([g["policy"] for g in games])
        val = np.concatenate([g["value"] for g in games])
        keep = spai.choose_multiple(len(val), k, seed=0, stream=rnd).astype(np.int64)
        ring_twin.push(enc[keep], pol[keep], val[keep])
        for _ in range(K):
            plain.train_batch(*ring_twin.pop(B))
        np.testing.assert_array_equal(plain.params(), R.params)
        # the refreshed self-play net is the learner's weights
        x = enc[:64].reshape(-1, 3, 6, 7)
        fresh = spai.Net(R.eng, 6, R.learner.params())
        lg_a, v_a = R.net.forward(x)
        lg_b, v_b = fresh.forward(x)
        fresh.close()
        np.testing.assert_array_equal(lg_a, lg_b)
        np.testing.assert_array_equal(v_a, v_b)
    assert R.totals["samples_trained"] == 2 * K * B
    assert not np.array_equal(R.params, spai.init_params(6, 64, seed=0))
    ring_twin.close()
    plain.close()
    R.close()


def test_c5_pipeline_full_shape(spai):
    """one 4096-game worker (4096 games per self-play GPU), 800 sims,
    6x64, batch 128, 20 batches x 10 iterations, ring 12,800"""
    p0 = spai.init_params(6, 64, seed=3)
    events = []
    st = spai.pipeline_run(p0, selfplay_devices=(0,), learner_device=0, games_per_batch=4096, num_searches=800,
                           batch_size=128, batches_per_iter=20, train_iters=10, replay_capacity=12800, blocks=6,
                           seed=4, events=events)
    r = check_events(events, st, capacity=12800, batch_size=128, fraction=0.3, batches_expected=200, workers=1)
    assert st["weight_version_published"] == 10
    assert r["overwritten"] > 0            # a 4096-game batch pushes ~30k samples into 12.8k slots
    assert st["games"] == 4096 * r["pushes"]
    assert all(np.isfinite(st["last_loss"])) and st["last_loss"][0] > 0


def test_c5_pipeline_several_workers_one_device(spai, tmp_path):
    """three self-play workers (engines on their own host threads) sharing device 0
    with the learner; their pushes interleave in the one ring"""
    p0 = spai.init_params(2, 64, seed=5)
    events = []
    st = spai.pipeline_run(p0, selfplay_devices=(0, 0, 0), learner_device=0, checkpoint_dir=str(tmp_path),
                           games_per_batch=64, num_searches=32, batch_size=64, batches_per_iter=4, train_iters=4,
                           replay_capacity=640, blocks=2, seed=6, events=events)
    r = check_events(events, st, capacity=640, batch_size=64, fraction=0.3, batches_expected=16, workers=3)
    assert st["weight_version_published"] == 4
    assert r["workers_seen"] == 3
    assert st["games"] == 64 * r["pushes"]
    for it in range(4):
        p = spai.load_params(str(tmp_path / ("%d.safetensors" % it)), 2)
        assert np.isfinite(p).all()


def test_bench_two_ranks_one_gpu(tmp_path):
    """bench.py's N > 1 path with libspai in both ranks: two rank processes on the
    one GPU (RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them,
    SPAI_BENCH_DEVICE=0), each playing its shard of game ids, the host group's
    barrier and max/sum reductions.  Games are independent and a position's
    evaluation does not depend on its batch, so the summed work of 2 ranks x G
    games equals one rank's 2G games exactly: simulations, evaluations,
    finished games and positions"""
    import json
    import socket
    import subprocess
    import sys
    from conftest import REPO
    G = 96
    args = ["--sims", "32", "--steps", "2", "--warmup", "0", "--no-cpu-baseline", "--no-isolated",
            "--no-rules-bench", "--no-chess", "--no-timing", "--no-lockstep-ref"]
    base = dict(os.environ, SPAI_BENCH_DEVICE="0")

    def run(world, games, extra=()):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        env = dict(base, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPAI_GROUP_PORT=str(port),
                   WORLD_SIZE=str(world))
        procs = [subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world),
                                   "--games", str(games)] + args + list(extra),
                                  env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for r in range(world)]
        try:
            outs = [p.communicate(timeout=240) for p in procs]
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
        return json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][-1])

    # the default (streamed) schedule: 2 steps' games through the tree slots; the two
    # ranks' id ranges [r k G, (r + 1) k G) cover the 1-rank run's [0, 2 k G); the
    # lockstep schedule plays the same ids in batches of 2G, so its work is equal too
    one, two = run(1, 2 * G), run(2, G)
    lock = run(1, 2 * G, ["--lockstep"])
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 2 * G
    for k in ("sims", "evals", "games", "positions"):
        assert two["work"][k] == one["work"][k] == lock["work"][k], (k, one["work"], two["work"], lock["work"])
    assert two["work"]["games"] == 2 * 2 * G
    assert "streamed" in one["config"]["workload"] and "lockstep" in lock["config"]["workload"]


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` exactly as the driver invokes the 1-GPU bench (no
    launcher, no RANK / WORLD_SIZE in the environment): bench.py starts the two
    rank processes itself.  Both share device 0 here (SPAI_BENCH_DEVICE=0), so
    RCCL (one rank per GPU) is skipped with a reason and the host group carries
    the reductions; the line says n_gpus 2 and its work equals one rank's 2G
    games.  The 1-rank run forms a 1-rank RCCL communicator whose sums must equal
    the host group's (main.rs:169-186,220-234)"""
    import json
    import subprocess
    import sys
    from conftest import REPO
    G = 96
    args = ["--sims", "32", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-isolated",
            "--no-rules-bench", "--no-chess", "--no-timing", "--no-lockstep-ref"]
    env = dict(os.environ, SPAI_BENCH_DEVICE="0")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)

    def run(gpus, games):
        p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus),
                            "--games", str(games)] + args, env=env, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = p.stdout.splitlines()
        assert len(lines) == 1 and lines[0].startswith("{"), p.stdout[-2000:]   # rank 0's one JSON line, nothing else
        return json.loads(lines[0])

    one, two = run(1, 2 * G), run(2, G)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["config"]["global_batch"] == 2 * G
    for k in ("sims", "evals", "games", "positions"):
        assert two["work"][k] == one["work"][k], (k, one["work"], two["work"])
    assert one["rccl_ranks"] == 1 and one["rccl"]["counters_agree"] is True, one["rccl"]
    assert two["rccl_ranks"] == 0 and "share" in two["rccl"]["note"], two["rccl"]
    # per-rank balance and the host-core budget: every rank reports its
    # own simulations, wall time and host CPU seconds; the ranks' work sums to the line's
    for line, world in ((one, 1), (two, 2)):
        pr = line["per_rank"]
        assert sorted(r["rank"] for r in pr) == list(range(world))
        assert sum(r["sims"] for r in pr) == line["work"]["sims"]
        assert sum(r["games"] for r in pr) == line["work"]["games"]
        for r in pr:
            assert r["wall_s"] > 0 and r["host_cpu_s"] > 0 and r["sims_per_sec"] > 0
            assert abs(r["host_cpu_share"] - r["host_cpu_s"] / r["wall_s"]) < 1e-9
        assert line["host"]["cpu_share_per_rank_max"] == max(r["host_cpu_share"] for r in pr)
        assert line["schedule"] == "streamed"

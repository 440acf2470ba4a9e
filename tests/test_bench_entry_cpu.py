"""bench.py's entry point on the CPU (no GPU, no library calls): how `--gpus N`
becomes N rank processes (the worker fan-out of main.rs:169-186,220-234 as one
process per GPU).

* `--gpus 1` without a launcher runs in-process (no spawn);
* `--gpus N` without a launcher spawns N ranks with RANK = LOCAL_RANK = r,
  WORLD_SIZE = N and MASTER_* on 127.0.0.1, the parent never importing spai;
* under a launcher WORLD_SIZE must equal --gpus;
* a rank that fails stops the others (a rank blocked in the host group's
  barrier would otherwise wait forever) and the parent exits non-zero.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO


class _Reached(Exception):
    pass


def _bench(monkeypatch, argv, env):
    sys.path.insert(0, REPO)
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    calls = []

    def fake_spawn(n):
        calls.append(n)
        return 0

    def fake_dist():
        raise _Reached()

    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.setattr(bench, "Dist", fake_dist)
    return bench, calls


def test_gpus_one_runs_in_process(monkeypatch):
    bench, calls = _bench(monkeypatch, ["--gpus", "1"], {})
    with pytest.raises(_Reached):
        bench.main()
    assert calls == []


def test_gpus_n_spawns_ranks(monkeypatch):
    bench, calls = _bench(monkeypatch, ["--gpus", "4", "--steps", "1"], {})
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert calls == [4] and ex.value.code == 0


def test_launcher_world_must_match(monkeypatch):
    bench, calls = _bench(monkeypatch, ["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0"})
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert calls == [] and "WORLD_SIZE=3" in str(ex.value.code)
    bench, calls = _bench(monkeypatch, ["--gpus", "2"], {"WORLD_SIZE": "2", "RANK": "0"})
    with pytest.raises(_Reached):   # a matching launcher world runs the rank in-process
        bench.main()
    assert calls == []


def test_spawned_ranks_env_and_failure(tmp_path):
    """the real spawn with a stand-in rank program: every rank sees its env; one
    rank failing stops a rank that would block forever, and the parent reports it"""
    sys.path.insert(0, REPO)
    import bench
    prog = tmp_path / "rank.py"
    prog.write_text(
        "import json, os, sys, time\n"
        "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', 'SPAI_GROUP_PORT')\n"
        "open(os.path.join(%r, 'r%%s.json' %% os.environ['RANK']), 'w').write(json.dumps({k: os.environ[k] for k in keys}))\n"
        "if os.environ['RANK'] == '1' and 'FAIL' in sys.argv: sys.exit(3)\n"
        "if os.environ['RANK'] == '0' and 'FAIL' in sys.argv: time.sleep(600)\n" % str(tmp_path))
    old_file, old_argv = bench.__file__, sys.argv
    try:
        bench.__file__ = str(prog)
        sys.argv = ["bench.py", "--gpus", "3"]
        assert bench.spawn_ranks(3) == 0
        envs = [json.loads((tmp_path / ("r%d.json" % r)).read_text()) for r in range(3)]
        for r, e in enumerate(envs):
            assert e["RANK"] == e["LOCAL_RANK"] == str(r) and e["WORLD_SIZE"] == "3"
            assert e["MASTER_ADDR"] == "127.0.0.1"
        assert len({e["MASTER_PORT"] for e in envs}) == 1 and len({e["SPAI_GROUP_PORT"] for e in envs}) == 1
        sys.argv = ["bench.py", "--gpus", "2", "FAIL"]
        t0 = time.time()
        assert bench.spawn_ranks(2) == 3
        assert time.time() - t0 < 60
    finally:
        bench.__file__, sys.argv = old_file, old_argv


def test_parent_does_not_load_the_library(tmp_path):
    """`python bench.py --gpus 2` as a process: its ranks fail here (no GPU), the
    parent exits non-zero without having imported spai (checked by a stand-in
    SPAI_LIB that does not exist: only a rank would try to load it)"""
    env = dict(os.environ, SPAI_LIB=str(tmp_path / "absent.so"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "rank exit status" in p.stderr
    assert "not built" in p.stderr   # the ranks, not the parent, reached the library


def test_schedule_flags_parse(monkeypatch):
    """the streamed schedule is the default; --lockstep selects one lockstep batch
    per step; --stream (the round-5 A/B flag) still parses"""
    sys.path.insert(0, REPO)
    import bench
    for argv, lock in (([], False), (["--lockstep"], True), (["--stream"], False)):
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        a = bench.parse()
        assert a.lockstep is lock and not a.no_lockstep_ref


@pytest.mark.parametrize("world", [1, 2, 8])
def test_stream_game_ids_partition(world):
    """the streamed bench's game ids: the ranks' ranges tile the job's range with no
    overlap, the warm-up stream's ids are disjoint from the timed region's, and at
    world 1 the stream plays the lockstep steps' ids (step i: [i G, (i + 1) G))"""
    sys.path.insert(0, REPO)
    import bench
    G, k, w = 96, 3, 2

    def ids(first, steps):
        out = []
        for r in range(world):
            b = bench.stream_base(first, steps, world, r, G)
            out.extend(range(b, b + steps * G))
        return out

    timed, warm = ids(0, k), ids(-w, w)
    assert sorted(timed) == list(range(0, k * world * G))
    assert sorted(warm) == list(range(-w * world * G, 0))
    if world == 1:
        assert timed == [g for i in range(k) for g in range(i * G, (i + 1) * G)]


_RCCL_FAIL = r"""
import sys
sys.path.insert(0, {repo!r})
import bench

class G:
    def allgather(self, x):
        return [0, 1] if isinstance(x, int) else [x, x]
    def broadcast_bytes(self, b):
        return b or bytes(128)

class D:
    world, rank, local = {world}, 0, 0
    g = G()

class S:
    @staticmethod
    def comm_unique_id():
        return bytes(128)
    class Comm:
        def __init__(self, *a):
            raise RuntimeError("ncclCommInitRank failed (simulated)")

comm, note = bench.rccl_comm(D(), S)
print("returned", comm, note)
"""


@pytest.mark.parametrize("world", [1, 2])
def test_rccl_failure_is_agreed_and_reported(tmp_path, world):
    """an RCCL communicator failure on a rank must not leave its peers
    blocked in a collective.  spai_comm_create waits with a bound (a failed or absent
    peer returns an error), the ranks then agree over the host group, and without a
    communicator on every rank none uses one: the line reports it and the run goes on
    (the host group carries the reductions)"""
    p = subprocess.run([sys.executable, "-c", _RCCL_FAIL.format(repo=REPO, world=world)], capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0, (p.stdout, p.stderr)
    assert "returned None RCCL communicator failed (rank 0: RuntimeError('ncclCommInitRank failed (simulated)')" \
        in p.stdout and "host group only" in p.stdout, p.stdout

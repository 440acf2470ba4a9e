"""Multi-GPU path on the CPU: games shard by id with no data-path collective.

Per-game trajectories depend only on (seed, game id) and the position-wise
evaluator, so a 2-rank run (gloo, world_size 2, each rank playing its shard of
game ids as bench.py assigns them) must reproduce the single-process run
exactly.  The oracle stands in for each rank's engine here (no GPU)."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np

from conftest import REPO


def _by_game(r):
    out = {}
    for i, g in enumerate(r["game"]):
        out.setdefault(int(g), []).append((float(r["value"][i]), r["policy"][i].tobytes()))
    return out


def test_shard_invariance_oracle(oracle):
    full = oracle.self_play(oracle.GAME_CONNECT4, 8, 12, 3, eval_kind=oracle.EVAL_HASH, max_plies=42)
    a = oracle.self_play(oracle.GAME_CONNECT4, 4, 12, 3, eval_kind=oracle.EVAL_HASH, game_id_base=0, max_plies=42)
    b = oracle.self_play(oracle.GAME_CONNECT4, 4, 12, 3, eval_kind=oracle.EVAL_HASH, game_id_base=4, max_plies=42)
    fg = _by_game(full)
    sa, sb = _by_game(a), _by_game(b)
    merged = dict(sa)
    merged.update({k + 4: v for k, v in sb.items()})
    assert merged == fg


WORKER = textwrap.dedent("""
    import os, sys, json
    sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "oracle"))
    import numpy as np, torch, torch.distributed as dist
    import oracle
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    G = 4
    res = oracle.self_play(oracle.GAME_CONNECT4, G, 12, 3, eval_kind=oracle.EVAL_HASH,
                           game_id_base=r * G, max_plies=42)   # bench.py: base = (step*world + rank) * G
    sims = torch.tensor([res["sims"]], dtype=torch.float64)
    dist.all_reduce(sims)                                      # bench.py sums work over ranks
    t = torch.tensor([float(r + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)                   # and takes the max time
    vals = [None] * w
    dist.all_gather_object(vals, (res["game"].tolist(), res["value"].tolist()))
    if r == 0:
        print(json.dumps({{"sims": sims.item(), "tmax": t.item(), "parts": vals}}))
    dist.destroy_process_group()
""")


def test_two_rank_gloo(oracle, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(repo=REPO))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    import json
    res = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][-1])
    full = oracle.self_play(oracle.GAME_CONNECT4, 8, 12, 3, eval_kind=oracle.EVAL_HASH, max_plies=42)
    assert res["sims"] == full["sims"]
    assert res["tmax"] == 2.0
    got = {}
    for r, (games, vals) in enumerate(res["parts"]):
        for g, v in zip(games, vals):
            got.setdefault(g + 4 * r, []).append(v)
    exp = {}
    for g, v in zip(full["game"].tolist(), full["value"].tolist()):
        exp.setdefault(g, []).append(v)
    assert got == exp

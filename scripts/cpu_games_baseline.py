"""CPU baseline records for bench.py (run on the GPU box's host cores).

  sweep:  sims/s of the CPU reference path (oracle/refcpu.py: oracle tree loop
          + libtorch CPU fp32 forward) at several intra-op thread counts, each a
          bounded window over 256 C4 games x 800 sims/move;
  games:  games/s of N games from the empty board played TO COMPLETION at 800
          sims/move with the best thread count.

Each measurement runs in its own subprocess.  Writes one JSON record, e.g.
    python scripts/cpu_games_baseline.py --out gpurun_out/cpu_baseline_r02.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def run(args, timeout):
    cmd = [sys.executable, os.path.join(REPO, "oracle", "refcpu.py"), json.dumps(args)]
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    if out.returncode != 0:
        raise RuntimeError(out.stderr[-2000:])
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    r["wall"] = time.time() - t0
    print(json.dumps({**args, **r}), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--threads", default="", help="comma list for the sweep (default: 8,16,32,quota; r02a measured 64 threads at 0.23x of 16 under a 16-CPU quota)")
    ap.add_argument("--sweep-seconds", type=float, default=12.0)
    ap.add_argument("--sweep-games", type=int, default=256)
    ap.add_argument("--games", type=int, default=256)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--no-games", action="store_true")
    a = ap.parse_args()
    import refcpu
    quota, ncpu = refcpu.cpu_quota(), os.cpu_count()
    ts = [int(t) for t in a.threads.split(",")] if a.threads else sorted({8, 16, 32, quota})
    rec = dict(cpu_model=refcpu.cpu_model(), os_cpu_count=ncpu, cpu_quota=quota, sweep=[])
    for t in ts:
        r = run(dict(mode="sims", games=a.sweep_games, sims=a.sims, seconds=a.sweep_seconds, blocks=a.blocks,
                     threads=t), timeout=a.sweep_seconds * 6 + 120)
        rec["sweep"].append(dict(threads=t, **r))
    best = max(rec["sweep"], key=lambda r: r["sims_per_sec"])
    rec["best_threads"] = best["threads"]
    if not a.no_games:
        rec["games_run"] = dict(threads=best["threads"], **run(
            dict(mode="games", games=a.games, sims=a.sims, blocks=a.blocks, threads=best["threads"]), timeout=3000))
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()

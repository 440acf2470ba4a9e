# Round 6 session i: bench.py --gpus 4 and --gpus 8 rehearsed on the one GPU (every rank
# on device 0: the spawn, the host group's barrier and reductions, per-rank fields,
# the lockstep figure on every rank; RCCL is skipped for ranks sharing a device)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06i} && mkdir -p $O
for n in 4 8; do
  SPAI_BENCH_DEVICE=0 timeout -k 10 300 python3 bench.py --gpus $n --games 64 --sims 32 --steps 2 --warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_n$n.json 2> $O/bench_n$n.err || { tail -5 $O/bench_n$n.err; exit 1; }
  python3 - $O/bench_n$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1]); n = int(sys.argv[2])
pr = d["per_rank"]
assert d["n_gpus"] == n and len(pr) == n and sorted(r["rank"] for r in pr) == list(range(n))
assert sum(r["sims"] for r in pr) == d["work"]["sims"] and d["work"]["games"] == n * 2 * 64
assert d["lockstep"]["n_gpus"] == n and d["rccl_ranks"] == 0 and "share" in d["rccl"]["note"]
print("n", n, "ok:", round(d["value"] / 1e6, 3), "M sims/s;", "host", {k: d["host"][k] for k in ("sync", "cpus_available", "ranks_on_node", "cpu_share_per_rank_max")}, "spread", round(d["host"]["sims_per_sec_rank_spread"], 3))
PY
done

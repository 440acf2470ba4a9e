# Round 6 session f: host waits spinning vs sleeping (SPAI_BLOCKING_SYNC), interleaved,
# 4-step streamed benches: sims/s and host CPU seconds per rank; then one default
# bench line (all legs: isolated, rules, chess window + chess CPU leg, C4 CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06f} && mkdir -p $O
timeout -k 10 120 ./scripts/ubench/grid_barrier > $O/grid_barrier.txt 2>&1 || { cat $O/grid_barrier.txt; exit 1; }
cat $O/grid_barrier.txt
for r in 1 2; do
  for b in 0 1; do
    n=sync${b}_$r
    SPAI_BLOCKING_SYNC=$b timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s, host cores per rank', round(d['host']['cpu_share_per_rank_max'],3))"
  done
done
[ -n "${SKIP_FULL:-}" ] && exit 0
timeout -k 10 900 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().splitlines()[-1]); print('default', round(d['value']/1e6,3), 'M sims/s', d['roofline']['frac'], d.get('chess',{}).get('cpu_baseline'), d.get('cpu_baseline',{}).get('value'))"

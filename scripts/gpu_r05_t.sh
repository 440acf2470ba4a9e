# Round 5 session t: the streamed line against K (2, 10, 40 steps) and the lockstep line at K = 10, one box
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05t} && mkdir -p $O
for v in "2 " "10 " "40 " "10 --lockstep"; do
  set -- $v; k=$1; n=stream_k$k; [ -n "$2" ] && n=lock_k$k
  timeout -k 10 400 python3 bench.py --steps $k --warmup 2 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref $2 > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', round(d['roofline']['frac'],4))"
done

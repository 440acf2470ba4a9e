# the whole -m gpu suite (streaming parity included), then an interleaved
# lockstep vs streaming bench A/B (timed region only) and one default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
for r in 1 2; do
  for v in "" "--stream"; do
    n=lock; [ -n "$v" ] && n=stream
    timeout -k 10 300 python3 bench.py --steps ${SSTEPS:-4} --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess $v > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { tail -5 $O/bench_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/bench_${n}_$r.json') if l.startswith('{')][-1]); print('$n $r', round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', round(d['roofline']['frac'],4), d['ms_per_step'])"
  done
done

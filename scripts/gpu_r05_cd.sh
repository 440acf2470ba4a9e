# the whole -m gpu suite, then sessions c (chess forward A/B, PMC traffic) and d
# (learner BN fusion A/B, rocprof) without their own parity tests, then a check that
# the bench prints exactly one line on stdout
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05cd && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
SKIP_TESTS=1 bash scripts/gpu_r05_c.sh && SKIP_TESTS=1 bash scripts/gpu_r05_d.sh
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_stdout.txt 2> $O/bench_stderr.txt; rc=$?
echo "bench rc=$rc stdout lines: $(wc -l < $O/bench_stdout.txt)"; head -c 300 $O/bench_stdout.txt; echo
for r in 1 2; do
  for v in "" "--stream"; do
    n=lock; [ -n "$v" ] && n=stream
    timeout -k 10 300 python3 bench.py --steps ${SSTEPS:-4} --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess $v > $O/bench_${n}_$r.json 2> $O/bench_${n}_$r.err || { tail -5 $O/bench_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/bench_${n}_$r.json') if l.startswith('{')][-1]); print('$n $r', round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', round(d['roofline']['frac'],4))"
  done
done

# Round 6 final, part a (at the committed head): the -m gpu suite, smoke(), a
# rocprofv3 kernel-trace of the bench command (2 streamed steps), and the default
# bench line
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06final} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; cat $O/smoke.log; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/ktrace
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktrace -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_ktrace.json 2> $O/bench_ktrace.err; rc=$?
[ $rc -eq 0 ] || { tail -5 $O/bench_ktrace.err; exit $rc; }
cp $(find /tmp/ktrace -name '*kernel_stats*.csv' | head -1) $O/trace_kernel_stats.csv
head -8 $O/trace_kernel_stats.csv
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print('default', round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', round(d['roofline']['frac'],4), d['roofline']['per_launch']['avg_launch_ms'])"

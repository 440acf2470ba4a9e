# Round 5 session c: chess forward without scratch spills (thread id laundered per
# pass): chess parity tests, then an interleaved A/B of the chess window against
# the previous forward (build_exp/libspai_chessold.so), then the PMC traffic of
# the new forward (FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_summary.py).
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05c} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_chess_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_chess.log 2>&1
  rc=$?; tail -3 $O/pytest_chess.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for L in build_exp/libspai_chessold.so self-play-ai_amd/libspai.so ${CHESS_EXTRA:-build_exp/libspai_chesspf.so}; do
    n=$(basename $L .so)_$r
    SPAI_LIB=$L timeout -k 10 300 python3 scripts/chess_bench.py --moves 2 --no-cpu-baseline > $O/chess_$n.json 2> $O/chess_$n.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/chess_$n.err; exit $rc; }
    python3 -c "import json; d=json.loads([l for l in open('$O/chess_$n.json') if l.startswith('{')][-1]); print('$n', round(d['value']), d['roofline']['avg_launch_ms'] if 'avg_launch_ms' in d['roofline'] else '', round(d['roofline']['frac'],4))"
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/cpmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d /tmp/cpmc_$c -o p -- \
    python3 scripts/chess_bench.py --moves 1 --no-cpu-baseline > $O/traffic_$c.json 2> $O/traffic_$c.err
  rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/traffic_$c.err; exit $rc; }
done
python3 scripts/pmc_summary.py $O/forward_traffic.json $(find /tmp/cpmc_FETCH_SIZE /tmp/cpmc_WRITE_SIZE -name '*counter_collection*.csv') > $O/pmc.txt 2>&1; tail -20 $O/pmc.txt

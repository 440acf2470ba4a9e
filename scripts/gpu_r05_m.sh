# Round 5 session m: chess streaming -- the chess GPU tests (per-game streaming
# parity included), then full games: 2 x 1024 games at 100 sims/move (20x256 net)
# as two lockstep batches against one stream through 1024 tree slots
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05m} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_chess_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_chess.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_chess.log | tail -2; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_chess.log | head -20; exit $rc; }
for v in "" "--stream"; do
  n=lock; [ -n "$v" ] && n=stream
  timeout -k 10 400 python3 scripts/chess_bench.py --full --batches 2 --sims ${CSIMS:-100} --no-cpu-baseline $v > $O/chess_full_$n.json 2> $O/chess_full_$n.err || { tail -5 $O/chess_full_$n.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/chess_full_$n.json') if l.startswith('{')][-1]); print('$n', round(d['value']), 'sims/s', round(d['games_per_sec'],3), 'games/s', round(d['seconds'],1), 's', round(d['roofline']['frac'],4))"
done

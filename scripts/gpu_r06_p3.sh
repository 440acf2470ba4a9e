# Round 6: the chess forward's 3-position passes (SPAI_CHESS_P3) -- the chess -m gpu
# tests, then this build against the head library (build_exp/libspai_head.so) on the
# chess window at 600 / 700 / 768 / 1024 trees, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-p3} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python3 -u -m pytest tests/test_chess_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_chess.log 2>&1; rc=$?
tail -3 $O/pytest_chess.log; [ $rc -eq 0 ] || exit $rc
for g in 700 600 768 1024; do
  for i in 1 2; do
    for v in p3 head; do
      if [ $v = head ]; then L=build_exp/libspai_head.so; else L=self-play-ai_amd/libspai.so; fi
      SPAI_LIB=$L timeout -k 10 300 python3 scripts/chess_bench.py --games $g --moves 2 --no-cpu-baseline > $O/${v}_${g}_$i.json 2> $O/${v}_${g}_$i.err || { tail -5 $O/${v}_${g}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${g}_$i.json').read().splitlines()[-1]); r=d.get('roofline',{}); print('$v $g $i', round(d['value']/1e3,1), 'k sims/s', r.get('frac'), r.get('avg_launch_ms', r.get('per_launch')))"
    done
  done
done

# Round 6: the -m gpu suite with the interleave hints off by default, then the new default
# against the old (head) library and two ring-depth variants on top of it, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-sched2} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ARGS="--no-cpu-baseline --no-rules-bench --no-chess"
for i in 1 2; do
  for v in new head da6 db3; do
    if [ $v = new ]; then L=self-play-ai_amd/libspai.so; else L=ablibs/libspai_$v.so; fi
    SPAI_LIB=$L timeout -k 10 300 python3 bench.py $ARGS > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().splitlines()[-1]); r=d['roofline']; print('$v $i', round(d['value']/1e6,3), 'M sims/s lockstep', round(d['lockstep']['value']/1e6,3), 'conc2', round(r['isolated'][[k for k in r['isolated'] if 'conc2' in k][0]]['frac'],4), 'job', round(r['frac'],4))"
  done
done

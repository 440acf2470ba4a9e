# Round 6: the fused last tap's per-task hints / fence (SPAI_FINAL_HINTS / SPAI_FINAL_FENCE)
# and the S = 4 B ring (SPAI_DB4 = 3) on top of the round-6 default, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-sched3} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
ARGS="--no-cpu-baseline --no-rules-bench --no-chess"
for i in ${REPS:-1 2}; do
  for v in new fh0 fh0ff0 db4; do
    if [ $v = new ]; then L=self-play-ai_amd/libspai.so; else L=ablibs/libspai_$v.so; fi
    SPAI_LIB=$L timeout -k 10 300 python3 bench.py $ARGS > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().splitlines()[-1]); r=d['roofline']; print('$v $i', round(d['value']/1e6,3), 'M sims/s lockstep', round(d['lockstep']['value']/1e6,3), 'conc2', round(r['isolated'][[k for k in r['isolated'] if 'conc2' in k][0]]['frac'],4), 'job', round(r['frac'],4))"
  done
done

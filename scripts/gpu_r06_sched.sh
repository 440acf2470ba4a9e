# Round 6: C4 forward k-step scheduling knobs (SPAI_KSTEP_FENCE=0: no scheduling fence
# closing each ordinary k-step; SPAI_ISSUE_HINTS=0: no MFMA/VALU/LDS/VMEM interleave
# hints) against the head library, interleaved, the streamed line without CPU/chess/rules legs
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-sched} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
ARGS="--no-cpu-baseline --no-rules-bench --no-chess"
for i in 1 2; do
  for v in nofence head nohints; do
    SPAI_LIB=ablibs/libspai_$v.so timeout -k 10 300 python3 bench.py $ARGS > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().splitlines()[-1]); r=d['roofline']; print('$v $i', round(d['value']/1e6,3), 'M sims/s lockstep', round(d['lockstep']['value']/1e6,3), 'iso', r.get('isolated'))"
  done
done

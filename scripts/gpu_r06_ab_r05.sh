# Round 6: the round-5 head (0db920e, built in build_exp/r05) against this head on
# one box, interleaved, the default streamed line without the CPU / chess / rules legs
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-ab_r05} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
ARGS="--no-cpu-baseline --no-isolated --no-rules-bench --no-chess"
for i in 1 2; do
  for v in head r05; do
    if [ $v = head ]; then B=bench.py; else B=build_exp/r05/bench.py; fi
    timeout -k 10 300 python3 $B $ARGS > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$i.json').read().splitlines()[-1]); print('$v $i', round(d['value']/1e6,3), 'M sims/s', 'lockstep', round(d.get('lockstep',{}).get('value',0)/1e6,3))"
  done
done

# Round 6: the default bench line at the committed head (after bench.py's --pmc-json default moved)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-line} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; cat $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); r=d['roofline']; print('default', round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', round(r['frac'],4), r['executed']['source'][:60])"

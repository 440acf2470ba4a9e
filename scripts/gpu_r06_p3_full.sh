# Round 6: the chess forward's 3-position passes against the head library on whole
# streamed games: 1,024 games through 1,024 tree slots at 400 sims/move, 20x256
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-p3_full} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
for v in p3 head; do
  if [ $v = head ]; then L=build_exp/libspai_head.so; else L=self-play-ai_amd/libspai.so; fi
  SPAI_LIB=$L timeout -k 10 500 python3 scripts/chess_bench.py --full --stream --batches 1 --no-cpu-baseline > $O/${v}.json 2> $O/${v}.err || { tail -5 $O/${v}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${v}.json').read().splitlines()[-1]); print('$v', {k: d[k] for k in d if k in ('value','games_per_sec','seconds')}, d.get('roofline',{}).get('frac'), d.get('roofline',{}).get('avg_leaves_per_launch'))"
done

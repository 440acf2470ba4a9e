# Round 6 session c: BASELINE config 4 played to completion -- 2 x 1,024 chess games at
# 400 sims/move, 20x256 bf16, with a per-move trace; MODE=lockstep (two batches of
# 1,024 started together) or MODE=stream (2,048 games through 1,024 tree slots)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06c} && mkdir -p $O
M=${MODE:-lockstep}; X=""; [ "$M" = stream ] && X="--stream"
rm -f $O/moves_$M.csv
SPAI_TRACE_MOVES=$O/moves_$M.csv timeout -k 10 1000 python3 scripts/chess_bench.py --full --batches 2 $X --no-cpu-baseline > $O/full_$M.json 2> $O/full_$M.err || { tail -5 $O/full_$M.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/full_$M.json').read().splitlines()[-1]); print('$M', round(d['value']), 'sims/s', round(d['games_per_sec'], 3), 'games/s', round(d['seconds'], 1), 's', d['roofline']['frac'])"

# round-4 session o: the one-chain switch (SPAI_MIN_CHAIN_LEAVES: one search chain
# once the previous call averaged fewer leaves per iteration; default 64), swept
# on the committed build
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_o} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for m in 64 16 32 128 256; do
    SPAI_MIN_CHAIN_LEAVES=$m SPAI_TRACE_MOVES=$PWD/$O/moves_m${m}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_m${m}_$r.json 2> $O/bench_m${m}_$r.err || { tail -3 $O/bench_m${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_m${m}_$r.json'));print('min_chain_leaves $m run $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done

# round-4 session j: group-size policy constants A/B (build_exp variants of
# net_c4.hip: kChainCycles 20k / 31k (base) / 45k, kConcMinCount 450 / 600 (base) / 800)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_j} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
for r in 1 2; do
  for v in base cc20 cc45 mc450 mc800; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done

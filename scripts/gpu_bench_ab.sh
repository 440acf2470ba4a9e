# bench.py A/B of library builds (build_exp/libspai_<v>.so), interleaved rounds;
# optional phase stamps of the diagnostic build first.
#   VARS="base l2warm" ROUNDS=2 PHASES=1 TAG=x bash scripts/gpu_bench_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-benchab}; mkdir -p $O
if [ -n "${PHASES:-}" ]; then
  SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 180 python scripts/net_phases.py > $O/phases.txt 2>&1 || { cat $O/phases.txt; exit 1; }
  cat $O/phases.txt
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 300 python bench.py --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us', 'sel', round(d['kernel_ms']['select']*1e3,2), 'exp', round(d['kernel_ms']['expand']*1e3,2))"
  done
done 2>&1 | tee $O/bench.txt

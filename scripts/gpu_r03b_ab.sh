# forward sweep + bench A/B of build_exp variants, optional phase stamps of the diag build
#   FWD="a b" BENCHV="a b" PHASES=1 bash scripts/gpu_r03b_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r03b_ab} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
fi
if [ -n "${PHASES:-}" ]; then
  SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 300 python scripts/net_phases.py > $O/phases.txt 2>&1; rc=$?; tail -9 $O/phases.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${FWD:-}" ]; then
LIBS=$(for v in $FWD; do printf "build_exp/libspai_$v.so,"; done); LIBS=${LIBS%,}
  for r in 1 2; do
    timeout -k 10 300 python scripts/fwd_sweep.py --libs $LIBS --counts ${COUNTS:-256,512,1006,1536,2048,4096} > $O/sweep_$r.txt 2>&1 || { cat $O/sweep_$r.txt; exit 1; }
    cat $O/sweep_$r.txt
  done
fi
for r in 1 2; do
  for v in $BENCHV; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us')"
  done
done 2>&1 | tee $O/bench.txt

# forward prefetch-depth knobs at S = 4 (sweep + bench A/B) and the chess P = 2-only
# register experiment (chess_quick, 1024 trees x 48 sims)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r03b_knobs} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
FWD=${FWD:-"base db3 da3 da9"}
LIBS=$(for v in $FWD; do printf "build_exp/libspai_$v.so,"; done); LIBS=${LIBS%,}
for r in 1 2; do
  timeout -k 10 300 python scripts/fwd_sweep.py --libs $LIBS --counts ${COUNTS:-256,512,1006,1536,2048,4096} > $O/sweep_$r.txt 2>&1 || { cat $O/sweep_$r.txt; exit 1; }
  cat $O/sweep_$r.txt
done
for r in 1 2; do
  for v in ${BENCHV:-base db3 da9}; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us')"
  done
done 2>&1 | tee $O/bench.txt
for r in 1 2; do
  for v in cbase cp2; do
    echo "== $v $r"
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 200 python scripts/chess_quick.py --sims 48 || exit $?
  done
done 2>&1 | tee $O/chess.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "learner" --timeout 200 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; tail -2 $O/pytest_learner.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_learner.log | head -20; exit $rc; }
for v in lprev new lprev new; do
  if [ $v = new ]; then unset SPAI_LIB; else export SPAI_LIB=$PWD/build_exp/libspai_$v.so; fi
  timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_$v.json 2> $O/learner_$v.err || { tail -3 $O/learner_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/learner_$v.json'));print('== $v', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
done 2>&1 | tee $O/learner.txt

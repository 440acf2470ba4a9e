# A/B of library builds (build_exp/libspai_<v>.so): optional tests on the in-tree
# build, the forward-alone sweep per build, then interleaved bench rounds.
#   VARS="base pref" ROUNDS=2 TESTS="tests/test_gpu_parity.py -m gpu -k net_" TAG=x bash scripts/gpu_lib_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-libab}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  eval timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS \
      > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PHASES:-}" ]; then   # per-phase stamps of the diagnostic build (make -C self-play-ai_amd diag)
  SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 180 python scripts/net_phases.py > $O/phases.txt 2>&1 \
      || { cat $O/phases.txt; exit 1; }
  cat $O/phases.txt
fi
libs=$(for v in $VARS; do printf "build_exp/libspai_%s.so," $v; done)
for sw in $(seq 1 ${SWEEPS:-2}); do   # the variants alternate: A B A B
  timeout -k 10 300 python scripts/fwd_sweep.py --libs ${libs%,} --counts ${COUNTS:-256,512,1006,1500,2048,4096} \
      > $O/sweep_$sw.txt 2>&1 || { tail -5 $O/sweep_$sw.txt; exit 1; }
  cat $O/sweep_$sw.txt
done | tee $O/sweep.txt || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline \
        --no-isolated ${BENCH_ARGS:-} > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us', 'sel', round(d['kernel_ms']['select']*1e3,2), 'chip_frac', round(d['roofline']['chip_frac'],3))"
  done
done 2>&1 | tee $O/bench.txt

# bench.py A/B over environment settings of ONE library build, interleaved rounds,
# plus the forward-alone sweep (spai_net_bench) under each setting.
#   ENVS="SPAI_FWD_SMALL=0 SPAI_FWD_SMALL=1" ROUNDS=2 TAG=x bash scripts/gpu_env_ab.sh
# (ENVS items are single NAME=VALUE words; "base" means no extra variable)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-envab}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  eval timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS \
      > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for v in $ENVS; do
  e=$v; [ "$v" = base ] && e=SPAI_UNUSED=0
  env $e timeout -k 10 300 python scripts/fwd_sweep.py --counts ${COUNTS:-256,512,1006,1500,2048,4096} > $O/sweep_$v.txt 2>&1 \
      || { tail -5 $O/sweep_$v.txt; exit 1; }
  echo "== sweep $v"; cat $O/sweep_$v.txt
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $ENVS; do
    e=$v; [ "$v" = base ] && e=SPAI_UNUSED=0
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} \
        > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us', 'sel', round(d['kernel_ms']['select']*1e3,2), 'chip_frac', round(d['roofline']['chip_frac'],3))"
  done
done 2>&1 | tee $O/bench.txt

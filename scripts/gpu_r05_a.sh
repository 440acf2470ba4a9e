# Round 5 session a: the whole -m gpu suite (bench --gpus 2 entry point, comm,
# host-comm world 1 included), then an interleaved one-box A/B of the chain
# policy with the per-move trace: default (2 chains), SPAI_CHAINS=1, and one
# chain at or above SPAI_HI_LEAVES leaves per iteration.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05a} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; grep -E "passed|failed|FAIL|ERROR" $O/pytest_gpu.log | tail -8; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for ab in ${VARIANTS:-base SPAI_CHAINS=1 SPAI_HI_LEAVES=3000 SPAI_HI_LEAVES=2000}; do
    L=$(echo $ab | tr '=,' '__')_$rep
    env $(echo $ab | tr ',' ' ' | sed 's/^base$//') SPAI_TRACE_MOVES=$PWD/$O/moves_$L.csv timeout -k 10 300 \
      python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_$L.json 2> $O/bench_$L.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_$L.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/bench_$L.json')); print('$L', round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4), d['rccl_ranks'])"
  done
done

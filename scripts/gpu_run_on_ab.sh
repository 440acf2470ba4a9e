# A/B of the terminal run-on in select (SPAI_RUN_ON; the experiment is
# profiles/r02/search/run_on/run_on_experiment.patch, not in the product):
# the -m gpu suite, benches over run-on caps, a per-move trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run_on}
mkdir -p $O
SPAI_RUN_ON=${TEST_RUN_ON:-1} timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in ${RUNS:-1 2 4 8 1}; do
  SPAI_RUN_ON=$r timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_run_on$r.json 2> $O/bench_run_on$r.err
  rc=$?; echo "run_on=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys;d=json.load(open('$O/bench_run_on$r.json'));print('run_on=$r', round(d['value']/1e6,3),'M sims/s', round(d['games_per_sec'],1),'games/s', round(d['ms_per_step'],1),'ms')" | tee -a $O/ab.txt
done
[ -n "$TRACE" ] || exit 0
rm -f $O/moves.csv
SPAI_RUN_ON=$TRACE SPAI_TRACE_MOVES=$O/moves.csv timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err
rc=$?; echo "trace rc=$rc"; exit $rc

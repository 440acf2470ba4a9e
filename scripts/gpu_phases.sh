set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ph}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 300 python scripts/net_phases.py 2>&1 | tee gpurun_out/phases_$TAG.txt
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"; exit $rc

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== gpu tests" 
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== small bench"
timeout -k 10 600 python bench.py --steps 1 --warmup 0 --games 1024 --sims 200 --no-cpu-baseline > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err
rc=$?; cat gpurun_out/bench_small.json; tail -5 gpurun_out/bench_small.err; echo "bench rc=$rc"

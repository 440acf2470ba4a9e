# GPU tests, full-config bench and rocprofv3 kernel stats in one call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r01}
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -40 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_full.sh

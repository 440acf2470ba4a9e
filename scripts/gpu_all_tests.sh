# the whole -m gpu suite (one process) as the driver runs it at round end
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu_all.log | tail -45; echo "pytest rc=$rc"
exit $rc

# Round 6 session e: the whole -m gpu suite on the current build (new C-ABI client
# tests included), the grid-barrier microbenchmark (persistent-learner question),
# then the roofline PMC passes of the bench command (scripts/gpu_roofline_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06e} && mkdir -p $O
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/ubench/grid_barrier > $O/grid_barrier.txt 2>&1; rc=$?; cat $O/grid_barrier.txt; [ $rc -eq 0 ] || exit $rc
[ -n "${SKIP_PMC:-}" ] && exit 0
TAG=${TAG:-r06e}/pmc COMMIT=${COMMIT:-unknown} bash scripts/gpu_roofline_pmc.sh

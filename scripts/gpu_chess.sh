# chess GPU tests + a timing run of one chess search move
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_chess_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_chess.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_chess.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/chess_quick.py ${CHESS_ARGS:-} > gpurun_out/chess_quick.json 2> gpurun_out/chess_quick.err
rc=$?; cat gpurun_out/chess_quick.json; tail -5 gpurun_out/chess_quick.err; echo "quick rc=$rc"
exit $rc

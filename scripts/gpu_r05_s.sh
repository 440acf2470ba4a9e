# Round 5 session s: the streaming parity tests (C4 hash / temperatures / fp32 net, chess, TicTacToe)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05s} && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -k "stream" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $O/pytest_stream.log | tail -16; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_stream.log | head; exit $rc; }

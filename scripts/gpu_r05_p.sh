# Round 5 session p: the full-size tests (streamed vs lockstep per game at C2)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05p} && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_fullsize.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" $O/pytest_fullsize.log | tail -6; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_fullsize.log | head -20; exit $rc; }

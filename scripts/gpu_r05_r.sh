# Round 5 session r: bench entry after the stream_base refactor (bench tests + one short line)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05r} && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -k bench -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_bench.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_bench.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_bench.log | head; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc lines $(wc -l < $O/bench.json)"; head -c 300 $O/bench.json; echo

# BASELINE config 4 to completion: 1024 chess games x 400 sims/move, 20x256 net (heartbeat on stderr)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u scripts/chess_bench.py --full --no-cpu-baseline ${CHESS_ARGS:-} > gpurun_out/bench_chess_full.json 2> gpurun_out/bench_chess_full.err
rc=$?; cat gpurun_out/bench_chess_full.json; tail -3 gpurun_out/bench_chess_full.err; echo "rc=$rc"
exit $rc

# BASELINE config 4 to completion with the per-move trace (move, active games, leaves, seconds)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/chess_trace; mkdir -p $O; rm -f $O/moves.csv
SPAI_TRACE_MOVES=$O/moves.csv timeout -k 10 1100 python -u scripts/chess_bench.py --full --no-cpu-baseline ${CHESS_ARGS:-} > $O/bench_chess_full.json 2> $O/bench_chess_full.err
rc=$?; cat $O/bench_chess_full.json; tail -2 $O/bench_chess_full.err; echo "rc=$rc"
exit $rc

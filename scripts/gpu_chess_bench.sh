# chess config-4 bench (bounded moves) + rocprofv3 kernel stats of a shorter run of the same command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-chess}
timeout -k 10 600 python -u scripts/chess_bench.py ${CHESS_ARGS:---moves 4} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/cprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cprof -o trace -- \
    python3 scripts/chess_bench.py --moves 2 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/bench_prof_$TAG.err
mkdir -p gpurun_out/prof_$TAG
find /tmp/cprof -name '*stats*.csv' -exec cp {} gpurun_out/prof_$TAG/ \;
cat gpurun_out/prof_$TAG/*kernel_stats*.csv 2>/dev/null | cut -c1-250 | head -12
exit $rc

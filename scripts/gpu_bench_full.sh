# Full BASELINE config bench + rocprofv3 kernel stats of a shorter run of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err
rc=$?; cat gpurun_out/bench_full_$TAG.json; tail -5 gpurun_out/bench_full_$TAG.err; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
rm -rf /tmp/prof
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o trace -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/bench_prof_$TAG.err
mkdir -p gpurun_out/prof_$TAG
find /tmp/prof -name '*stats*.csv' -exec cp {} gpurun_out/prof_$TAG/ \;
ls -la gpurun_out/prof_$TAG
cat gpurun_out/prof_$TAG/*kernel_stats*.csv 2>/dev/null | head -20
exit $rc

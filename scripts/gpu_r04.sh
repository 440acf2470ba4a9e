# round-4 validation: -m gpu suite (with the bf16-vs-fp32 search statistics written
# out), smoke, the default bench line (rules kernels + chess window included).
# TESTS=<pytest selection> narrows the suite; NOBENCH=1 skips the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt
SPAI_STATS_OUT=$PWD/$O/bf16_search_stats.json timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -30; exit $rc; }
grep -h "search statistics" $O/pytest_gpu.log | head -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc

# round-5 validation of the in-tree build: -m gpu suite, smoke, the default bench
# line (as the driver runs it), the N = 2 entry point, rocprof kernel stats of the
# bench, FETCH/WRITE PMC passes (HBM traffic per k_forward launch).
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05_final} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 900 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json | cut -c1-600; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  rm -rf /tmp/prof_b && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_b -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated --no-lockstep-ref > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || { tail -5 $O/bench_under_rocprof.err; exit 1; }
  find /tmp/prof_b -name '*kernel_stats.csv' -exec cp {} $O/trace_kernel_stats_two_chains.csv \;
  head -8 $O/trace_kernel_stats_two_chains.csv | cut -c1-160
  t=$(find /tmp/prof_b -name '*kernel_trace.csv' | head -1); [ -n "$t" ] && python3 scripts/step_anatomy.py $t $O/anatomy.json > $O/anatomy.txt 2>&1; tail -5 $O/anatomy.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/pmc_$c
    timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_$c -o p -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-lockstep-ref > $O/traffic_bench_$c.json 2> $O/traffic_bench_$c.err
    rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/traffic_bench_$c.err; exit $rc; }
  done
  python3 scripts/pmc_summary.py $O/forward_traffic.json $(find /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE -name '*counter_collection*.csv') && grep -A5 '"k_forward<false>"' $O/forward_traffic.json
fi

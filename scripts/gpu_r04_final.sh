# round-4 final validation of the in-tree build: -m gpu suite, smoke, forward
# phase stamps (diag build), full bench line, rocprof kernel stats of the bench,
# FETCH/WRITE PMC passes (HBM traffic per k_forward launch).
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_final} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 300 python scripts/net_phases.py > $O/phases.txt 2>&1; rc=$?; tail -12 $O/phases.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/prof_b && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_b -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || { tail -5 $O/bench_under_rocprof.err; exit 1; }
find /tmp/prof_b -name '*kernel_stats.csv' -exec cp {} $O/trace_kernel_stats_two_chains.csv \;
head -8 $O/trace_kernel_stats_two_chains.csv | cut -c1-160
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$c
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_$c -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated > $O/traffic_bench_$c.json 2> $O/traffic_bench_$c.err
  rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/traffic_bench_$c.err; exit $rc; }
done
python3 scripts/pmc_summary.py $O/forward_traffic.json $(find /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE -name '*counter_collection*.csv') && grep -A5 '"k_forward<false>"' $O/forward_traffic.json
if [ -n "${LV:-}" ]; then
  for r in 1 2; do
    for v in $LV; do
      SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_${v}_$r.json 2> $O/learner_${v}_$r.err || { tail -3 $O/learner_${v}_$r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/learner_${v}_$r.json'));print('== $v $r', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
    done
  done 2>&1 | tee $O/learner_variants.txt
fi
# L2 hit rate of the tree kernels (the descent's per-level record loads)
if [ -n "${TREE_PMC:-}" ]; then
  rm -rf /tmp/pmc_tcc && timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pmc_tcc -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/tcc_bench.json 2> $O/tcc_bench.err || { tail -5 $O/tcc_bench.err; exit 1; }
  python3 scripts/pmc_summary.py $O/tree_l2.json $(find /tmp/pmc_tcc -name '*counter_collection*.csv') && grep -B1 -A4 '"k_expand_select' $O/tree_l2.json | head -30
fi

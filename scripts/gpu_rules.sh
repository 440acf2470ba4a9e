# Rules-kernel measurement (scripts/rules_bench.py): HIP-event JSON, a rocprofv3
# kernel-trace/stats run, and two --pmc passes (FETCH_SIZE, WRITE_SIZE) for HBM bytes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/rules
mkdir -p $OUT
timeout -k 10 300 python3 scripts/rules_bench.py > $OUT/rules.json 2> $OUT/rules.err || { tail -20 $OUT/rules.err; exit 1; }
cat $OUT/rules.json
rm -rf /tmp/rt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rt -o r -- \
  python3 scripts/rules_bench.py --iters 5 > $OUT/rules_under_rocprof.json 2> $OUT/rt.err || { tail -20 $OUT/rt.err; exit 1; }
for f in $(find /tmp/rt -name '*kernel_stats.csv'); do cp $f $OUT/trace_kernel_stats.csv; done
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_$c -o p -- \
    python3 scripts/rules_bench.py --iters 3 > $OUT/pmc_$c.json 2> $OUT/pmc_$c.err
  rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/pmc_$c.err; exit $rc; }
done
python3 scripts/pmc_summary.py $OUT/traffic.json $(find /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE -name '*counter_collection*.csv')

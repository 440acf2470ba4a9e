# HBM traffic of the bench workload's kernels: separate rocprofv3 --pmc passes
# for FETCH_SIZE and WRITE_SIZE (they do not fit one pass), summarised per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-tr}
mkdir -p gpurun_out/traffic_$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$c
  timeout -k 10 900 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_$c -o p -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/traffic_$TAG/bench_$c.json 2> gpurun_out/traffic_$TAG/bench_$c.err
  rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/traffic_$TAG/bench_$c.err; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/traffic_$TAG/summary.json $(find /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE -name '*counter_collection*.csv') && mkdir -p gpurun_out/traffic_$TAG/csv && for f in $(find /tmp/pmc_FETCH_SIZE /tmp/pmc_WRITE_SIZE -name "*counter_collection*.csv"); do gzip -c $f > gpurun_out/traffic_$TAG/csv/$(basename $(dirname $(dirname $f)))_$(basename $f).gz; done

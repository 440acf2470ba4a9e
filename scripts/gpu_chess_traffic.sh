# HBM traffic per chess forward launch: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over the chess bench workload (first move of 1024 games), summarised per launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_chess
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/cpmc_$c
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d /tmp/cpmc_$c -o p -- \
    python3 scripts/chess_bench.py --moves 1 --no-cpu-baseline > gpurun_out/traffic_chess/bench_$c.json 2> gpurun_out/traffic_chess/bench_$c.err
  rc=$?; echo "pass $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/traffic_chess/bench_$c.err; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/traffic_chess/summary.json $(find /tmp/cpmc_FETCH_SIZE /tmp/cpmc_WRITE_SIZE -name '*counter_collection*.csv')

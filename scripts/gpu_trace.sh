set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -f gpurun_out/moves.csv
SPAI_TRACE_MOVES=gpurun_out/moves.csv timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_trace.json 2>&1
rc=$?; tail -c 300 gpurun_out/bench_trace.json; echo; echo rc=$rc; exit $rc

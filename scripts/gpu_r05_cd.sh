# sessions c and d back to back without their parity tests (run by the full suite first)
set -o pipefail
cd $GRAFT_REPO_ROOT
SKIP_TESTS=1 bash scripts/gpu_r05_c.sh && SKIP_TESTS=1 bash scripts/gpu_r05_d.sh
O=gpurun_out/r05cd && mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_stdout.txt 2> $O/bench_stderr.txt; rc=$?
echo "bench rc=$rc stdout lines: $(wc -l < $O/bench_stdout.txt)"; head -c 300 $O/bench_stdout.txt; echo

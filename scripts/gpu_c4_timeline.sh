# C4 bench under rocprofv3 --kernel-trace (timestamps) for a gap analysis
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf /tmp/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl -o tl -- \
    python3 bench.py --steps 1 --warmup 0 --sims 64 --no-cpu-baseline > gpurun_out/tl_bench.json 2> gpurun_out/tl_bench.err
rc=$?; echo "rc=$rc"
f=$(find /tmp/tl -name '*kernel_trace.csv' | head -1)
python3 scripts/timeline_gaps.py "$f" > gpurun_out/tl_gaps.txt 2>&1; cat gpurun_out/tl_gaps.txt
exit $rc

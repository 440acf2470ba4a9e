# Config C3 (sharded self-play + DP learner over RCCL) and C5 (train_concurrent pipeline)
# records on one GPU, the learner throughput record and its rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c3c5}; mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "learner or pipeline" \
    --timeout 200 --timeout-method thread > $O/pytest_learner.log 2>&1 || { tail -20 $O/pytest_learner.log; exit 1; }
tail -1 $O/pytest_learner.log
timeout -k 10 600 python scripts/c3_selfplay_dp.py ${C3_ARGS:-} > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
cat $O/c3.json
timeout -k 10 600 python scripts/pipeline_bench.py ${C5_ARGS:-} > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
cat $O/c5.json
timeout -k 10 300 python scripts/learner_dp.py --steps 100 > $O/learner.json 2> $O/learner.err || { tail -5 $O/learner.err; exit 1; }
cat $O/learner.json
rm -rf /tmp/prof_learner
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_learner -o trace -- \
    python3 scripts/learner_dp.py --steps 50 > $O/learner_prof.json 2> $O/learner_prof.err || { tail -5 $O/learner_prof.err; exit 1; }
mkdir -p $O/prof_learner && find /tmp/prof_learner -name '*stats*.csv' -exec cp {} $O/prof_learner/ \;
head -12 $O/prof_learner/*kernel_stats*.csv | cut -c1-200

# Round 5 session d: the learner with the trunk's BatchNorm fused into the next
# conv's staging (BnIn) -- learner parity tests (oracle, DDP restatement, torch
# goldens), then an interleaved throughput A/B against SPAI_LEARNER_BN_FUSE=0
# (one k_bn_fwd kernel per conv) and a rocprof kernel summary of the fused step.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05d} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_learner_dp_gpu.py tests/test_gpu_parity.py -k "learner" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
  rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_learner.log | tail -15; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for v in SPAI_LEARNER_BN_FUSE=0 SPAI_LEARNER_BNB_FUSE=0 SPAI_LEARNER_BN_FUSE=1; do
    n=$(echo $v | tr '=' '_')_$r
    env $v timeout -k 10 200 python scripts/learner_dp.py --steps 300 > $O/learner_$n.json 2> $O/learner_$n.err || { tail -3 $O/learner_$n.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/learner_$n.json') if l.startswith('{')][-1]);print('$n', round(d['value']), 'samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
rm -rf /tmp/lprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lprof -o lp -- python3 scripts/learner_dp.py --steps 100 > $O/learner_prof.json 2> $O/learner_prof.err; rc=$?; echo "rocprof rc=$rc"
f=$(find /tmp/lprof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/learner_kernel_stats.csv && head -25 $O/learner_kernel_stats.csv | cut -c1-160

# Round 5 session f: the learner's BatchNorm hand-off merged inside the producer
# conv (last-arriving workgroup per channel slice) -- learner parity tests and the
# bench entry tests (streamed default), a fused vs unfused learner A/B, rocprof of
# the fused step, then one default bench line (streamed headline + lockstep ref)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05f} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_learner_dp_gpu.py tests/test_gpu_parity.py tests/test_configs_gpu.py -k "learner or bench" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_learner.log | tail -20; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest_learner.log | head -20; exit $rc; }
for r in 1 2; do
  for v in SPAI_LEARNER_BN_FUSE=0 SPAI_LEARNER_BNB_FUSE=0 SPAI_LEARNER_BN_FUSE=1; do
    n=$(echo $v | tr '=' '_')_$r
    env $v timeout -k 10 200 python scripts/learner_dp.py --steps 300 > $O/learner_$n.json 2> $O/learner_$n.err || { tail -3 $O/learner_$n.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/learner_$n.json') if l.startswith('{')][-1]);print('$n', round(d['value']), 'samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
rm -rf /tmp/lprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lprof -o lp -- python3 scripts/learner_dp.py --steps 100 > $O/learner_prof.json 2> $O/learner_prof.err; rc=$?; echo "rocprof rc=$rc"
f=$(find /tmp/lprof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/learner_kernel_stats.csv
timeout -k 10 400 python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err; rc=$?; echo "bench rc=$rc"
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().splitlines()[-1]); print(round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4), 'lockstep', round(d['lockstep']['value']/1e6,3), round(d['lockstep']['frac'],4))"

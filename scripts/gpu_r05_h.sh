# Round 5 session h: the plain learner convs with two samples per workgroup
# (k_conv_mfma_spw) -- learner parity tests, an interleaved A/B against the
# one-sample build (build_exp/libspai_spw1.so), rocprof of the step
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05h} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_learner_dp_gpu.py tests/test_gpu_parity.py -k "learner" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_learner.log | tail -2; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_learner.log | head -20; exit $rc; }
for r in 1 2; do
  for v in default spw1; do
    L=""; [ $v = spw1 ] && L=build_exp/libspai_spw1.so
    SPAI_LIB=$L timeout -k 10 200 python scripts/learner_dp.py --steps 300 > $O/learner_${v}_$r.json 2> $O/learner_${v}_$r.err || { tail -3 $O/learner_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/learner_${v}_$r.json') if l.startswith('{')][-1]);print('${v}_$r', round(d['value']), 'samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
rm -rf /tmp/lprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lprof -o lp -- python3 scripts/learner_dp.py --steps 100 > $O/learner_prof.json 2> $O/learner_prof.err; rc=$?; echo "rocprof rc=$rc"
f=$(find /tmp/lprof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f $O/learner_kernel_stats.csv && head -12 $O/learner_kernel_stats.csv | cut -d, -f1-8 | cut -c1-150

# Round 5 session n: spai_learner_train_batches (k steps per call, one host sync)
# -- the equivalence test with the other learner tests, then an interleaved A/B of
# one step per call against 20 per call (scripts/learner_dp.py --group)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05n} && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_learner_dp_gpu.py tests/test_gpu_parity.py -k "learner" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_learner.log | tail -2; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_learner.log | head -20; exit $rc; }
for r in 1 2; do
  for g in 1 20; do
    timeout -k 10 200 python scripts/learner_dp.py --steps 300 --group $g > $O/learner_g${g}_$r.json 2> $O/learner_g${g}_$r.err || { tail -3 $O/learner_g${g}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/learner_g${g}_$r.json') if l.startswith('{')][-1]);print('g${g}_$r', round(d['value']), 'samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done

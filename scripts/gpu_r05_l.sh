# Round 5 session l: the learner step as a hipGraph (SPAI_LEARNER_GRAPH=1, captured
# once per batch size) -- learner parity tests under the graph, then an
# interleaved eager vs graph A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05l} && mkdir -p $O
SPAI_LEARNER_GRAPH=1 timeout -k 10 600 python -u -m pytest tests/test_learner_dp_gpu.py tests/test_gpu_parity.py -k "learner" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_learner_graph.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_learner_graph.log | tail -2; echo "pytest rc=$rc"; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_learner_graph.log | head -20; exit $rc; }
for r in 1 2; do
  for v in SPAI_LEARNER_GRAPH=0 SPAI_LEARNER_GRAPH=1; do
    n=$(echo $v | tr '=' '_')_$r
    env $v timeout -k 10 200 python scripts/learner_dp.py --steps 300 > $O/learner_$n.json 2> $O/learner_$n.err || { tail -3 $O/learner_$n.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/learner_$n.json') if l.startswith('{')][-1]);print('$n', round(d['value']), 'samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
rm -rf /tmp/lg
SPAI_LEARNER_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/lg -o lg -- python3 scripts/learner_dp.py --steps 60 > $O/learner_graph_trace.json 2> $O/learner_graph_trace.err; rc=$?; echo "rocprof rc=$rc"
t=$(find /tmp/lg -name '*kernel_trace.csv' | head -1); [ -n "$t" ] && python3 scripts/stream_gaps.py $t | tee $O/stream_gaps_graph.txt

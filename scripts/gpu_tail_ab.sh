# tail run-on mode A/B: the search / self-play parity tests on the default build,
# then bench.py with the mode on (default) and off (SPAI_TAIL_LEAVES=0),
# interleaved twice, each with the per-move trace
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-tail} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_abi_c.py tests/test_fullsize_gpu.py} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for v in on off; do
    E=""; [ $v = off ] && E="SPAI_TAIL_LEAVES=0"
    env $E SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v $r', round(d['value']/1e6,2), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done

# round-4 session n: tail mode uncapped (one pass, a check per pass) after a
# search call that evaluated nothing.  Search/self-play parity on that build, then
# the A/B against the committed build (adv)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_n} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
SPAI_LIB=$PWD/build_exp/libspai_uc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_fullsize_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_uc.log 2>&1
rc=$?; tail -2 $O/pytest_uc.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_uc.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in adv uc; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step', 'select', round(d['kernel_ms']['select']*1e3,2))"
  done
done

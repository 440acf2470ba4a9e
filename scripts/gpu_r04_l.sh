# round-4 session l: the move step on the device (search.hip k_advance: sampling
# and the new root on the device, the next move launched before the host's
# bookkeeping).  Full GPU suite on the in-tree build, then the A/B against the
# committed build (base)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_l} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for v in base adv al8; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done
# the aligned children blocks (SPAI_CHILD_ALIGN=8) through the search/self-play parity tests
SPAI_LIB=$PWD/build_exp/libspai_al8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_al8.log 2>&1
rc=$?; tail -2 $O/pytest_al8.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_al8.log | head -20; exit $rc; }
# three search chains (SPAI_CHAINS=3, the group-size policy at conc = 3) on the new build
for r in 1 2; do
  SPAI_CHAINS=3 SPAI_LIB=$PWD/build_exp/libspai_adv.so SPAI_TRACE_MOVES=$PWD/$O/moves_ch3_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_ch3_$r.json 2> $O/bench_ch3_$r.err || { tail -3 $O/bench_ch3_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_ch3_$r.json'));print('ch3 $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
done

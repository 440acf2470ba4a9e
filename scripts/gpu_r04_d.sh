# round-4 session d: tail-mode parity on the in-tree build, then the tail policy
# A/B: SPAI_TAIL_TREE_EVALS (tail mode once no tree of the previous search call
# evaluated that many leaves; 0 = off, the average-only policy of session c)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_d} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for tt in 0 16 48 128; do
    SPAI_TAIL_TREE_EVALS=$tt SPAI_TRACE_MOVES=$PWD/$O/moves_t${tt}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_t${tt}_$r.json 2> $O/bench_t${tt}_$r.err || { tail -3 $O/bench_t${tt}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_t${tt}_$r.json'));print('tail_tree $tt run $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done

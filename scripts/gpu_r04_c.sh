# round-4 session c: search parity on the new build, then interleaved A/B benches
# of the search library (old: one PUCT shuffle per level, per-level backup loads;
# new: DPP argmax, batched backups, tail mode at < 0.05 leaves/iteration) and the
# learner library (old / new k_wgrad_reduce)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_c} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_abi_c.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for v in old new; do
    E=""; [ $v = old ] && E="SPAI_TAIL_LEAVES=0"
    env $E SPAI_LIB=$PWD/build_exp/libspai_search_$v.so SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('search $v $r', round(d['value']/1e6,2), 'M sims/s', round(d['ms_per_step'],1), 'ms/step', 'select', round(d['kernel_ms']['select']*1e3,1), 'us')"
  done
done
for r in 1 2; do
  for v in lr_old lr_new; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_${v}_$r.json 2> $O/learner_${v}_$r.err || { tail -3 $O/learner_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/learner_${v}_$r.json'));print('learner $v $r', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
  done
done

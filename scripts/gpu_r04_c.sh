# round-4 session c: parity on the in-tree build (v3), then interleaved A/B benches
# of the search library variants:
#   old  round-3 search (one PUCT shuffle per level, per-level backup loads)
#   new  DPP argmax, batched backups, tail mode at < 0.05 leaves/iteration
#   v2   + column lanes, 64-bit key argmax, branch-free level
#   v3   + forward launch constants loaded at kernel entry (the in-tree library)
# the forward phase stamps of the base and prologue diagnostic builds, and the
# learner library (old / new k_wgrad_reduce)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_c} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_abi_c.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for v in base pro; do
  SPAI_LIB=$PWD/build_exp/libspai_diag_$v.so timeout -k 10 300 python scripts/net_phases.py > $O/phases_$v.txt 2>&1 || { tail -5 $O/phases_$v.txt; exit 1; }
  echo "== $v"; grep -E "^S=(1|4|8):" $O/phases_$v.txt | cut -c1-60,200-330
done
for r in 1 2; do
  for v in old new v2 v3; do
    E=""; [ $v = old ] && E="SPAI_TAIL_LEAVES=0"
    env $E SPAI_LIB=$PWD/build_exp/libspai_search_$v.so SPAI_TRACE_MOVES=$PWD/$O/moves_${v}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rules-bench --no-chess > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -3 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('search $v $r', round(d['value']/1e6,2), 'M sims/s', round(d['ms_per_step'],1), 'ms/step', 'select', round(d['kernel_ms']['select']*1e3,1), 'us', 'fwd', round(d['kernel_ms']['evaluate']*1e3,1), 'us', 'iso1006', round(d['roofline']['isolated']['1006']['ms']*1e3,2))"
  done
done
for r in 1 2; do
  for v in lr_old lr_new; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_${v}_$r.json 2> $O/learner_${v}_$r.err || { tail -3 $O/learner_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/learner_${v}_$r.json'));print('learner $v $r', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
  done
done

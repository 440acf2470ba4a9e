# round-4 session h: parity of the in-tree build (forward group size chosen for two
# concurrent search chains: group_size_conc), then the A/B against the
# latency-optimal group size (SPAI_FWD_CONC=0), same library
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_h} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_abi_c.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for c in 0 1; do
    SPAI_FWD_CONC=$c SPAI_TRACE_MOVES=$PWD/$O/moves_c${c}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_c${c}_$r.json 2> $O/bench_c${c}_$r.err || { tail -3 $O/bench_c${c}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_c${c}_$r.json'));print('conc $c run $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us', 'leaves/launch', round(d['roofline']['avg_leaves_per_launch'],1))"
  done
done

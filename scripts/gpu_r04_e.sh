# round-4 session e: tail-mode parity (run cap) on the in-tree build, the launch
# prologue's phase stamps (diagnostic entry build), then the tail policy A/B:
# SPAI_TAIL_TREE_EVALS x SPAI_TAIL_RUN
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r04_e} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest.log | head -20; exit $rc; }
SPAI_PRINT_ENTRY=1 SPAI_LIB=$PWD/build_exp/libspai_diag_entry.so timeout -k 10 300 python scripts/net_phases.py > $O/phases_entry.txt 2>&1 || { tail -5 $O/phases_entry.txt; exit 1; }
grep -E "^S=(1|4|8):|entry \(" $O/phases_entry.txt | cut -c1-150
for r in 1 2; do
  for cfg in "0 64" "48 64" "160 64" "160 32"; do
    set -- $cfg; tt=$1; tr=$2
    SPAI_TAIL_TREE_EVALS=$tt SPAI_TAIL_RUN=$tr SPAI_TRACE_MOVES=$PWD/$O/moves_t${tt}_r${tr}_$r.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_t${tt}_r${tr}_$r.json 2> $O/bench_t${tt}_r${tr}_$r.err || { tail -3 $O/bench_t${tt}_r${tr}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_t${tt}_r${tr}_$r.json'));print('tail_tree $tt run $tr rep $r', round(d['value']/1e6,3), 'M sims/s', round(d['ms_per_step'],1), 'ms/step')"
  done
done

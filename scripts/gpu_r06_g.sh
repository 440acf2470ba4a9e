# Round 6 session g: the two-tap final phase (SPAI_FINAL2, DA = 6 at S >= 5) against the
# default and a DA = 6-only build: net tests and bit-identity with the default, phase
# stamps, isolated forward, interleaved streamed benches
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06g} && mkdir -p $O
V=${VAR:-final2}
SPAI_LIB=build_exp/libspai_$V.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "net_ or search_chain or bf16" > $O/pytest_$V.log 2>&1; rc=$?; tail -2 $O/pytest_$V.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/net_dump.py $O/dump_default.npz && SPAI_LIB=build_exp/libspai_$V.so timeout -k 10 120 python3 scripts/net_dump.py $O/dump_$V.npz && python3 scripts/net_dump.py --compare $O/dump_default.npz $O/dump_$V.npz || exit 1
for v in diag diag_$V diag_da6; do
  SPAI_LIB=build_exp/libspai_$v.so timeout -k 10 120 python3 scripts/net_phases.py > $O/p_$v.txt 2>&1 || { tail -20 $O/p_$v.txt; exit 1; }
  echo "== $v"; grep "^  stem" $O/p_$v.txt | head -1; grep "^S=[4-8]" $O/p_$v.txt | cut -c1-120
done
timeout -k 10 400 python3 scripts/fwd_sweep.py --libs self-play-ai_amd/libspai.so,build_exp/libspai_$V.so,build_exp/libspai_da6.so --counts 1024,1539,2048,3078,4096 --conc 2 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for r in 1 2; do
  for v in self-play-ai_amd/libspai.so build_exp/libspai_$V.so; do
    n=$(basename $v .so)_$r
    SPAI_LIB=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4))"
  done
done

# Round 6 session j: the pair-split task plan at the large group sizes (each wave two co
# tiles over half the position tiles: half the weight fragments per CU and k-step) --
# S = 5..8 (pair) or S = 5..6 (pair18): tests and bit-identity, phase stamps, isolated
# forward, interleaved streamed benches
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06j} && mkdir -p $O
timeout -k 10 120 python3 scripts/net_dump.py $O/dump_default.npz || exit 1
for V in pair pair18; do
  SPAI_LIB=build_exp/libspai_$V.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "net_ or search_chain or bf16" > $O/pytest_$V.log 2>&1; rc=$?; tail -1 $O/pytest_$V.log; [ $rc -eq 0 ] || exit $rc
  SPAI_LIB=build_exp/libspai_$V.so timeout -k 10 120 python3 scripts/net_dump.py $O/dump_$V.npz && python3 scripts/net_dump.py --compare $O/dump_default.npz $O/dump_$V.npz || exit 1
done
for v in diag diag_pair diag_pair18; do
  SPAI_LIB=build_exp/libspai_$v.so timeout -k 10 120 python3 scripts/net_phases.py > $O/p_$v.txt 2>&1 || { tail -20 $O/p_$v.txt; exit 1; }
  echo "== $v"; grep "^  stem" $O/p_$v.txt | head -1; grep "^S=[5-8]" $O/p_$v.txt | cut -c1-110
done
timeout -k 10 400 python3 scripts/fwd_sweep.py --libs self-play-ai_amd/libspai.so,build_exp/libspai_pair.so,build_exp/libspai_pair18.so --counts 1024,1539,2048,3078,4096 --conc 2 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for r in 1 2; do
  for v in self-play-ai_amd/libspai.so build_exp/libspai_pair.so build_exp/libspai_pair18.so; do
    n=$(basename $v .so)_$r
    SPAI_LIB=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4))"
  done
done

# Round 5 session j: the C4 forward's ring depths at S >= 5 (weights DA - 1 k-steps
# ahead, activations DB - 1): default DA 3 / DB 2 against DA 6 (build_exp/
# libspai_da8_6.so) and DB 3 (libspai_db8_3.so), streamed bench with the isolated
# forward, interleaved, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05j} && mkdir -p $O
for r in 1 2; do
  for L in self-play-ai_amd/libspai.so build_exp/libspai_da8_6.so build_exp/libspai_db8_3.so; do
    n=$(basename $L .so)_$r
    SPAI_LIB=$L timeout -k 10 300 python3 bench.py --steps ${SSTEPS:-5} --warmup 1 --no-cpu-baseline --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); r=d['roofline']
print('$n', round(d['value']/1e6,3), 'M sims/s', round(r['frac'],4), round(d['ms_per_step'],1), 'ms/step', {k: round(v['frac'],4) for k, v in r['isolated'].items()})"
  done
done

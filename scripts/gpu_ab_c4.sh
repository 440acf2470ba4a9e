# A/B of net_c4 variants: head phases (diag builds) + short bench runs (prod builds), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab_c4; mkdir -p $OUT
for v in ${DIAGS:-}; do
  echo "== phases $v"; SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 120 python scripts/net_head_phases.py || exit 1
done 2>&1 | tee $OUT/phases.txt
for r in 1 2; do
  for v in base ${VARS:-}; do
    if [ $v = base ]; then L=$PWD/self-play-ai_amd/libspai.so; else L=$PWD/build_exp/libspai_$v.so; fi
    SPAI_LIB=$L timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_${v}_$r.json 2> $OUT/bench_${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us', 'frac', round(d['roofline']['frac'],4))"
  done
done 2>&1 | tee $OUT/bench.txt

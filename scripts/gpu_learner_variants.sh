# learner variants (build_exp/libspai_<tag>.so from scripts/build_learner_variant.sh):
# first-step gradient error vs the float64 restatement and training throughput
cd $GRAFT_REPO_ROOT && O=gpurun_out/lvar && mkdir -p $O
for v in base ${VARIANTS:-}; do
  if [ $v = base ]; then unset SPAI_LIB; else export SPAI_LIB=$PWD/build_exp/libspai_$v.so; fi
  for cfg in "6 128" "2 128"; do
    timeout -k 10 100 python scripts/learner_grad_debug.py $cfg > $O/dbg_${v}_${cfg// /_}.txt 2>&1 || { tail -3 $O/dbg_${v}_${cfg// /_}.txt; exit 1; }
    echo "== $v $cfg: $(sed -n 2p $O/dbg_${v}_${cfg// /_}.txt)"
  done
  timeout -k 10 200 python scripts/learner_dp.py --steps 100 > $O/learner_$v.json 2> $O/learner_$v.err || { tail -3 $O/learner_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/learner_$v.json'));print('== $v', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
done

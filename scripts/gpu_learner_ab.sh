# learner throughput A/B: the in-tree build against build_exp/libspai_<v>.so variants
# (scripts/build_learner_variant.sh), base measured first and last
cd $GRAFT_REPO_ROOT && O=gpurun_out/lvar2 && mkdir -p $O
for v in base ${VARIANTS:-} base; do
  if [ $v = base ]; then unset SPAI_LIB; else export SPAI_LIB=$PWD/build_exp/libspai_$v.so; fi
  timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_$v.json 2> $O/learner_$v.err || { tail -3 $O/learner_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/learner_$v.json'));print('== $v', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
done

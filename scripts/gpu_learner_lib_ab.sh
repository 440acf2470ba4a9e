# learner throughput A/B of build_exp/libspai_<v>.so variants (interleaved, 2 rounds),
# learner parity tests on the in-tree build first
#   LV="a b" bash scripts/gpu_learner_lib_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-learner_ab} && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py -m gpu -x -q -p no:cacheprovider -k "learner or c3" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for v in $LV; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_${v}_$r.json 2> $O/learner_${v}_$r.err || { tail -3 $O/learner_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/learner_${v}_$r.json'));print('== $v $r', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
  done
done 2>&1 | tee $O/learner.txt

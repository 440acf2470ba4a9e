# Forward prologue A/B (SPAI_EARLY_PARAMS; the experiment is
# profiles/r02/forward/early_params_experiment.patch): the -m gpu suite on the new build, isolated sweeps of both builds, interleaved benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-early}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python scripts/fwd_sweep.py --libs build_exp/libspai_base.so,build_exp/libspai_early.so \
      --counts 40,256,1006,2012,4096 > $O/sweep_$r.txt 2>&1
  rc=$?; cat $O/sweep_$r.txt; [ $rc -eq 0 ] || exit $rc
done
VARS="base early" ROUNDS=3 STEPS=2 TAG=${TAG:-early} bash scripts/gpu_bench_ab.sh

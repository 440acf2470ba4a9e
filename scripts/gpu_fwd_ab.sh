# forward-alone A/B of library builds (scripts/fwd_sweep.py), two interleaved rounds,
# then the net / search parity tests on the default build
#   LIBS="build_exp/libspai_a.so,build_exp/libspai_b.so" TAG=x bash scripts/gpu_fwd_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fwdab}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python scripts/fwd_sweep.py --libs $LIBS --counts ${COUNTS:-256,512,1024,1300,1536,1792,2048,4096} > $O/sweep_$r.txt 2>&1 || { cat $O/sweep_$r.txt; exit 1; }
  cat $O/sweep_$r.txt
done
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; exit $rc
fi

# current build: net/search parity tests + phase stamps (diag build); A/B of build_exp/libspai_base.so vs
# build_exp/libspai_$NEW.so: forward-alone sweeps and bench runs
cd $GRAFT_REPO_ROOT && O=gpurun_out/${TAG:-abfull} && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_fullsize_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "net or search or self_play or c2" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 120 python scripts/net_phases.py > $O/phases.txt 2>&1 || { cat $O/phases.txt; exit 1; }
tail -8 $O/phases.txt
LIBS=build_exp/libspai_base.so,build_exp/libspai_$NEW.so TAG=${TAG:-abfull} bash scripts/gpu_fwd_ab.sh || exit 1
VARS="base $NEW" ROUNDS=2 TAG=${TAG:-abfull} bash scripts/gpu_bench_ab.sh

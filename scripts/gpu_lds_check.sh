# correctness of the current build (net + search parity), then forward-alone and bench A/B vs build_exp/libspai_base.so
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/${TAG:-lds} && O=gpurun_out/${TAG:-lds}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_chess_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "net or search or self_play" > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS=build_exp/libspai_base.so,build_exp/libspai_lds.so TAG=${TAG:-lds} bash scripts/gpu_fwd_ab.sh || exit 1
VARS="base lds" ROUNDS=2 TAG=${TAG:-lds} bash scripts/gpu_bench_ab.sh

cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02i && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp32.py tests/test_fullsize_gpu.py tests/test_gpu_faults.py tests/test_abi_c.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not c4c" > gpurun_out/r02i/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r02i/pytest.log; [ $rc -eq 0 ] || exit $rc
VARS="base fused" ROUNDS=2 TAG=r02i bash scripts/gpu_bench_ab.sh

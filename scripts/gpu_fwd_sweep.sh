cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02d && \
timeout -k 10 300 python scripts/fwd_sweep.py --libs self-play-ai_amd/libspai.so,build_exp/libspai_noA.so,build_exp/libspai_noepi.so,build_exp/libspai_afixed.so > gpurun_out/r02d/fwd_sweep.txt 2>&1; rc=$?; cat gpurun_out/r02d/fwd_sweep.txt; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02d/bench.json 2> gpurun_out/r02d/bench.err; rc=$?; cat gpurun_out/r02d/bench.json; tail -3 gpurun_out/r02d/bench.err; exit $rc

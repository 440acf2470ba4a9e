# epilogue store-width experiment: phase stamps (diag builds) and forward-alone sweep
cd $GRAFT_REPO_ROOT && O=gpurun_out/${TAG:-epi} && mkdir -p $O
for v in diag diag128; do
  echo "== $v"; SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 120 python scripts/net_phases.py 2>&1 | tail -8 || exit 1
done > $O/phases.txt; cat $O/phases.txt
LIBS=build_exp/libspai_base.so,build_exp/libspai_epi128.so TAG=${TAG:-epi} bash scripts/gpu_fwd_ab.sh

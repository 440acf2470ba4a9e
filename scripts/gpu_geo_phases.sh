# phase stamps: diagnostic build vs the same with the geometry forced before the stem's barrier
cd $GRAFT_REPO_ROOT && O=gpurun_out/${TAG:-geo} && mkdir -p $O
for v in diag diaggeo; do
  echo "== $v"; SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 120 python scripts/net_phases.py 2>&1 | tail -8 || exit 1
done > $O/phases_geo.txt; cat $O/phases_geo.txt

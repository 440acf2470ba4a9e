# Round 6 session h: epilogue stores at conflict-free addresses (timing only) vs default
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06h} && mkdir -p $O
for v in diag diag_storeb128 diag_storelin; do
  SPAI_LIB=build_exp/libspai_$v.so timeout -k 10 120 python3 scripts/net_phases.py > $O/p_$v.txt 2>&1 || { tail -20 $O/p_$v.txt; exit 1; }
  echo "== $v"; grep "^  stem" $O/p_$v.txt | head -1; grep "^S=[48]" $O/p_$v.txt | cut -c1-120
done

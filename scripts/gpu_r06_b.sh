# Round 6 session b: epilogue deletion experiments (timing only, wrong results):
# phase stamps of the diag build vs no conversion VALU / no epilogue at all / lag 3
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r06b} && mkdir -p $O
for v in diag diag_noepi diag_noepiall diag_lag3 diag; do
  echo "== $v" >> $O/phases.txt
  SPAI_LIB=build_exp/libspai_$v.so timeout -k 10 120 python3 scripts/net_phases.py > $O/p_$v.txt 2>&1 || { tail -20 $O/p_$v.txt; exit 1; }
  grep "^S=\|^  stem" $O/p_$v.txt >> $O/phases.txt
done
cat $O/phases.txt

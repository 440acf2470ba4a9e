# forward phase stamps (scripts/net_phases.py) for each diagnostic library variant
#   VARIANTS="base noa nob" TAG=x bash scripts/gpu_diag_phases.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-diag} && mkdir -p $O
for v in ${VARIANTS:-base}; do
  SPAI_LIB=$PWD/build_exp/libspai_diag_$v.so timeout -k 10 300 python scripts/net_phases.py > $O/phases_$v.txt 2>&1 || { tail -5 $O/phases_$v.txt; exit 1; }
  echo "== $v"; grep -E "^S=(1|2|4|8):" $O/phases_$v.txt | cut -c1-200
done

# run the forward phase breakdown for every variant library under build_exp/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in $(ls build_exp/*.so 2>/dev/null); do
  echo "== $lib"
  SPAI_LIB=$PWD/$lib timeout -k 10 120 python scripts/net_phases.py || exit $?
done 2>&1 | tee gpurun_out/exp_${TAG:-x}.txt

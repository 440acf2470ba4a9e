# time the chess forward of every build_exp/libspai_*.so variant (chess_quick.py, 1024 trees x 48 sims)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in $(ls build_exp/libspai_*.so); do
  echo "== $lib"
  SPAI_LIB=$PWD/$lib timeout -k 10 120 python scripts/chess_quick.py --sims 48 ${CHESS_ARGS:-} || exit $?
done 2>&1 | tee gpurun_out/chess_variants_${TAG:-x}.txt

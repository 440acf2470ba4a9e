# A/B of chess_net variants (build_exp/libspai_<v>.so) against the in-tree build: chess_quick forward timing, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  for v in base ${VARS:-}; do
    if [ $v = base ]; then L=$PWD/self-play-ai_amd/libspai.so; else L=$PWD/build_exp/libspai_$v.so; fi
    echo "== $v $r"
    SPAI_LIB=$L timeout -k 10 120 python scripts/chess_quick.py --sims 48 ${CHESS_ARGS:-} || exit 1
  done
done 2>&1 | tee gpurun_out/chess_ab.txt

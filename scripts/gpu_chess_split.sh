# chess forward work split: balanced persistent passes (in-tree build) vs P = 2 rounds
# (build_exp/libspai_rounds.so), chess_quick at several tree counts; then the chess GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/chess_split; mkdir -p $O
for t in ${TREES:-300 520 600 700 800 1024}; do
  for v in base rounds; do
    if [ $v = base ]; then L=$PWD/self-play-ai_amd/libspai.so; else L=$PWD/build_exp/libspai_$v.so; fi
    SPAI_LIB=$L timeout -k 10 120 python scripts/chess_quick.py --trees $t --sims 48 > $O/q_${v}_$t.json 2> $O/q_${v}_$t.err || { tail -3 $O/q_${v}_$t.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/q_${v}_$t.json'));print('$v', $t, 'leaves %.0f'%d['leaves_per_forward'], 'fwd ms %.3f'%(d['kernel_ms'][1]/d['launches'][1]), 'TF %.0f'%d['forward_tflops'], 'sims/s %.0f'%d['sims_per_s'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_chess_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_chess.log 2>&1; rc=$?; tail -2 $O/pytest_chess.log; exit $rc

# forward-only kernel time: production library vs the 2-workgroups-per-CU experiment
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in prod duo duo2; do
  lib=$PWD/self-play-ai_amd/libspai.so; [ $v != prod ] && lib=$PWD/build_duo/libspai_$v.so
  SPAI_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/duo_$v -o run -- python3 scripts/net_forward_bench.py 4096 20 > /dev/null 2>&1 || exit $?
  f=$(find gpurun_out/duo_$v -name '*kernel_stats.csv' | head -1); echo "== $v"; cat "$f" | cut -d, -f1-8 | head -5
done

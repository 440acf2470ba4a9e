# build_exp/libspai_diag_<tag>.so: the diagnostic (phase-stamp) library with
# net_c4.hip under extra flags, e.g. the timing-only deletion experiments
# usage: scripts/build_diag_variant.sh tag "-DFLAG ..." [tag "-D..."]...
set -e
# UNROLL: extra unroll flags for the variant (e.g. -mllvm -pragma-unroll-threshold=1000000)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/self-play-ai_amd
make -s -j8
mkdir -p ../build_exp
tags=""
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2; tags="$tags $tag"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $UNROLL -DSPAI_DIAG $flags -c csrc/net_c4.hip -o ../build_exp/net_c4_diag_$tag.o &
done
wait
objs=$(ls build/*.o | grep -v "net_c4.hip.o\|net_c4_diag")
for tag in $tags; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build_exp/libspai_diag_$tag.so $objs ../build_exp/net_c4_diag_$tag.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build_exp/libspai_diag_$tag.so"
done

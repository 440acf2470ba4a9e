# build_exp/libspai_<tag>.so: the library with net_c4.hip rebuilt under extra flags
# usage: scripts/build_c4_variant.sh tag "-DFLAG=..." [tag "-D..."]...
set -e
# UNROLL: extra unroll flags for the variant (e.g. -mllvm -pragma-unroll-threshold=1000000)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/self-play-ai_amd
make -s -j8
mkdir -p ../build_exp
tags=""
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2; tags="$tags $tag"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $UNROLL $flags -c csrc/net_c4.hip -o ../build_exp/net_c4_$tag.o &
done
wait
objs=$(ls build/*.o | grep -v "net_c4.hip.o\|net_c4_diag")
for tag in $tags; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build_exp/libspai_$tag.so $objs ../build_exp/net_c4_$tag.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build_exp/libspai_$tag.so"
done

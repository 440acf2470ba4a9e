# build_exp/libspai_<tag>.so: the library with net_c4.hip rebuilt under extra flags
# usage: scripts/build_c4_variant.sh tag "-DFLAG=..." [tag "-D..."]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/self-play-ai_amd
make -s -j8
mkdir -p ../build_exp
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags -c csrc/net_c4.hip -o ../build_exp/net_c4_$tag.o &
done
wait
for o in ../build_exp/net_c4_*.o; do
  tag=$(basename $o .o); tag=${tag#net_c4_}
  objs=$(ls build/*.o | grep -v net_c4.hip.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build_exp/libspai_$tag.so $objs $o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build_exp/libspai_$tag.so"
done

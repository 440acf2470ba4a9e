# build_exp/libspai_<tag>.so: the library with learner.hip rebuilt under extra flags (tag flags ...)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/self-play-ai_amd
make -s -j8
mkdir -p ../build_exp
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags -c csrc/learner.hip -o ../build_exp/learner_$tag.o
  objs=$(ls build/*.o | grep -v "build/learner.hip.o\|net_c4_diag")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build_exp/libspai_$tag.so $objs ../build_exp/learner_$tag.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built build_exp/libspai_$tag.so"
done

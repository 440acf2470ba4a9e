# build_exp/libspai_<tag>.so: the library with one source file rebuilt under extra flags
# usage: scripts/build_variant.sh <source, e.g. learner.hip> tag "-DFLAG=..." [tag "-D..."]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd $ROOT/self-play-ai_amd
make -s -j8
mkdir -p ../build_exp
src=$1; shift
base=${src%.*}
tags=""
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2; tags="$tags $tag"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags -c csrc/$src -o ../build_exp/${base}_$tag.o &
done
wait
objs=$(ls build/*.o | grep -v "$src.o\|net_c4_diag")
for tag in $tags; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../build_exp/libspai_$tag.so $objs ../build_exp/${base}_$tag.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm -f ../build_exp/${base}_$tag.o
  echo "built build_exp/libspai_$tag.so"
done

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in prod duo; do
  lib=$PWD/self-play-ai_amd/libspai.so; [ $v = duo ] && lib=$PWD/build_duo/libspai_duo.so
  rm -rf /tmp/dp_$v
  SPAI_LIB=$lib timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS \
    --output-format csv -d /tmp/dp_$v -o p -- python3 scripts/net_forward_bench.py 4096 10 > /dev/null 2>&1 || exit $?
  mkdir -p gpurun_out/duo_pmc_$v; find /tmp/dp_$v -name '*counter_collection*.csv' -exec cp {} gpurun_out/duo_pmc_$v/ \;
done

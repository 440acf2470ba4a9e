set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/pmc_$TAG
rocprofv3 -L > gpurun_out/pmc_$TAG/counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf /tmp/pmc$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o p -- python3 scripts/net_forward_bench.py ${FWD_N:-4096} ${FWD_REPS:-10} > gpurun_out/pmc_$TAG/run$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  find /tmp/pmc$i -name '*counter_collection*.csv' -exec cp {} gpurun_out/pmc_$TAG/pass$i.csv \;
  [ $rc -eq 0 ] || exit $rc
done
ls -la gpurun_out/pmc_$TAG

# SQ counter passes over the device learner (scripts/learner_dp.py, 20 steps), one pass per counter set
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_learner; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  rm -rf /tmp/lpmc$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d /tmp/lpmc$i -o p -- python3 scripts/learner_dp.py --steps 20 --warmup 2 > $O/run$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  find /tmp/lpmc$i -name '*counter_collection*.csv' -exec cp {} $O/pass$i.csv \;
  [ $rc -eq 0 ] || exit $rc
done
for k in "k_conv_mfma<64, 1" "k_wgrad_mfma<64>" "k_bn_bwd" "k_bn_fwd"; do
  echo "== $k"; python3 scripts/pmc_ratios.py $O "$k"
done > $O/summary.txt
cat $O/summary.txt

# round-3 learner staging/k-loop change: parity tests, throughput A/B vs the
# previous learner (build_exp/libspai_lold.so), rocprof stats and conv/wgrad PMC
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r03b_learner && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py -m gpu -x -q -p no:cacheprovider -k "learner or pipeline or c3" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head -20; exit $rc; }
for v in old new old new; do
  if [ $v = new ]; then unset SPAI_LIB; else export SPAI_LIB=$PWD/build_exp/libspai_lold.so; fi
  timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_$v.json 2> $O/learner_$v.err || { tail -3 $O/learner_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/learner_$v.json'));print('== $v', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
done
unset SPAI_LIB
rm -rf /tmp/prof_l && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l -o trace -- python3 scripts/learner_dp.py --steps 50 > $O/learner_prof.json 2> $O/learner_prof.err || { tail -5 $O/learner_prof.err; exit 1; }
mkdir -p $O/prof && find /tmp/prof_l -name '*stats*.csv' -exec cp {} $O/prof/ \;
head -8 $O/prof/*kernel_stats*.csv | cut -c1-150
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1)); rm -rf /tmp/lpmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/lpmc$i -o p -- python3 scripts/learner_dp.py --steps 20 --warmup 2 > $O/pmc_run$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  find /tmp/lpmc$i -name '*counter_collection*.csv' -exec cp {} $O/pass$i.csv \;
  [ $rc -eq 0 ] || exit $rc
done
for k in "k_conv_mfma<64, 1" "k_wgrad_mfma<64>"; do
  echo "== $k"; python3 scripts/pmc_ratios.py $O "$k"
done > $O/pmc_summary.txt
cat $O/pmc_summary.txt

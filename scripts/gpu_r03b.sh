# round-3 (session b) GPU call: full -m gpu suite on the in-tree build, learner
# A/B + stats + PMC, forward sweep A/B and bench A/B of build_exp variants.
#   FWD="lh0 lh1 hb1" BENCHV="lh0 hb1" bash scripts/gpu_r03b.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r03b} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
if [ -n "${LEARNER:-1}" ]; then
for v in old new old new; do
  if [ $v = new ]; then unset SPAI_LIB; else export SPAI_LIB=$PWD/build_exp/libspai_lold.so; fi
  timeout -k 10 200 python scripts/learner_dp.py --steps 200 > $O/learner_$v.json 2> $O/learner_$v.err || { tail -3 $O/learner_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/learner_$v.json'));print('== $v', round(d['value']), 'samples/s', round(d['ms_per_step'],3), 'ms/step')"
done
unset SPAI_LIB
rm -rf /tmp/prof_l && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l -o trace -- python3 scripts/learner_dp.py --steps 50 > $O/learner_prof.json 2> $O/learner_prof.err || { tail -5 $O/learner_prof.err; exit 1; }
mkdir -p $O/lprof && find /tmp/prof_l -name '*stats*.csv' -exec cp {} $O/lprof/ \;
head -8 $O/lprof/*kernel_stats*.csv | cut -c1-150
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1)); rm -rf /tmp/lpmc$i; mkdir -p $O/lpmc
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/lpmc$i -o p -- python3 scripts/learner_dp.py --steps 20 --warmup 2 > $O/lpmc/run$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  find /tmp/lpmc$i -name '*counter_collection*.csv' -exec cp {} $O/lpmc/pass$i.csv \;
  [ $rc -eq 0 ] || exit $rc
done
for k in "k_conv_mfma<64, 1" "k_wgrad_mfma<64>"; do
  echo "== $k"; python3 scripts/pmc_ratios.py $O/lpmc "$k"
done > $O/lpmc/summary.txt
cat $O/lpmc/summary.txt
fi
if [ -n "${FWD:-}" ]; then
  LIBS=$(for v in $FWD; do printf "build_exp/libspai_$v.so,"; done); LIBS=${LIBS%,}
  for r in 1 2; do
    timeout -k 10 300 python scripts/fwd_sweep.py --libs $LIBS --counts ${COUNTS:-40,256,512,1006,1536,2048,4096} > $O/sweep_$r.txt 2>&1 || { cat $O/sweep_$r.txt; exit 1; }
    cat $O/sweep_$r.txt
  done
fi
if [ -n "${BENCHV:-}" ]; then
for r in 1 2; do
  for v in $BENCHV; do
    SPAI_LIB=$PWD/build_exp/libspai_$v.so timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-isolated > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err || { tail -5 $O/bench_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us')"
  done
done 2>&1 | tee $O/bench.txt
fi

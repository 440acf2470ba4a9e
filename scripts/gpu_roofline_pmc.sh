# rocprofv3 --pmc passes of the bench command itself (one step of the streamed
# schedule, 4096 games x 800 sims): FETCH_SIZE, WRITE_SIZE and the SQ/GRBM set
# (executed MFMAs, MFMA busy cycles, wave-cycle split) in separate passes, combined by
# scripts/roofline_pmc.py into gpurun_out/$TAG/forward_pmc.json
#   COMMIT=$(git rev-parse --short HEAD) TAG=x bash scripts/gpu_roofline_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-rpmc}; O=gpurun_out/$TAG; mkdir -p $O
# a pass prints nothing for minutes: keep gpurun's silence watchdog informed
( while sleep 50; do date >> $O/heartbeat.txt; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
BA="--warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref ${BENCH_ARGS:-}"
# the traffic passes over one streamed step; the SQ pass over SQ_STEPS (default 2), so its
# mix of group sizes (and so executed / algorithmic MFMA FLOPs) is nearer the default run's
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/rpmc$i
  steps=1; [ $i -eq 3 ] && steps=${SQ_STEPS:-2}
  timeout -k 10 900 rocprofv3 --pmc $set --output-format csv -d /tmp/rpmc$i -o p -- python3 bench.py --steps $steps $BA > $O/bench_pass$i.json 2> $O/bench_pass$i.err
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench_pass$i.err; exit $rc; }
done
python3 scripts/roofline_pmc.py $O/forward_pmc.json $O/bench_pass3.json ${COMMIT:-unknown} $(find /tmp/rpmc1 /tmp/rpmc2 /tmp/rpmc3 -name '*counter_collection*.csv')

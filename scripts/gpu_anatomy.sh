# Anatomy of one C4 bench step: rocprofv3 kernel trace of bench.py (1 step, no
# warm-up) cut into moves at k_advance (k_root_stats before it; scripts/step_anatomy.py), plus the
# per-move host trace.  ENV_AB="VAR=val ..." runs a second traced step with those
# environment settings for comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-anatomy} && mkdir -p $O
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!; trap "kill $HB 2>/dev/null" EXIT
run() {   # $1 = label, rest = env assignments
  local L=$1; shift
  rm -rf /tmp/an_$L
  env "$@" SPAI_TRACE_MOVES=$PWD/$O/moves_$L.csv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/an_$L -o an -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess > $O/bench_$L.json 2> $O/bench_$L.err || { tail -5 $O/bench_$L.err; return 1; }
  f=$(find /tmp/an_$L -name '*kernel_trace.csv' | head -1)
  python3 scripts/step_anatomy.py "$f" $O/anatomy_$L.json ${DUMP_MOVES:-2,12,25,33,39} $O/timeline_$L.csv > $O/anatomy_$L.txt && tail -48 $O/anatomy_$L.txt
}
run base && for ab in ${ENV_AB:-}; do run $(echo $ab | tr '=,' '__') $(echo $ab | tr ',' ' ') || exit 1; done

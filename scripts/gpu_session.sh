# One GPU call: the -m gpu suite, the default bench, a per-move trace, rocprof
# kernel stats (two search chains and one), and the CPU thread sweep.
# Steps are chained: the first failure ends the call.
#   STEPS="tests bench trace prof prof1 cpusweep cpugames" TAG=r02a bash scripts/gpu_session.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
STEPS=${STEPS:-"tests bench trace prof prof1 cpusweep"}
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
stats() {   # $1 = name, rest = env for the profiled bench
  local n=$1; shift
  rm -rf /tmp/prof_$n
  env "$@" timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$n -o trace -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_prof_$n.json 2> $O/bench_prof_$n.err
  local rc=$?; echo "rocprof $n rc=$rc"; [ $rc -eq 0 ] || return $rc
  mkdir -p $O/prof_$n
  find /tmp/prof_$n -name '*stats*.csv' -exec cp {} $O/prof_$n/ \;
  head -8 $O/prof_$n/*kernel_stats*.csv
}
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
      > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
  rc=$?; cat $O/bench.json; tail -3 $O/bench.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if has trace; then
  rm -f $O/moves.csv
  SPAI_TRACE_MOVES=$O/moves.csv timeout -k 10 600 python bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      > $O/bench_trace.json 2> $O/bench_trace.err
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if has prof; then stats two SPAI_UNUSED=0 || exit $?; fi
if has prof1; then stats one SPAI_CHAINS=1 || exit $?; fi
if has ubench; then
  timeout -k 10 120 ./scripts/ubench/weight_stream > $O/ubench_weight_stream.txt 2>&1
  rc=$?; cat $O/ubench_weight_stream.txt; echo "ubench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if has cpusweep; then
  timeout -k 10 900 python scripts/cpu_games_baseline.py --out $O/cpu_sweep.json --no-games > $O/cpu_sweep.log 2>&1
  rc=$?; tail -2 $O/cpu_sweep.log; echo "cpu sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if has cpugames; then
  timeout -k 10 1100 python scripts/cpu_games_baseline.py --out $O/cpu_baseline.json ${CPU_ARGS:-} > $O/cpu_games.log 2>&1
  rc=$?; tail -2 $O/cpu_games.log; echo "cpu games rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "session done"

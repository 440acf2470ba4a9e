# Round-3 GPU session steps (one gpurun call; the first failing step ends it).
#   STEPS="newtests tests bench c5" TAG=r03a bash scripts/gpu_r03.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
STEPS=${STEPS:-"newtests tests bench"}
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $O/host.txt
( while true; do sleep 50; date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
pyt() {   # $1 = log name, rest = pytest args
  local n=$1; shift
  timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread "$@" \
      > $O/$n.log 2>&1
  local rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/$n.log | tail -60; echo "$n rc=$rc"; return $rc
}
if has newtests; then
  pyt pytest_new tests/test_configs_gpu.py tests/test_gpu_parity.py tests/test_chess_gpu.py tests/test_gpu_fp32.py -m gpu \
      -k "learner or pipeline or c3 or c5 or perft or f32_net" \
      --durations=0 || exit $?
fi
if has tests; then pyt pytest_gpu tests -m gpu --durations=15 || exit $?; fi
if has bench; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
  rc=$?; cat $O/bench.json; tail -3 $O/bench.err; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
c5() {   # $1 = name, rest = pipeline_bench args
  local n=$1; shift
  timeout -k 10 600 python scripts/pipeline_bench.py "$@" > $O/c5_$n.json 2> $O/c5_$n.err
  local rc=$?; cat $O/c5_$n.json; tail -3 $O/c5_$n.err; echo "c5 $n rc=$rc"; return $rc
}
if has c5; then
  # reference defaults (100 games x 600 sims, 4 blocks): 1 and 6 self-play workers (main.rs:169)
  c5 ref_w1 --selfplay-devices 0 || exit $?
  c5 ref_w6 --selfplay-devices 0,0,0,0,0,0 || exit $?
  # SURVEY §8d per-GPU shape: 4096-game workers, 800 sims, 6x64
  c5 g4096_w1 --selfplay-devices 0 --games 4096 --sims 800 --blocks 6 || exit $?
  c5 g4096_w6 --selfplay-devices 0,0,0,0,0,0 --games 4096 --sims 800 --blocks 6 || exit $?
fi
if has c3; then
  timeout -k 10 600 python scripts/c3_selfplay_dp.py > $O/c3.json 2> $O/c3.err
  rc=$?; cat $O/c3.json; tail -3 $O/c3.err; echo "c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0

# Round 5 session i: (1) chess forward with the issue-order hints (SPAI_CHESS_SCHED=1,
# build_exp/libspai_chsched.so) against the default, chess window, interleaved;
# (2) the C4 forward's group size under the streamed schedule: the two-chain
# model's pick against forced S = 6 / 7 and a 192-CU grid cap, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05i} && mkdir -p $O
for r in 1 2; do
  for L in self-play-ai_amd/libspai.so build_exp/libspai_chsched.so; do
    n=$(basename $L .so)_$r
    SPAI_LIB=$L timeout -k 10 300 python3 scripts/chess_bench.py --moves 2 --no-cpu-baseline > $O/chess_$n.json 2> $O/chess_$n.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/chess_$n.err; exit $rc; }
    python3 -c "import json; d=json.loads([l for l in open('$O/chess_$n.json') if l.startswith('{')][-1]); print('$n', round(d['value']), d['roofline'].get('avg_launch_ms'), round(d['roofline']['frac'],4))"
  done
done
for r in 1 2; do
  for v in SPAI_NONE=0 SPAI_FWD_S=6 SPAI_FWD_S=7 SPAI_FWD_GRID=192; do
    n=$(echo $v | tr '=' '_')_$r
    env $v timeout -k 10 300 python3 bench.py --steps ${SSTEPS:-5} --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4), round(d['ms_per_step'],1), 'ms/step')"
  done
done

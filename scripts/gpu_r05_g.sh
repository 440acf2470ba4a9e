# Round 5 session g: the chain policy under the streamed schedule (the leaf batch
# stays near full width): 1 / 2 / 3 chains and the one-chain-above-N-leaves knob,
# interleaved, two rounds, 6 steps each (timed region only)
set -o pipefail
cd $GRAFT_REPO_ROOT && O=gpurun_out/${TAG:-r05g} && mkdir -p $O
for r in 1 2; do
  for v in SPAI_CHAINS=2 SPAI_CHAINS=1 SPAI_CHAINS=3 SPAI_HI_LEAVES=3000; do
    n=$(echo $v | tr '=' '_')_$r
    env $v timeout -k 10 300 python3 bench.py --steps ${SSTEPS:-6} --warmup 1 --no-cpu-baseline --no-isolated --no-rules-bench --no-chess --no-lockstep-ref > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().splitlines()[-1]); print('$n', round(d['value']/1e6,3), 'M sims/s', round(d['roofline']['frac'],4), round(d['ms_per_step'],1), 'ms/step')"
  done
done

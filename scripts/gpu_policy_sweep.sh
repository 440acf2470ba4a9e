# bench under several search-chain policies (env knobs of search.hip chains_for), interleaved rounds
cd $GRAFT_REPO_ROOT && O=gpurun_out/${TAG:-policy} && mkdir -p $O
CONFIGS=${CONFIGS:-"base:SPAI_MID_LEAVES=0 m2400c2g128:SPAI_MID_LEAVES=2400,SPAI_MID_CHAINS=2,SPAI_MID_GRID=128 m2400c3g85:SPAI_MID_LEAVES=2400,SPAI_MID_CHAINS=3,SPAI_MID_GRID=85 m1600c2g128:SPAI_MID_LEAVES=1600,SPAI_MID_CHAINS=2,SPAI_MID_GRID=128 m1600c3g85:SPAI_MID_LEAVES=1600,SPAI_MID_CHAINS=3,SPAI_MID_GRID=85 m2400c4g64:SPAI_MID_LEAVES=2400,SPAI_MID_CHAINS=4,SPAI_MID_GRID=64"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in $CONFIGS; do
    name=${c%%:*}; envs=$(echo ${c#*:} | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-isolated > $O/bench_${name}_$r.json 2> $O/bench_${name}_$r.err || { tail -5 $O/bench_${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${name}_$r.json')); print('$name', $r, round(d['value']/1e6,3), 'M sims/s', round(d['games_per_sec'],1), 'games/s', 'fwd', round(d['kernel_ms']['evaluate']*1e3,2), 'us')"
  done
done 2>&1 | tee $O/policy.txt

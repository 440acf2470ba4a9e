# A/B: the C4 bench with and without the sampled per-kernel HIP events
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "" "--no-timing" "" "--no-timing"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$a', d['value'], d['ms_per_step'])"
done

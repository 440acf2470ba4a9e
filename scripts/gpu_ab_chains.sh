# GPU parity tests, then the bench with two search chains (default) and with one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ch}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${CHAINS:-2 1}; do
  SPAI_CHAINS=$c timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_c$c.json 2> gpurun_out/bench_${TAG}_c$c.err
  rc=$?; echo "chains=$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_c$c.json')); print('chains=$c', round(d['value']/1e6,2), 'M sims/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
done

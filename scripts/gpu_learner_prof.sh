set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf /tmp/lprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lprof -o lt -- \
  python3 scripts/learner_dp.py --steps 50 > gpurun_out/learner_prof.json 2> gpurun_out/learner_prof.err
rc=$?; cat gpurun_out/learner_prof.json; echo "rc=$rc"
mkdir -p gpurun_out/learner_prof
find /tmp/lprof -name '*stats*.csv' -exec cp {} gpurun_out/learner_prof/ \;
exit $rc

# learner parity tests, throughput record and rocprof kernel stats on the current build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-learner} && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "learner or pipeline" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/learner_dp.py --steps 100 > $O/learner.json 2> $O/learner.err || { tail -5 $O/learner.err; exit 1; }
cat $O/learner.json
rm -rf /tmp/prof_l && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l -o trace -- python3 scripts/learner_dp.py --steps 50 > $O/learner_prof.json 2> $O/learner_prof.err || { tail -5 $O/learner_prof.err; exit 1; }
mkdir -p $O/prof && find /tmp/prof_l -name '*stats*.csv' -exec cp {} $O/prof/ \;
head -14 $O/prof/*kernel_stats*.csv | cut -c1-150

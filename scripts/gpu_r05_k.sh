# Round 5 session k: the learner step's kernel timeline (rocprofv3 --kernel-trace):
# per-stream busy fraction and launch gaps (scripts/stream_gaps.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05k} && mkdir -p $O
rm -rf /tmp/lk
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/lk -o lk -- python3 scripts/learner_dp.py --steps 60 > $O/learner.json 2> $O/learner.err; rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/learner.err; exit $rc; }
t=$(find /tmp/lk -name '*kernel_trace.csv' | head -1); cp $t $O/learner_kernel_trace.csv && python3 scripts/stream_gaps.py $O/learner_kernel_trace.csv | tee $O/stream_gaps.txt

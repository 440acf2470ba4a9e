# learner: 1-rank benchmark, then the 2-rank RCCL data-parallel launch (RCCL refuses two ranks on one
# GPU — "invalid usage" — so on a 1-GPU box the second step only shows that refusal; it needs 2+ GPUs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/learner_dp.py --steps 50 > gpurun_out/learner_n1.json 2> gpurun_out/learner_n1.err
rc=$?; cat gpurun_out/learner_n1.json; tail -3 gpurun_out/learner_n1.err; echo "n1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
SPAI_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29631 scripts/learner_dp.py --steps 20 \
  > gpurun_out/learner_n2.json 2> gpurun_out/learner_n2.err
rc=$?; cat gpurun_out/learner_n2.json; tail -8 gpurun_out/learner_n2.err; echo "n2 rc=$rc"; exit $rc

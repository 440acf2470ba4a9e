# Rehearse the driver's N=2 launch on a 1-GPU box: two ranks (both on device 0),
# torch.distributed.run as the launcher, bench.py's host group for the barrier/reductions.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SPAI_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 1 --warmup 0 --games 1024 \
  > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err
rc=$?; cat gpurun_out/rehearse_n2.json; tail -5 gpurun_out/rehearse_n2.err; echo "rc=$rc"; exit $rc

# round-4 session: validation (scripts/gpu_r04.sh: -m gpu suite, smoke, default
# bench line), then the step anatomy (scripts/gpu_anatomy.sh) and the forward's
# phase stamps (diag build) at every group size.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${TAG:-r04} bash scripts/gpu_r04.sh || exit $?
TAG=${TAG:-r04}_anatomy bash scripts/gpu_anatomy.sh || exit $?
O=gpurun_out/${TAG:-r04}
SPAI_LIB=$PWD/build_exp/libspai_diag.so timeout -k 10 300 python scripts/net_phases.py > $O/phases.txt 2>&1; rc=$?; tail -12 $O/phases.txt; exit $rc

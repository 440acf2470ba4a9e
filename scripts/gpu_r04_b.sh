# round-4 session b: tail-mode parity + A/B (scripts/gpu_tail_ab.sh), then the step
# anatomy with a kernel timeline of five moves (scripts/gpu_anatomy.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
TAG=${TAG:-r04_b}_tail bash scripts/gpu_tail_ab.sh || exit $?
TAG=${TAG:-r04_b}_anatomy bash scripts/gpu_anatomy.sh

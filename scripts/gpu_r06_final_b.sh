# Round 6 final (second session): scripts/gpu_r06_final_a.sh (the -m gpu suite, smoke,
# kernel trace of the bench command, default line), then the PMC passes of the bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r06final_s3} bash scripts/gpu_r06_final_a.sh || exit $?
COMMIT=${COMMIT:-unknown} TAG=${TAG:-r06final_s3}_pmc bash scripts/gpu_roofline_pmc.sh

# sessions c and d back to back without their parity tests (run by the full suite first)
set -o pipefail
cd $GRAFT_REPO_ROOT
SKIP_TESTS=1 bash scripts/gpu_r05_c.sh && SKIP_TESTS=1 bash scripts/gpu_r05_d.sh

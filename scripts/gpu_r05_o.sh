# Round 5 session o: PMC counters of the C4 forward alone at 2,048 leaves (S = 8,
# 256 workgroups, one round: the streamed schedule's group size) -- MFMA busy, wave
# waits, LDS bank conflicts, instruction mix, HBM bytes (scripts/gpu_pmc.sh passes)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
FWD_N=2048 FWD_REPS=20 TAG=r05_s8 timeout -k 10 900 bash scripts/gpu_pmc.sh && python3 scripts/pmc_ratios.py gpurun_out/pmc_r05_s8 k_forward | tee gpurun_out/pmc_r05_s8/ratios.txt

# PMC passes over chess_quick.py (1024 trees x 16 sims, 20 blocks) for the chess forward
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-cpmc}
LIBARG=${SPAI_LIB:+SPAI_LIB=$SPAI_LIB}
mkdir -p gpurun_out/pmc_$TAG
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf /tmp/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o p -- python3 scripts/chess_quick.py --sims 16 > gpurun_out/pmc_$TAG/run$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  find /tmp/pmc$i -name '*counter_collection*.csv' -exec cp {} gpurun_out/pmc_$TAG/pass$i.csv \;
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, collections, glob, os
tag = os.environ.get("TAG", "cpmc")
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/pass*.csv")):
    for r in csv.DictReader(open(f)):
        if "k_chess_forward" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]]["v"] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
for c in sorted(acc): print(c, acc[c]["v"] / max(1, len(n[c])), "per dispatch over", len(n[c]))
PY

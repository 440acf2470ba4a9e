# Round 5 session q: TA (vector-memory address unit) busy fraction of both forwards,
# the C4 forward alone at 2,048 leaves (S = 8) and the chess forward (1,024 trees):
# the per-CU weight-fragment stream is the claimed limiter of the C4 k-loop
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r05q} && mkdir -p $O
rm -rf /tmp/ta1 /tmp/ta2
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d /tmp/ta1 -o p -- python3 scripts/net_forward_bench.py 2048 20 > $O/c4.log 2>&1; rc=$?; echo "c4 pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d /tmp/ta2 -o p -- python3 scripts/chess_quick.py --sims 16 > $O/chess.log 2>&1; rc=$?; echo "chess pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
find /tmp/ta1 -name '*counter_collection*.csv' -exec cp {} $O/c4_ta.csv \;
find /tmp/ta2 -name '*counter_collection*.csv' -exec cp {} $O/chess_ta.csv \;
python3 - <<'PY'
import csv, collections, os
O = os.environ.get("O", "gpurun_out/r05q")
for f, k in (("c4_ta.csv", "k_forward"), ("chess_ta.csv", "k_chess_forward")):
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join("gpurun_out/r05q", f))):
        if k in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
    per = {c: acc[c] / max(1, len(n[c])) for c in acc}
    print(k, per, "TA busy avr / GRBM active per dispatch: %.3f" % (per.get("TA_BUSY_avr", 0) / max(1, per.get("GRBM_GUI_ACTIVE", 1))))
PY

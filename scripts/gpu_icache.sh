# instruction-cache counters of the forward alone (one pass, killed if the counter set is refused)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/icache && mkdir -p $O
timeout -k 10 60 python scripts/fwd_once.py 1006 300 || exit 1
for set in "SQC_ICACHE_REQ SQC_ICACHE_MISSES" "SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA"; do
  tag=$(echo $set | cut -d' ' -f1)
  rm -rf /tmp/ic_$tag
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d /tmp/ic_$tag -o p -- python3 scripts/fwd_once.py 1006 300 > $O/run_$tag.log 2>&1
  echo "pass $tag rc=$?"; tail -3 $O/run_$tag.log
  find /tmp/ic_$tag -name '*counter_collection*.csv' -exec cp {} $O/pass_$tag.csv \;
done
for f in $O/pass_*.csv; do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_forward" not in r.get("Kernel_Name", ""): continue
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in tot: print(k, tot[k], "dispatch-rows", n[k])
PY
done

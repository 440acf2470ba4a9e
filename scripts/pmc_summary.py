"""Summarise rocprofv3 --pmc CSVs (one per pass) into mean counter values and HBM
bytes per launch for each kernel (and the L2 hit rate when TCC_HIT/TCC_MISS are there): bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (counters in KiB;
FETCH_SIZE doubled: on gfx950 it reads half the bytes of wide coalesced reads,
MI355X_MICROARCH.md section HBM)."""
import collections
import csv
import json
import re
import sys

out_path, files = sys.argv[1], sys.argv[2:]
per = collections.defaultdict(lambda: collections.defaultdict(float))   # kernel -> counter -> sum
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in files:
    for r in csv.DictReader(open(f)):
        m = re.search(r"\b(k_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"].split("(")[0].strip()
        c = r["Counter_Name"]
        per[k][c] += float(r["Counter_Value"])
        disp[k][c].add(r["Dispatch_Id"])
res = {}
for k, cs in per.items():
    n = {c: len(disp[k][c]) for c in cs}
    fetch = cs.get("FETCH_SIZE", 0.0) / max(1, n.get("FETCH_SIZE", 1))
    write = cs.get("WRITE_SIZE", 0.0) / max(1, n.get("WRITE_SIZE", 1))
    res[k] = {"launches": max(n.values()), "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
              "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
              "per_launch": {c: cs[c] / max(1, n[c]) for c in cs}}
    if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
        res[k]["l2_hit_rate"] = cs["TCC_HIT_sum"] / max(1.0, cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
json.dump(res, open(out_path, "w"), indent=1)
for k, v in sorted(res.items(), key=lambda kv: -kv[1]["launches"]):
    print(k, v)

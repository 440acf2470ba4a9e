"""Per-stream kernel gaps from a rocprofv3 kernel_trace.csv: for each queue/stream,
the idle time between consecutive kernels, grouped by (previous -> next) kernel."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
print("columns:", list(rows[0].keys())[:20])
by = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    m = re.search(r"\b(k_\w+)", name)
    k = m.group(1) if m else name.split("(")[0][:30]
    by[r.get(key, "0")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
t_all0 = min(s for v in by.values() for s, _, _ in v)
t_all1 = max(e for v in by.values() for _, e, _ in v)
print("wall (first start -> last end): %.1f ms" % ((t_all1 - t_all0) / 1e6))
for q, ks in sorted(by.items()):
    ks.sort()
    gaps = collections.defaultdict(list)
    busy = collections.defaultdict(float)
    for (s0, e0, k0), (s1, e1, k1) in zip(ks, ks[1:]):
        gaps[(k0, k1)].append(max(0, s1 - e0) / 1e3)
    for s, e, k in ks:
        busy[k] += (e - s) / 1e3
    print("stream %s: %d kernels, busy %.1f ms" % (q, len(ks), sum(busy.values()) / 1e3))
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:6]:
        print("   busy %-16s %.1f ms" % (k, v / 1e3))
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:6]:
        v.sort()
        print("   gap %-14s -> %-14s n=%6d median %.2f us mean %.2f us total %.1f ms" %
              (a, b, len(v), v[len(v) // 2], sum(v) / len(v), sum(v) / 1e3))

"""Busy fraction and inter-kernel gaps per stream (queue) of a rocprofv3
--kernel-trace CSV, over the middle of the trace (skips the first and last 10 %).
usage: stream_gaps.py kernel_trace.csv"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key],
                 (re.search(r"\b(k_\w+)", r["Kernel_Name"]) or re.search(r"(\w+)", r["Kernel_Name"])).group(1))
                for r in rows)
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    lo, hi = t0 + (t1 - t0) // 10, t1 - (t1 - t0) // 10
    ks = [k for k in ks if lo <= k[0] and k[1] <= hi]
    span = hi - lo
    by = collections.defaultdict(list)
    for k in ks:
        by[k[2]].append(k)
    # union of all kernels (any stream busy)
    busy, end = 0, lo
    for s, e, _, _ in ks:
        if e > end:
            busy += e - max(s, end)
            end = e
    print("window %.1f us, kernels %d, any-stream busy %.3f" % (span / 1e3, len(ks), busy / span))
    for q, L in sorted(by.items(), key=lambda x: -len(x[1])):
        b = sum(e - s for s, e, _, _ in L)
        gaps = [L[i + 1][0] - L[i][1] for i in range(len(L) - 1)]
        gaps = sorted(g for g in gaps if g >= 0)
        med = gaps[len(gaps) // 2] if gaps else 0
        names = collections.Counter(n for _, _, _, n in L).most_common(3)
        print("stream %s: %d kernels, busy %.3f, median gap %.2f us, gaps < 20 us total %.1f us; %s"
              % (q, len(L), b / span, med / 1e3, sum(g for g in gaps if g < 20000) / 1e3, names))


if __name__ == "__main__":
    main()

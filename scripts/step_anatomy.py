"""Anatomy of one self-play step from a rocprofv3 --kernel-trace CSV: the step is
cut into moves at each k_advance (self-play's move step; k_root_stats in builds
before it: one per search call), and per move the
script reports the wall time, the forward (k_forward) launches with their mean
duration, the tree-kernel launches (k_select / k_expand_select / k_expand) with
theirs, and how the wall splits into time with 0, 1 or 2 forwards running.
usage: step_anatomy.py kernel_trace.csv [out.json] [moves_to_dump out.csv]
(moves_to_dump: comma-separated move numbers; their first 120 kernels are written
with stream, start and end in microseconds from the move's first kernel)"""
import collections
import csv
import json
import re
import sys


def kname(s):
    m = re.search(r"\b(k_\w+)", s)
    return m.group(1) if m else s.split("(")[0][:30]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skey = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"]),
                 r.get(skey, "0") if skey else "0") for r in rows)
    moves, cur = [], []
    for k in ks:
        cur.append(k)
        if k[2] in ("k_advance", "k_root_stats"):
            moves.append(cur)
            cur = []
    out = []
    for i, mv in enumerate(moves):
        t0, t1 = mv[0][0], mv[-1][1]
        by = collections.defaultdict(list)
        for s, e, n, _ in mv:
            by[n].append((e - s) / 1e3)
        # time with 0/1/2+ forwards running (sweep over forward intervals)
        ev = []
        for s, e, n, _ in mv:
            if n == "k_forward":
                ev += [(s, 1), (e, -1)]
        ev.sort()
        lvl, last, occ = 0, t0, collections.Counter()
        for t, d in ev:
            occ[min(lvl, 2)] += t - last
            lvl += d
            last = t
        occ[0] += t1 - last
        wall = (t1 - t0) / 1e3
        rec = {"move": i, "wall_us": wall,
               "fwd_n": len(by["k_forward"]), "fwd_mean_us": sum(by["k_forward"]) / max(1, len(by["k_forward"])),
               "tree_n": sum(len(by[k]) for k in ("k_select", "k_expand_select", "k_expand")),
               "tree_mean_us": sum(sum(by[k]) for k in ("k_select", "k_expand_select", "k_expand")) /
                               max(1, sum(len(by[k]) for k in ("k_select", "k_expand_select", "k_expand"))),
               "no_fwd_frac": occ[0] / 1e3 / wall if wall else 0, "one_fwd_frac": occ[1] / 1e3 / wall if wall else 0,
               "two_fwd_frac": occ[2] / 1e3 / wall if wall else 0}
        out.append(rec)
    tot = sum(r["wall_us"] for r in out)
    print("moves %d, wall %.1f ms" % (len(out), tot / 1e3))
    print("move   wall_ms  fwd_n fwd_us  tree_n tree_us  no_fwd one_fwd two_fwd")
    for r in out:
        print("%4d %8.2f %6d %6.1f %7d %7.1f %7.2f %7.2f %7.2f" % (
            r["move"], r["wall_us"] / 1e3, r["fwd_n"], r["fwd_mean_us"], r["tree_n"], r["tree_mean_us"],
            r["no_fwd_frac"], r["one_fwd_frac"], r["two_fwd_frac"]))
    agg = collections.Counter()
    for r in out:
        for k in ("no_fwd_frac", "one_fwd_frac", "two_fwd_frac"):
            agg[k] += r[k] * r["wall_us"]
    print("whole step: no forward %.3f, one %.3f, two %.3f of the wall" %
          tuple(agg[k] / tot for k in ("no_fwd_frac", "one_fwd_frac", "two_fwd_frac")))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=0)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write("move,kernel,stream,start_us,end_us\n")
            for m in (int(v) for v in sys.argv[3].split(",")):
                if m < len(moves):
                    t0 = moves[m][0][0]
                    for s, e, n, q in moves[m][:120]:
                        f.write("%d,%s,%s,%.2f,%.2f\n" % (m, n, q, (s - t0) / 1e3, (e - t0) / 1e3))


if __name__ == "__main__":
    main()

"""Combine the rocprofv3 --pmc passes of one bench command (scripts/gpu_roofline_pmc.sh)
into profiles/<round>/final/forward_pmc.json, the file bench.py's `roofline.executed`
and `roofline.traffic` read:
  * per kernel: launches and mean counters per launch (pmc_summary.py's format);
  * derived, for k_forward<false>: executed MFMA FLOPs per launch (SQ_INSTS_MFMA x
    16*16*32*2, every MFMA of the kernel is v_mfma_f32_16x16x32_bf16) over the
    algorithmic FLOPs per launch (the pass's own bench line: work.evals x flop_per_eval
    / launches); mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x
    1024 SIMDs); the wave-cycle split (parked on s_waitcnt/barriers, issue-stalled,
    issuing) from SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES.
usage: roofline_pmc.py out.json bench_line.json commit pass.csv [pass.csv ...]"""
import collections
import csv
import json
import re
import sys

out_path, bench_path, commit, files = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
per = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in files:
    for r in csv.DictReader(open(f)):
        m = re.search(r"\b(k_\w+(?:<[^>]*>)?)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"].split("(")[0].strip()
        c = r["Counter_Name"].replace("_sum", "")
        per[k][c] += float(r["Counter_Value"])
        disp[k][c].add(r["Dispatch_Id"])
res = {"commit": commit}
for k, cs in per.items():
    n = {c: len(disp[k][c]) for c in cs}
    fetch = cs.get("FETCH_SIZE", 0.0) / max(1, n.get("FETCH_SIZE", 1))
    write = cs.get("WRITE_SIZE", 0.0) / max(1, n.get("WRITE_SIZE", 1))
    res[k] = {"launches": max(n.values()), "per_launch": {c: cs[c] / max(1, n[c]) for c in cs}}
    if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
        res[k].update({"FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "hbm_bytes_per_launch": (2 * fetch + write) * 1024})
line = json.loads([l for l in open(bench_path).read().splitlines() if l.startswith("{")][-1])
kf = res.get("k_forward<false>")
if kf and "SQ_INSTS_MFMA" in kf["per_launch"]:
    pl = kf["per_launch"]
    L = len(disp["k_forward<false>"]["SQ_INSTS_MFMA"])
    fpe = line["roofline"]["flop_per_eval"]
    alg = line["work"]["evals"] * fpe / L
    exe = pl["SQ_INSTS_MFMA"] * 16 * 16 * 32 * 2
    d = {"launches": L, "leaves_per_launch": line["work"]["evals"] / L, "mfma_insts_per_launch": pl["SQ_INSTS_MFMA"],
         "executed_flop_per_launch": exe, "algorithmic_flop_per_launch": alg, "executed_over_algorithmic": exe / alg}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in pl and "GRBM_GUI_ACTIVE" in pl:
        d["mfma_busy"] = pl["SQ_VALU_MFMA_BUSY_CYCLES"] / (pl["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "SQ_WAVE_CYCLES" in pl:
        w = pl["SQ_WAVE_CYCLES"]
        d["wave_cycles"] = {"parked_waitcnt_barrier": pl.get("SQ_WAIT_ANY", 0) / w,
                            "issue_stalled": pl.get("SQ_WAIT_INST_ANY", 0) / w,
                            "issuing": pl.get("SQ_ACTIVE_INST_ANY", 0) / w}
    if "SQ_INSTS_VALU" in pl:
        d["valu_per_mfma"] = pl["SQ_INSTS_VALU"] / pl["SQ_INSTS_MFMA"]
    if "SQ_INSTS_LDS" in pl:
        d["lds_per_mfma"] = pl["SQ_INSTS_LDS"] / pl["SQ_INSTS_MFMA"]
    d["bench_line_of_the_pass"] = {"value": line["value"], "work": line["work"], "config": line["config"]}
    res["derived"] = d
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res.get("derived", {}), indent=1))
for k in ("k_forward<false>", "k_expand_select<false>", "k_select<false>"):
    if k in res:
        print(k, res[k]["launches"], {c: round(v, 1) for c, v in res[k]["per_launch"].items()})

"""Per-kernel ratios from the gpu_pmc.sh passes (SQ counters summed over dispatches
of the named kernel; SQ_*_CYCLES wave counters are in quad-cycles, MFMA busy in cycles)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_forward"
tot = collections.defaultdict(float)
for f in sorted(glob.glob(d + "/pass*.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}")
wc = tot.get("SQ_WAVE_CYCLES", 0)
if wc:
    print("wait_any/wave_cycles      %.3f" % (tot["SQ_WAIT_ANY"] / wc))
    print("wait_inst_any/wave_cycles %.3f" % (tot["SQ_WAIT_INST_ANY"] / wc))
    print("active_inst/wave_cycles   %.3f" % (tot["SQ_ACTIVE_INST_ANY"] / wc))
if tot.get("SQ_BUSY_CYCLES") and tot.get("SQ_VALU_MFMA_BUSY_CYCLES"):
    print("mfma_busy/(busy*4 simd)   %.3f" % (tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["SQ_BUSY_CYCLES"] * 4)))
if tot.get("SQ_LDS_IDX_ACTIVE"):
    print("lds_conflict/lds_active   %.3f" % (tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_LDS_IDX_ACTIVE"]))
if tot.get("SQ_INSTS_MFMA"):
    print("valu/mfma insts           %.2f" % (tot["SQ_INSTS_VALU"] / tot["SQ_INSTS_MFMA"]))
    print("lds/mfma insts            %.2f" % (tot["SQ_INSTS_LDS"] / tot["SQ_INSTS_MFMA"]))

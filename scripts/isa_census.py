"""Instruction census of the C4 forward's trunk block loop from a device .s file.

usage: python scripts/isa_census.py <file.s> [kernel-substring]
Finds every backward branch in the kernel; the trunk block loop of a wave is the
loop whose body holds the most MFMAs (two trunk convs).  Prints instruction
counts by class for each such loop, per wave and per MFMA.
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr_read"):
        return "valu.accvgpr_read"
    if op.startswith("v_accvgpr_write"):
        return "valu.accvgpr_write"
    if op.startswith("v_accvgpr_mov"):
        return "valu.accvgpr_mov"
    if op.startswith("v_cvt_pk_bf16"):
        return "valu.cvt_pk_bf16"
    if op.startswith("v_pk_max_i16"):
        return "valu.pk_max_i16"
    if op.startswith(("v_add_co", "v_addc_co", "v_lshl_add_u64", "v_add_u32", "v_add_nc", "v_mad_u64")):
        return "valu.addr_add"
    if op.startswith(("v_and_b32", "v_bfe_u32", "v_lshrrev_b32", "v_lshlrev_b32", "v_xor_b32", "v_or_b32",
                      "v_and_or", "v_xad", "v_lshl_or", "v_xor3", "v_or3", "v_perm", "v_alignbit", "v_bfi")):
        return "valu.bitops"
    if op.startswith("v_mov"):
        return "valu.mov"
    if op.startswith("v_"):
        return "valu.other"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds.read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "lds.write"
    if op.startswith("ds_"):
        return "lds.other"
    if op.startswith(("global_load", "buffer_load")):
        return "vmem.load"
    if op.startswith(("global_store", "buffer_store")):
        return "vmem.store"
    if op == "s_waitcnt":
        return "s_waitcnt"
    if op.startswith("s_barrier"):
        return "s_barrier"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "salu.branch"
    if op.startswith("s_"):
        return "salu.other"
    return "other:" + op


def main():
    path = sys.argv[1]
    ksub = sys.argv[2] if len(sys.argv) > 2 else "k_forwardILb0E"
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + ksub + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    insts = []   # (line index, op, text)
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        insts.append((i, op, s))
    loops = []
    for j, (i, op, s) in enumerate(insts):
        if op.startswith(("s_cbranch", "s_branch")):
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= j:
                a, b = labels[tgt], j
                nm = sum(1 for k in range(a, b + 1) if insts[k][1].startswith("v_mfma"))
                loops.append((a, b, nm))
    loops.sort(key=lambda x: -x[2])
    print(f"kernel {ksub}: {len(insts)} instructions, {sum(1 for x in insts if x[1].startswith('v_mfma'))} MFMAs, {len(loops)} loops")
    top = [l for l in loops if l[2] >= 0.8 * loops[0][2]] if loops else []
    for a, b, nm in sorted(top):
        c = Counter(classify(insts[k][1]) for k in range(a, b + 1))
        tot = sum(c.values())
        print(f"\nloop insts [{a}, {b}]: {tot} instructions, {nm} MFMA")
        groups = OrderedDict()
        for k, v in sorted(c.items(), key=lambda kv: (kv[0].split('.')[0], -kv[1])):
            print(f"  {k:22s} {v:6d}  {v / max(nm, 1):6.3f} per MFMA")
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        print(f"  {'VALU total':22s} {valu:6d}  {valu / max(nm, 1):6.3f} per MFMA")


if __name__ == "__main__":
    main()

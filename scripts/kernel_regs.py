"""Register footprint of the device kernels in a built library (or object).

    python scripts/kernel_regs.py build_exp/libspai_x.so [kernel-regex]

vgpr_count includes the AGPRs: one wave of a kernel leaves 512 - vgpr_count
registers per SIMD lane to co-resident waves (e.g. the other search chain's
tree kernels running beside the forward)."""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def kernels(path):
    """{kernel name: descriptor fields} of every gfx950 kernel in a built library"""
    out = {}
    with tempfile.TemporaryDirectory() as t:
        fb = os.path.join(t, "fb.bin")
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", path, os.path.join(t, "s")], check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for i, s in enumerate(starts):
            part = os.path.join(t, f"b{i}")
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = part + ".co"
            r = subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode:
                continue
            notes = subprocess.run([f"{B}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            for ent in notes.split("  - .agpr_count:")[1:]:
                f = dict(re.findall(r"\.(\w+):\s+(\S+)", ent))
                f["agpr_count"] = ent.split()[0]
                out[f.get("name", "?")] = f
    return out


def main():
    path, rx = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    for name, f in kernels(path).items():
        if rx.search(name):
            print(f"{name[:70]:70s} vgpr {f.get('vgpr_count')} (agpr {f['agpr_count']}) sgpr {f.get('sgpr_count')} "
                  f"vspill {f.get('vgpr_spill_count')} scratch {f.get('private_segment_fixed_size')} "
                  f"lds {f.get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()

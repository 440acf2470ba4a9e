"""Print the fused forward's per-phase cycle breakdown (diagnostic stamps)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
names = ["start", "stem"] + ["res%d" % i for i in range(12)] + ["head_conv", "linear", "end"]
for n in (2048, 4096):
    c = net.phase_cycles(n)
    d = np.diff(c)
    print(f"batch {n}: total {c[16]:.0f} cycles/wave = {c[16] / 2.1e3:.1f} us @2.1GHz")
    print("  " + "  ".join(f"{names[k + 1]}={d[k]:.0f}" for k in range(16)))
# per-group latency for every group size S (one group per workgroup, 256 workgroups)
for S in range(1, 9):
    os.environ["SPAI_PHASE_S"] = str(S)
    c = net.phase_cycles(256 * S)
    d = np.diff(c[:17])
    print(f"S={S}: {c[16]:.0f} cycles/wave = {c[16] / 2.1e3:.1f} us @2.1GHz  stem {d[0]:.0f} res0 {d[1]:.0f} "
          f"res1 {d[2]:.0f} res2 {d[3]:.0f} head {d[13]:.0f} linear {d[14]:.0f} end {d[15]:.0f}; "
          f"block0 conv1: k-loop {c[17] - c[1]:.0f}, epilogue {c[18] - c[17]:.0f}, barrier {c[19] - c[18]:.0f}; "
          f"wall: entry->group {c[21] / 1e3:.2f} us ({c[20]:.0f} cyc), group {c[22] / 1e3:.2f} us, "
          f"launch span {c[23] / 1e3:.2f} us, clock {c[16] / max(c[22], 1):.2f} GHz")
    if os.environ.get("SPAI_PRINT_ENTRY"):   # diagnostic build with -DSPAI_DIAG_ENTRY
        print(f"    entry (shader cycles): constants in LDS {c[20] + c[17]:.0f}, geometry + bitboards loaded "
              f"{c[20] + c[18]:.0f}, planes stored {c[20] + c[19]:.0f}, group start {c[20]:.0f}")
os.environ.pop("SPAI_PHASE_S")
net.close()
e.close()

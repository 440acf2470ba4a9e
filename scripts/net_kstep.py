"""Per-k-step timeline of one steady-state trunk conv (block 1, conv 1) of the C4
forward, from the k-step diagnostic build (-DSPAI_DIAG -DSPAI_DIAG_KSTEP):
cycles per k-step per wave (mean over workgroups), the conv's start -> barrier
passed, against the MFMA issue of that k-step.  usage: SPAI_LIB=... python scripts/net_kstep.py [S ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
for S in [int(a) for a in sys.argv[1:]] or [8]:
    os.environ["SPAI_PHASE_S"] = str(S)
    c = net.phase_cycles(256 * S)
    c = net.phase_cycles(256 * S)
    start = c[44]
    ks = [c[24 + k] for k in range(18)]
    prev = start
    parts = []
    for k in range(18):
        if ks[k] == 0:
            parts.append("  -")
            continue
        parts.append(f"{ks[k] - prev:5.0f}")
        prev = ks[k]
    print(f"S={S}: group {c[16]:.0f} cyc; conv start {start:.0f}; k-steps: " + " ".join(parts))
    print(f"   conv total {c[42] - start:.0f}, to barrier {c[43] - c[42]:.0f}; res2 phase {c[4] - c[3]:.0f}")
net.close()
e.close()

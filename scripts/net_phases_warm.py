"""Phase stamps of the fused forward with a cold vs warm instruction cache: one
group per workgroup (the stamps see the launch's first pass over the code) vs
four groups per workgroup (the stamps keep the last group, after three passes)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
for S in (1, 4, 8):
    os.environ["SPAI_PHASE_S"] = str(S)
    for groups in (1, 4):
        os.environ["SPAI_PHASE_GRID"] = "256"
        c = net.phase_cycles(256 * S * groups)
        d = np.diff(c[:17])
        print(f"S={S} groups/WG={groups}: {c[16]:.0f} cycles  stem {d[0]:.0f} res0 {d[1]:.0f} res1 {d[2]:.0f} "
              f"res2 {d[3]:.0f} res11 {d[12]:.0f} head {d[13]:.0f} linear {d[14]:.0f} end {d[15]:.0f}")
net.close()
e.close()

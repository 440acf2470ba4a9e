"""Head-phase breakdown of the fused C4 forward (diagnostic build with
-DSPAI_DIAG -DSPAI_DIAG_HEAD: stamp 19 = before the head, 17 = head k-loop done,
18 = head features written, 14 = after the barrier, 15 = linear done)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
for S in range(1, 9):
    os.environ["SPAI_PHASE_S"] = str(S)
    c = net.phase_cycles(256 * S)
    print(f"S={S}: total {c[16]:.0f}  trunk-end {c[13]:.0f}  pre-head {c[19] - c[13]:.0f}  head k-loop {c[17] - c[19]:.0f}  "
          f"H write {c[18] - c[17]:.0f}  barrier {c[14] - c[18]:.0f}  linear {c[15] - c[14]:.0f}  end {c[16] - c[15]:.0f}")
net.close()
e.close()

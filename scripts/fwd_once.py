"""One forward-alone timing run in this process (for rocprofv3 --pmc passes):
spai_net_bench at N leaves, 6x64 net, random reachable positions."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "self-play-ai_amd"))
import spai  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1006
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, 64, seed=0))
net.bench(n, iters=50)
ms = net.bench(n, iters=iters)
print(f"{n} leaves: {ms * 1e3:.2f} us per launch")
net.close()
e.close()

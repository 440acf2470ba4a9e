"""Dump the C4 bf16 net's priors and values (Model::predict through the search's
forward path, spai_predict) on fixed random positions at batch sizes that exercise
every group size, so two builds can be compared bit for bit:
  SPAI_LIB=a.so python scripts/net_dump.py a.npz; SPAI_LIB=b.so python scripts/net_dump.py b.npz
  python scripts/net_dump.py --compare a.npz b.npz"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "self-play-ai_amd"))
import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))]
    print("bit-identical" if not bad else "DIFFER: %s" % bad)
    sys.exit(1 if bad else 0)
import spai

e = spai.Engine(num_searches=1, max_trees=1)
net = spai.Net(e, 6, spai.init_params(6, seed=0))
rng = np.random.default_rng(5)
e.games_resize(4096)
for _ in range(14):   # random reachable positions
    lm = e.legal_mask(4096)
    r = rng.random((4096, 7)) * ((lm[:, None] >> np.arange(7)) & 1)
    e.apply(np.argmax(r, 1).astype(np.int32), check=False)
st = e.games_read(4096)
st = st[st["status"] == 0]
out = {}
for n in (1, 7, 100, 300, 600, 1000, 1300, 1600, 2048, len(st)):
    pr, v = net.predict(st[:n])
    out["p%d" % n], out["v%d" % n] = np.asarray(pr, np.float32), np.asarray(v, np.float32)
np.savez(sys.argv[1], **out)
print("dumped", len(out) // 2, "batches of up to", len(st), "positions")

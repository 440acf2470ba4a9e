"""Numerics of experimental forward builds against the default library: every
build (SPAI_LIB per subprocess) predicts the same reachable positions; prints
the largest prior / value differences to the first build (the default).
usage: python scripts/variant_check.py a.so,b.so [--counts 1000]"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(counts, out):
    sys.path.insert(0, os.path.join(REPO, "self-play-ai_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import spai
    from test_gpu_parity import _reachable_positions
    states = _reachable_positions(spai, 3000, 14, seed=9)
    e = spai.Engine(num_searches=1, max_trees=1)
    net = spai.Net(e, 6, spai.init_params(6, 64, seed=2))
    res = {}
    for n in counts:
        p, v = net.predict(states[:n])
        res["p%d" % n], res["v%d" % n] = p, v
    np.savez(out, **res)
    net.close()
    e.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs")
    ap.add_argument("--counts", default="1000")
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    counts = [int(c) for c in a.counts.split(",")]
    if a.child:
        child(counts, a.child)
        return
    outs = []
    for i, lib in enumerate(a.libs.split(",")):
        o = "/tmp/variant_check_%d.npz" % i
        r = subprocess.run([sys.executable, __file__, a.libs, "--counts", a.counts, "--child", o],
                           env=dict(os.environ, SPAI_LIB=lib), capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(lib, "FAILED", r.stderr[-1500:])
            sys.exit(1)
        outs.append(np.load(o))
    for lib, d in zip(a.libs.split(",")[1:], outs[1:]):
        for n in counts:
            dp = np.abs(d["p%d" % n] - outs[0]["p%d" % n]).max()
            dv = np.abs(d["v%d" % n] - outs[0]["v%d" % n]).max()
            print(json.dumps({"lib": os.path.basename(lib), "n": n, "max_dprior": float(dp), "max_dvalue": float(dv),
                              "finite": bool(np.isfinite(d["p%d" % n]).all())}))


if __name__ == "__main__":
    main()

"""Forward-alone timing sweep (spai_net_bench) over leaf counts for one or more
library builds: SPAI_LIB=<path> per run, or --libs a.so,b.so (one subprocess each).
Prints one line per (lib, count): ms per launch, TFLOP/s, fraction of 2.5 PF."""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FPE = 39016572


def one(counts, iters, blocks, conc=1):
    sys.path.insert(0, os.path.join(REPO, "self-play-ai_amd"))
    import spai
    e = spai.Engine(num_searches=1, max_trees=1)
    net = spai.Net(e, blocks, spai.init_params(blocks, 64, seed=0))
    net.bench(max(counts), iters=max(1, int(0.2e6 / 120 / 1)))   # ~0.2 s of launches: settle the clock first
    out = {}
    for n in counts:
        ms = net.bench(n, iters=iters, conc=conc)
        out[n] = ms
    net.close()
    e.close()
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--counts", default="1,64,256,512,768,1024,1280,1536,1792,2048,3072,4096")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--conc", type=int, default=1, help="group size for this many concurrent chains (spai_net_bench_conc)")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    counts = [int(c) for c in a.counts.split(",")]
    if a.child:
        one(counts, a.iters, a.blocks, a.conc)
        return
    libs = a.libs.split(",") if a.libs else [os.environ.get("SPAI_LIB", os.path.join(REPO, "self-play-ai_amd", "libspai.so"))]
    for lib in libs:
        env = dict(os.environ, SPAI_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "--child", "--counts", a.counts, "--iters", str(a.iters),
                            "--blocks", str(a.blocks), "--conc", str(a.conc)], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(lib, "FAILED", r.stderr[-800:])
            sys.exit(1)
        res = json.loads(r.stdout.strip().splitlines()[-1])
        for n, ms in res.items():
            tf = FPE * int(n) / (ms * 1e-3) / 1e12
            print("%-28s n %5s  %8.2f us  %7.1f TF/s  frac %.3f" % (os.path.basename(lib), n, ms * 1e3, tf, tf / 2500))


if __name__ == "__main__":
    main()

"""Assemble profiles/<round>/chess_full/record.json from the two full-game runs of
scripts/gpu_r06_c.sh (scripts/chess_bench.py --full --batches 2 [--stream]): BASELINE
config 4 (1,024 games x 400 sims/move, 20x256 bf16) played to completion, lockstep and
streamed, with the per-move traces beside it.  bench.py quotes the record in its
`chess.record` field.  usage: chess_record.py DIR COMMIT"""
import csv
import json
import os
import sys

d, commit = sys.argv[1], sys.argv[2]
rec = {"workload": "BASELINE config 4: chess self-play, 1,024 parallel games x 400 sims/move, 20x256 ResNet bf16, "
                   "2 x 1,024 games from the start position played to completion",
       "commit": commit}
for mode in ("lockstep", "stream"):
    p = os.path.join(d, "full_%s.json" % mode)
    if not os.path.exists(p):
        continue
    r = json.loads([l for l in open(p).read().splitlines() if l.startswith("{")][-1])
    row = {"games": r["games_finished"], "seconds": r["seconds"], "games_per_sec": r["games_per_sec"],
           "sims_per_sec": r["value"], "moves": r["moves"], "forward_frac": r["roofline"]["frac"],
           "forward_avg_leaves": r["roofline"]["avg_leaves_per_launch"],
           "schedule": ("two lockstep batches of 1,024 games (every game of a batch starts together; the batch "
                        "is searched until its last game ends)" if mode == "lockstep" else
                        "2,048 games through 1,024 tree slots (spai_chess_selfplay_stream)")}
    t = os.path.join(d, "moves_%s.csv" % mode)
    if os.path.exists(t):
        rows = [x for x in csv.reader(open(t)) if x and x[0].strip().lstrip("-").isdigit()]
        row["trace"] = {"file": os.path.basename(t), "moves_logged": len(rows)}
    rec[mode] = row
json.dump(rec, open(os.path.join(d, "record.json"), "w"), indent=1)
print(json.dumps(rec, indent=1))

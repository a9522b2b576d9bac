"""Kernel + memory-copy events of a rocprofv3 run (kernel_trace.csv, memory_copy_trace.csv) in time
order, the last N of them, with their queue/stream: a step's timeline.
usage: python3 scripts/trace_merge.py <dir> [N] [name-regex]"""
import csv
import glob
import re
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 80
pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if pat and not pat.search(name):
            continue
        name = name[name.find("k_"):name.find("(")] if "k_" in name else name[:40]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", r.get("Stream_Id", "?"))))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?"), r.get("Queue_Id", r.get("Stream_Id", "?"))))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0] if ev else 0
for s, e, name, qid in ev:
    print(f"{(s - t0) / 1e6:10.3f} ms {(e - s) / 1e3:9.1f} us  q{qid:>3}  {name}")

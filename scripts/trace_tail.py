"""Print the last N kernel launches of a rocprofv3 kernel_trace.csv (start offset, duration, name).
usage: python3 scripts/trace_tail.py <kernel_trace.csv> [N] [name-regex]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
if pat:
    rows = [r for r in rows if pat.search(r["Kernel_Name"])]
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    name = name[name.find("k_"):name.find("(")] if "k_" in name else name[:40]
    print(f"{(s - t0) / 1e6:10.3f} ms {(e - s) / 1e3:10.1f} us  {name}  grid={r['Grid_Size_X']}")

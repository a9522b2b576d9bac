"""HBM traffic of one IVF search's list scans (k_screen_mfma_mapped + k_ivf_scan_dyn first pass) from
two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), per MI355X_MICROARCH.md: bytes = 2 * 1024 *
FETCH_SIZE (gfx950 reports half of wide streaming reads) + 1024 * WRITE_SIZE.
usage: python3 scripts/ivf_traffic.py <fetch_dir> <write_dir> <out.json> <skew> <n_rows> [max_dyn_ms]
Dyn dispatches longer than max_dyn_ms (the bench's GEMV-only run beside) are excluded."""
import collections
import csv
import glob
import json
import sys


def load(d, counter):
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    dur = {}
    if kt:
        for r in csv.DictReader(open(kt[0])):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    per = collections.defaultdict(lambda: [None, 0.0, 0.0])
    for r in csv.DictReader(open(cc)):
        if r["Counter_Name"] != counter:
            continue
        n = r["Kernel_Name"]
        if "mapped" in n:
            kind = "mapped"
        elif "ivf_scan_dyn" in n:
            kind = "dyn"
        else:
            continue
        p = per[r["Dispatch_Id"]]
        p[0] = kind
        p[1] += float(r["Counter_Value"])
        p[2] = dur.get(r["Dispatch_Id"], 0.0)
    return per


fetch, write, out, skew, nrows = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4]), int(sys.argv[5])
max_dyn = float(sys.argv[6]) if len(sys.argv) > 6 else 50.0
res = {}
for name, d, counter, scale in (("read", fetch, "FETCH_SIZE", 2048.0), ("write", write, "WRITE_SIZE", 1024.0)):
    per = load(d, counter)
    acc = collections.defaultdict(list)
    for kind, v, ms in per.values():
        if kind == "dyn" and ms > max_dyn:
            continue
        acc[kind].append(v * scale)
    res[name] = {k: sum(v) / len(v) for k, v in acc.items()}
    res[name + "_n"] = {k: len(v) for k, v in acc.items()}
tot = sum(res["read"].values()) + sum(res["write"].values())
json.dump({"workload": "cfg5", "n_local": nrows, "skew": skew,
           "kernel": "k_screen_mfma_mapped + k_ivf_scan_dyn (the list scans of one search)",
           "hbm_bytes_per_launch": tot, "read_bytes": res["read"], "write_bytes": res["write"],
           "dispatches": {"read": res["read_n"], "write": res["write_n"]},
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (scripts/ivf_traffic.py)"},
          open(out, "w"), indent=1)
print(open(out).read())

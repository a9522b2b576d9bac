#!/usr/bin/env python3
"""Summarise one scripts/gpu_prof.sh run into profiles/<tag>_*.{csv,json,md}.

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE is in KiB and on gfx950
reports half the bytes of wide coalesced streaming reads, so traffic = 2 * 1024 * FETCH_SIZE;
WRITE_SIZE (KiB) is taken as is.  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def per_dispatch(d):
    kt = {r["Dispatch_Id"]: r for r in csv.DictReader(open(os.path.join(d, "p_kernel_trace.csv")))}
    out = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "p_counter_collection.csv"))):
        did = r["Dispatch_Id"]
        out[did]["name"] = short(r["Kernel_Name"])
        out[did]["grid"] = int(r["Grid_Size"])
        out[did][r["Counter_Name"]] = out[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        k = kt.get(did)
        if k:
            out[did]["dur_s"] = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) * 1e-9
    return out


def group(disp):
    g = collections.defaultdict(list)
    for v in disp.values():
        g[(v["name"], v["grid"])].append(v)
    return g


def main():
    src, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.environ.get("PROF_OUT") or os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench_line = None
    for line in open(os.path.join(src, "kt.log")):
        if line.startswith("{"):
            bench_line = json.loads(line)
    summary = {"tag": tag, "bench_args_line": bench_line and {k: bench_line.get(k) for k in
                                                              ("value", "ms_per_step", "config")},
               "kernels": {}}
    passes = {p: group(per_dispatch(os.path.join(src, p))) for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_lds")
              if os.path.exists(os.path.join(src, p, "p_counter_collection.csv"))}
    keys = set()
    for g in passes.values():
        keys |= set(g)
    for key in sorted(keys):
        name, grid = key
        ent = {}
        for p, g in passes.items():
            ds = g.get(key, [])
            if not ds:
                continue
            ds = ds[len(ds) // 2:]  # steady state: drop the first half (warmup)
            for c in ds[0]:
                if c in ("name", "grid"):
                    continue
                ent.setdefault(c + "_by_pass", {})[p] = sum(x.get(c, 0.0) for x in ds) / len(ds)
        if not ent:
            continue
        flat = {}
        for c, byp in ent.items():
            base = c[: -len("_by_pass")]
            flat[base] = byp.get("pmc_sq", next(iter(byp.values())))
        if "FETCH_SIZE" in flat:
            flat["hbm_read_bytes_corrected"] = flat["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in flat:
            flat["hbm_write_bytes"] = flat["WRITE_SIZE"] * 1024
        if "GRBM_GUI_ACTIVE" in flat and flat.get("dur_s"):
            flat["clock_ghz"] = flat["GRBM_GUI_ACTIVE"] / 8 / flat["dur_s"] / 1e9
        summary["kernels"][f"{name} grid={grid}"] = flat
    # the bench's dominant screen (its roofline kernel; the seed pass's <.., true> variant excluded)
    kind = (bench_line or {}).get("roofline", {}).get("kernel", "")
    pat = {"k_screen_i8d": ("k_screen_i8d",), "k_screen_i8d_ms": ("k_screen_i8d_ms",),
           "k_screen_mfma_i8": ("k_screen_mfma<3,", "k_screen_i8d"),
           "k_screen_mfma": ("k_screen_mfma<",), "k_screen_gemv_i8": ("k_screen_gemv<3,",),
           "k_screen_gemv": ("k_screen_gemv<",)}
    screens = {k: v for k, v in summary["kernels"].items()
               if any(p in k for p in pat.get(kind, ("k_screen",))) and "true>" not in k and v.get("dur_s")
               and not (kind in ("k_screen_mfma", "k_screen_gemv") and "<3," in k)}
    if screens and bench_line and bench_line["config"]["workload"] != "cfg5":
        top = max(screens, key=lambda k: screens[k]["dur_s"])
        t = screens[top]
        cfg = bench_line["config"]
        rd = t.get("hbm_read_bytes_corrected")
        wr = t.get("hbm_write_bytes", 0.0)
        traffic = {"workload": cfg["workload"], "n_local": cfg["n_local"], "kernel": top,
                   "hbm_bytes_per_launch": None if rd is None else rd + wr,
                   "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                   "profiled_kernel_ms": t["dur_s"] * 1e3, "clock_ghz": t.get("clock_ghz"),
                   "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"}
        suffix = "" if cfg["n_local"] == cfg.get("N") else f"_n{cfg['n_local']}"
        kname = {"k_screen_i8d": "k_screen_mfma_i8", "k_screen_i8d_ms": "k_screen_mfma_i8"}.get(kind, kind)  # (the bench's traffic lookup key)
        with open(os.path.join(prof, f"traffic_{cfg['workload']}_{kname.replace('k_screen_', '')}{suffix}.json"), "w") as f:
            json.dump(traffic, f, indent=1)
        summary["dominant"] = traffic
    # IVF (cfg5): one search launches k_ivf_scan once per query-count class; traffic per search =
    # all scan dispatches / searches run (warmup + steps; every search is the same batch)
    ivf = {k: v for k, v in summary["kernels"].items() if "k_ivf_scan" in k}
    if ivf and bench_line and bench_line["config"]["workload"] == "cfg5":
        searches = bench_line["steps"] + bench_line["warmup"]
        tot = {}
        for p in ("pmc_fetch", "pmc_write"):
            disp = per_dispatch(os.path.join(src, p))
            tot[p] = sum(v.get("FETCH_SIZE" if p == "pmc_fetch" else "WRITE_SIZE", 0.0)
                         for v in disp.values() if "k_ivf_scan" in v["name"])
        kt = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv"))))
        scan_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt if "k_ivf_scan" in r["Kernel_Name"])
        rd, wr = tot["pmc_fetch"] * 1024 * 2 / searches, tot["pmc_write"] * 1024 / searches
        skew = float(bench_line["config"].get("skew", 0.0) or 0.0)
        traffic = {"workload": "cfg5", "n_local": bench_line["config"]["N"], "skew": skew,
                   "kernel": "k_ivf_scan (all scan launches of one search)",
                   "hbm_bytes_per_launch": rd + wr, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                   "profiled_kernel_ms": scan_ns * 1e-6 / searches,
                   "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"}
        with open(os.path.join(prof, "traffic_cfg5_ivf_scan" + (f"_skew{skew:g}" if skew else "") + ".json"), "w") as f:
            json.dump(traffic, f, indent=1)
        summary["dominant"] = traffic
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary.get("dominant"), indent=1))


if __name__ == "__main__":
    main()

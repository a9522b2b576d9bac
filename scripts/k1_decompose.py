"""K1 decomposition: the direct int8 screen's loop taken apart into cycles and clock, in ONE process
on one box, variants interleaved so drift cancels (DESIGN §5 "Where K1 int8's time goes").

Variants (include/vs.h ``vs_k1_probe``; csrc/vs_k1probe.hip), each over the whole cfg3 index with
every threshold at +inf (no survivors), on the real packed query tile and on a zeroed one:
  loads  -- corpus loads + query LDS-DMAs + the per-K-step barriers
  lds    -- + the query-fragment LDS reads
  mfma   -- + the 32 MFMAs per wave and K-step (no tile epilogue)
  full   -- + the epilogue's bound test (the product kernel's loop)
  full_ms, full_prio, full_ms_prio -- the whole loop under the mid-step-barrier schedule / static
            priority for waves 4-7 (the schedules compared; a form with the tile epilogue interleaved
            into the next tile's first K-step was measured too and removed: profiles/r06_k1_decompose_il.log)
Each workgroup stamps s_memtime (shader cycles) and s_memrealtime (100 MHz) around its loop, so a
launch splits into cycles per workgroup and the clock it held.  Between rounds the product search
runs (the same steps bench.py times), so the probes see the board in the product's thermal state.

Output JSON (``--out``): per (screen, variant, operands) the launch's wall ms (HIP events, median of
the reps after the first of each burst), the median / max workgroup loop cycles, cycles per K-step,
the in-kernel clock (median over workgroups), and the HBM fraction of the launch's algorithmic bytes.

Run (GPU box): python scripts/k1_decompose.py --out gpurun_out/k1_decomposition.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--heat-s", type=float, default=2.0, help="product searches before each round (s)")
    ap.add_argument("--variants", default="loads,lds,mfma,full,full_ms,full_prio,full_ms_prio")
    ap.add_argument("--native-variants", default="loads,mfma,full")
    ap.add_argument("--out", default="gpurun_out/k1_decomposition.json")
    args = ap.parse_args()

    import torch

    from photo_search_engine_amd.index import FlatIndex, synthesize_device
    SEED_CORPUS, SEED_QUERIES = 20260417, 20260418

    N, d, nq, k = args.rows, args.d, args.nq, args.k
    dev = torch.device("cuda", 0)
    t0 = time.time()
    ix = FlatIndex(d, "ip", "bf16", device=0)
    ix.reserve(N)
    ix.add_synthetic(SEED_CORPUS, 0, N, True)
    ix.set_screen("int8")
    q = torch.empty((nq, d), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    synthesize_device(0, SEED_QUERIES, 0, nq, d, q.data_ptr(), True, "bf16", stream)
    D = torch.empty((nq, k), dtype=torch.float32, device=dev)
    I = torch.empty((nq, k), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    print(f"index built in {time.time() - t0:.1f} s", flush=True)

    def heat(seconds: float) -> int:
        n, t = 0, time.time()
        while time.time() - t < seconds:
            for _ in range(10):
                ix.search_device_exact(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), None, 0, stream)
            torch.cuda.synchronize()
            n += 10
        return n

    tiles = (N + 255) // 256
    dpad8 = -(-d // 64) * 64
    nks_i8 = dpad8 // 64
    nks_bf = (-(-d // 32) * 32) // 32
    alg_i8 = N * (dpad8 + 4) + nq * dpad8 + nq * k * 12
    alg_bf = N * d * 2 + nq * d * 2 + nq * k * 12

    samples = {}
    heat(args.heat_s)
    for rnd in range(args.rounds):
        for screen, variants, nks, alg in (("int8", args.variants, nks_i8, alg_i8),
                                           ("native", args.native_variants, nks_bf, alg_bf)):
            for v in [x for x in variants.split(",") if x]:
                for zero in (False, True):
                    ms, st = ix.k1_probe(q.data_ptr(), nq, screen, v, zero, args.reps, stream)
                    G = st.shape[1]
                    for r in range(1, args.reps):  # the first launch of a burst follows a host gap
                        cyc = (st[r, :, 1] - st[r, :, 0]).astype("float64")
                        tick = (st[r, :, 3] - st[r, :, 2]).astype("float64")
                        ksteps = [((tiles - b + G - 1) // G) * nks for b in range(G)]
                        rec = samples.setdefault((screen, v, zero), {"ms": [], "cyc_med": [], "cyc_max": [],
                                                                     "cyc_per_kstep": [], "clock": [], "loop_us_max": []})
                        rec["ms"].append(ms[r])
                        rec["cyc_med"].append(float(statistics.median(cyc)))
                        rec["cyc_max"].append(float(cyc.max()))
                        rec["cyc_per_kstep"].append(float(statistics.median(cyc[b] / ksteps[b] for b in range(G))))
                        rec["clock"].append(float(statistics.median(cyc / tick * 0.1)))  # GHz
                        rec["loop_us_max"].append(float(tick.max() / 100.0))
        n = heat(args.heat_s)
        print(f"round {rnd}: {n} product searches between rounds", flush=True)

    out = {"config": {"rows": N, "d": d, "nq": nq, "k": k, "rounds": args.rounds, "reps": args.reps,
                      "note": "thresholds at +inf (no survivors); zero = the packed query tile zeroed; "
                              "cycles = s_memtime ticks per workgroup around the loop (shader clock); "
                              "clock = s_memtime / s_memrealtime x 100 MHz; wall = HIP events per launch"},
           "results": []}
    for (screen, v, zero), rec in samples.items():
        alg = alg_i8 if screen == "int8" else alg_bf
        wall = statistics.median(rec["ms"])
        out["results"].append({
            "screen": screen, "variant": v, "operands": "zero" if zero else "real",
            "wall_ms": round(wall, 4), "wall_ms_min": round(min(rec["ms"]), 4),
            "frac": round(alg / (wall * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "cycles_med": int(statistics.median(rec["cyc_med"])), "cycles_max": int(statistics.median(rec["cyc_max"])),
            "cycles_per_kstep": round(statistics.median(rec["cyc_per_kstep"]), 1),
            "clock_ghz": round(statistics.median(rec["clock"]), 3),
            "loop_us_max": round(statistics.median(rec["loop_us_max"]), 1),
            "n": len(rec["ms"])})
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    for r in out["results"]:
        print(f"{r['screen']:6s} {r['variant']:13s} {r['operands']:4s} wall {r['wall_ms']:.3f} ms  frac {r['frac']:.3f}  "
              f"cyc/WG {r['cycles_med']:>9d} (max {r['cycles_max']:>9d})  cyc/kstep {r['cycles_per_kstep']:7.1f}  "
              f"clock {r['clock_ghz']:.3f} GHz", flush=True)
    ix.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())

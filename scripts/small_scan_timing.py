"""Single-query calls over small corpora: the exact full scan (vs_set_scan_limit default) against the
screen path (GEMV screen + exact refine, scan limit 0), same index, same queries.  Per shape: wall
ms per FlatIndex.search call (host API end to end) and the timed kernel's mean ms (library HIP
events), both paths; answers compared.  python scripts/small_scan_timing.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O  # noqa: E402
from photo_search_engine_amd.index import FlatIndex  # noqa: E402

SHAPES = [(10_000, 1536, "f32", 10), (30_000, 1536, "f32", 10), (10_000, 1536, "bf16", 10),
          (100_000, 512, "f32", 10), (40_000, 1536, "f32", 100), (10_000, 4096, "f32", 10)]


def run(ix, qs, k, reps):
    for q in qs[:20]:
        ix.search(q, k)
    ix.timing_fetch()
    ix.set_timing(True)
    t0 = time.perf_counter()
    out = [ix.search(qs[i % len(qs)], k) for i in range(reps)]
    el = (time.perf_counter() - t0) / reps
    ix.set_timing(False)
    ms, kind = ix.timing_fetch()
    return el * 1e3, float(np.mean(ms)) if ms else float("nan"), kind, out


for N, d, dtype, k in SHAPES:
    ix = FlatIndex(d, "ip", dtype)
    ix.add_synthetic(O.SEED_CORPUS, 0, N, True)
    qs = [O.synth_rows(O.SEED_QUERIES, i, 1, d, True, "f32") for i in range(64)]
    wall_s, k_s, kind_s, out_s = run(ix, qs, k, 300)
    ix.set_scan_limit(0)
    wall_g, k_g, kind_g, out_g = run(ix, qs, k, 300)
    same = all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(out_s, out_g))
    print(json.dumps({"N": N, "d": d, "dtype": dtype, "k": k, "MB": round(N * d * (4 if dtype == "f32" else 2) / 1e6, 1),
                      "scan": {"wall_ms": round(wall_s, 4), "kernel_ms": round(k_s, 4), "kind": kind_s},
                      "screen": {"wall_ms": round(wall_g, 4), "kernel_ms": round(k_g, 4), "kind": kind_g},
                      "identical": same}), flush=True)
    ix.close()

"""The in-process multi-device store's step (vs_multi_search, host API end to end) beside one
index over the same rows on the same GPU: G shards of N/G rows (all on device 0 here -- the box
has one GPU -- so the shards' searches share it and the time is the shards' sum plus the
exchange; on G real GPUs they run side by side), d=1536 bf16, batch 256, k=100; the int8 screen
(two-phase step: phase A, floor merged on devices[0] and sent back, phase B, final merge) and the
native screen (one-phase).  Also checks the answers are identical to the single index's.
python scripts/multi_step_timing.py [--rows 3750000] [--shards 3] [--reps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from photo_search_engine_amd.index import FlatIndex, MultiDeviceFlatIndex  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=3_750_000)
ap.add_argument("--shards", type=int, default=3)
ap.add_argument("--d", type=int, default=1536)
ap.add_argument("--nq", type=int, default=256)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--reps", type=int, default=10)
args = ap.parse_args()

SEED_CORPUS, SEED_QUERIES = 20260417, 20260418
one = FlatIndex(args.d, "ip", "bf16", device=0)
one.add_synthetic(SEED_CORPUS, 0, args.rows, True)
multi = MultiDeviceFlatIndex(args.d, "ip", "bf16", devices=[0] * args.shards)
for r0 in range(0, args.rows, 1 << 18):  # through the host: the multi store deals rows in 64k chunks
    multi.add(one.reconstruct_n(r0, min(1 << 18, args.rows - r0)))
rng = np.random.default_rng(3)
q = rng.standard_normal((args.nq, args.d)).astype(np.float32)
q /= np.linalg.norm(q, axis=1, keepdims=True)


def med_ms(ix):
    ix.search(q, args.k)
    ts = []
    for _ in range(args.reps):
        t = time.perf_counter()
        out = ix.search(q, args.k)
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts)), out


res = {"rows": args.rows, "shards": args.shards, "d": args.d, "nq": args.nq, "k": args.k, "device": "one MI355X"}
for screen in ("int8", "native"):
    one.set_screen(screen)
    multi.set_screen(screen)
    t1, (D1, I1) = med_ms(one)
    tm, (Dm, Im) = med_ms(multi)
    res[screen] = {"one_index_ms": round(t1, 3), "multi_ms": round(tm, 3),
                   "step": "two-phase" if screen == "int8" else "one-phase",
                   "identical": bool(np.array_equal(I1, Im) and np.array_equal(D1, Dm))}
print(json.dumps(res), flush=True)
one.close()
multi.close()

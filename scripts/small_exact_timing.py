"""Exact flat search latency at photo-library sizes (host API end to end): N rows x d, bf16,
batch nq, k; prints per-call medians.  python scripts/small_exact_timing.py [--rows 100000] [--d 4096]"""
import argparse, os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from photo_search_engine_amd.index import FlatIndex

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000)
ap.add_argument("--d", type=int, default=4096)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--nq", type=int, default=0, help="only this batch (with --k)")
ap.add_argument("--k", type=int, default=10)
ap.add_argument("--sorted-mixture", action="store_true", help="64 Gaussian clusters (sigma 0.3), stored cluster by cluster")
args = ap.parse_args()
rng = np.random.default_rng(1)
ix = FlatIndex(args.d, "ip", args.dtype, device=0)
if args.sorted_mixture:
    cen = rng.standard_normal((64, args.d)).astype(np.float32)
    lab = np.sort(rng.integers(0, 64, args.rows))
for r0 in range(0, args.rows, 16384):
    m = min(16384, args.rows - r0)
    x = rng.standard_normal((m, args.d)).astype(np.float32)
    if args.sorted_mixture:
        x = cen[lab[r0:r0 + m]] + 0.3 * x
    ix.add(x / np.linalg.norm(x, axis=1, keepdims=True))
cases = ((args.nq, args.k),) if args.nq else ((1, 10), (16, 10), (64, 10), (256, 10), (256, 100))
for nq, k in cases:
    q = rng.standard_normal((nq, args.d)).astype(np.float32)
    if args.sorted_mixture:
        q = cen[rng.integers(0, 64, nq)] + 0.3 * q
    ix.search(q, k)
    ts = []
    for _ in range(args.reps):
        t = time.perf_counter()
        ix.search(q, k)
        ts.append(time.perf_counter() - t)
    tag = " sorted-mixture" if args.sorted_mixture else ""
    print(f"N={args.rows} d={args.d} {args.dtype}{tag} nq={nq} k={k}: {1e3 * np.median(ts):.3f} ms "
          f"(uncertified first passes so far: {ix.uncertified_count()})", flush=True)

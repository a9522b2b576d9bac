"""Screen health on clustered corpora, batch by batch: bench.py's mixture rows (64 unit centroids,
normalise(c + sigma g), inserted cluster by cluster with --sorted), d=1536 bf16, batch 256, k=100,
the int8 screen.  Per search: wall time, first-pass certificate failures, full-scanned queries and
the index's screen state (group residuals, margins, union depth, native routing).
python scripts/diag_mixture.py [--rows 2000000] [--sigma 0.3] [--sorted] [--batches 12]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=2_000_000)
ap.add_argument("--sigma", type=float, default=0.3)
ap.add_argument("--sorted", action="store_true")
ap.add_argument("--batches", type=int, default=12)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--check", action="store_true", help="exact top-k by fp64 torch matmul over the stored bf16 rows")
args = ap.parse_args()

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from photo_search_engine_amd.index import FlatIndex, synthesize_device  # noqa: E402

d, nq, k, N = 1536, 256, args.k, args.rows
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev).cuda_stream
cen = torch.empty((64, d), dtype=torch.float32, device=dev)
synthesize_device(0, bench.SEED_CENTROIDS, 0, 64, d, cen.data_ptr(), True, "bf16", st)
ix = FlatIndex(d, "ip", "bf16", device=0)
for r in range(0, N, 1 << 18):
    m = min(1 << 18, N - r)
    if args.sorted:
        xr = bench._mixture_rows_sorted(bench.SEED_CORPUS, r, m, N, d, cen, args.sigma, dev, st)
    else:
        xr = bench._mixture_rows(bench.SEED_CORPUS, r, m, d, cen, args.sigma, dev, st)
    ix.add_device(xr.data_ptr(), m, st)
    torch.cuda.synchronize()
q = bench._mixture_rows(bench.SEED_QUERIES, 0, nq, d, cen, args.sigma, dev, st).contiguous()
torch.cuda.synchronize()
exact_I = exact_S = None
if args.check:  # exact scores of the stored (bf16-rounded) rows, fp64, chunk by chunk; top-k merged
    qd = q.double()
    best_S = torch.full((nq, k), -float("inf"), dtype=torch.float64, device=dev)
    best_I = torch.full((nq, k), -1, dtype=torch.int64, device=dev)
    for r in range(0, N, 1 << 18):
        m = min(1 << 18, N - r)
        xr = (bench._mixture_rows_sorted(bench.SEED_CORPUS, r, m, N, d, cen, args.sigma, dev, st) if args.sorted
              else bench._mixture_rows(bench.SEED_CORPUS, r, m, d, cen, args.sigma, dev, st))
        sc = xr.to(torch.bfloat16).double() @ qd.T  # [m, nq]
        cs = torch.cat([best_S, sc.T], 1)
        ci = torch.cat([best_I, torch.arange(r, r + m, device=dev).expand(nq, m)], 1)
        best_S, o = torch.topk(cs, k, dim=1)
        best_I = torch.gather(ci, 1, o)
        del xr, sc
    exact_S, exact_I = best_S.cpu().numpy(), best_I.cpu().numpy()
    # rows within w of each query's k-th best score (the density the certificates work against)
    kth = best_S[:, -1]
    ws = (0.0005, 0.0011, 0.0022)
    near = torch.zeros((len(ws), nq), dtype=torch.int64, device=dev)
    for r in range(0, N, 1 << 18):
        m = min(1 << 18, N - r)
        xr = (bench._mixture_rows_sorted(bench.SEED_CORPUS, r, m, N, d, cen, args.sigma, dev, st) if args.sorted
              else bench._mixture_rows(bench.SEED_CORPUS, r, m, d, cen, args.sigma, dev, st))
        sc = xr.to(torch.bfloat16).double() @ qd.T
        for i, w in enumerate(ws):
            near[i] += (sc >= kth - w).sum(0)
        del xr, sc
    near = near.cpu().numpy()
    print(json.dumps({"check": "exact top-k computed", "kth_score_min": float(exact_S[:, -1].min()),
                      "rows_within": {str(w): {"median": int(np.median(near[i])), "max": int(near[i].max()),
                                               "argmax": int(near[i].argmax())} for i, w in enumerate(ws)}}), flush=True)
D = torch.empty((nq, k), dtype=torch.float32, device=dev)
I = torch.empty((nq, k), dtype=torch.int64, device=dev)
S = torch.empty((nq, k), dtype=torch.float64, device=dev)
ref = None
for screen in ("native", "int8"):
    ix.set_screen(screen)
    print(json.dumps({"screen": screen, "state": ix.screen_state()}), flush=True)
    for b in range(args.batches):
        u0, r0 = ix.uncertified_count(), ix.full_scan_count()
        t = time.perf_counter()
        ix.search_device_exact(q.data_ptr(), nq, k, D.data_ptr(), I.data_ptr(), S.data_ptr(), 0, st)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t)
        got = I.cpu().numpy().copy()
        if ref is None:
            ref = got
        bad = []
        if exact_I is not None:  # queries whose id SET differs from the exact top-k (fp64 ties aside)
            for qi in range(nq):
                if set(got[qi].tolist()) != set(exact_I[qi].tolist()):
                    bad.append(qi)
        print(json.dumps({"screen": screen, "batch": b, "ms": round(ms, 3),
                          "uncertified": ix.uncertified_count() - u0, "full_scan": ix.full_scan_count() - r0,
                          "identical_to_native": bool((got == ref).all()), "inexact_queries": bad,
                          "state": ix.screen_state()}), flush=True)
ix.close()

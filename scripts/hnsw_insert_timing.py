#!/usr/bin/env python3
"""Cost of extending a saved HNSW graph (insertion must cost the new rows, not the
graph's size per batch): a VectorStore(index_type='hnsw') of N rows; the first N0 rows' graph is
built at once (VECTOR_HNSW_GRAPH_MAX_ROWS = N0), then rows are inserted the way save() does
(hnsw.insert_rows, 4096-row batches) in chunks to N0 + C, + 2C, ...; prints the seconds per
inserted 4096-row batch at each graph size (flat = linear total cost).  One JSON line at the end.

  python scripts/hnsw_insert_timing.py [--rows 400000] [--n0 50000] [--chunk 50000] [--d 1536]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=400_000)
    ap.add_argument("--n0", type=int, default=50_000)
    ap.add_argument("--chunk", type=int, default=50_000)
    ap.add_argument("--d", type=int, default=1536)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    os.environ["VECTOR_DTYPE"] = args.dtype
    os.environ["VECTOR_HNSW_GRAPH_MAX_ROWS"] = str(args.n0)
    from photo_search_engine_amd import hnsw as hnsw_mod
    from photo_search_engine_amd.vector_store import VectorStore
    store = VectorStore(dimension=args.d, index_path="/tmp/hnsw_ins.index", metadata_path="/tmp/hnsw_ins.json",
                        metric="cosine", index_type="hnsw", hnsw_m=48, hnsw_ef_construction=320, hnsw_ef_search=192)
    rng = np.random.default_rng(7)
    centres = rng.standard_normal((1000, args.d)).astype(np.float32)
    centres /= np.linalg.norm(centres, axis=1, keepdims=True)
    for r0 in range(0, args.rows, 16384):
        m = min(16384, args.rows - r0)
        x = centres[rng.integers(0, 1000, m)] + (0.75 / np.sqrt(args.d)) * rng.standard_normal((m, args.d)).astype(np.float32)
        store.add(x.astype(np.float32), [{}] * m)
    t = time.perf_counter()
    g = store._build_graph_exact(args.n0)
    exact_s = time.perf_counter() - t
    print(f"exact graph of {args.n0} rows: {exact_s:.2f} s", flush=True)
    make = lambda: store._create_index(args.d)  # noqa: E731
    steps = []
    n = args.n0
    while n < args.rows:
        n1 = min(args.rows, n + args.chunk)
        t = time.perf_counter()
        g = hnsw_mod.insert_rows(store.index, g, n, n1, 320, make)
        dt = time.perf_counter() - t
        batches = (n1 - n + 4095) // 4096
        steps.append({"graph_rows_before": n, "inserted": n1 - n, "s": round(dt, 3),
                      "s_per_4096_batch": round(dt / batches, 4)})
        print(json.dumps(steps[-1]), flush=True)
        n = n1
    print(json.dumps({"workload": f"hnsw insert_rows d={args.d} {args.dtype} M=48 efConstruction=320, "
                                  f"exact graph of {args.n0} rows then {args.chunk}-row chunks to {args.rows}",
                      "exact_build_s": round(exact_s, 3), "steps": steps}))


if __name__ == "__main__":
    main()

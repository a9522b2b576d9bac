#!/usr/bin/env python3
"""HNSW graph search vs exact flat search on one MI355X, at the reference's
HNSW settings (.env.example:82-83: M=48, efConstruction=320, efSearch=192; EMBEDDING_DIMENSION
4096, TOP_K 10).  The graph is the one VectorStore.save() writes (VectorStore._build_graph: faiss's
level draw; every level's exact efConstruction candidates by the GPU flat search, then faiss's
neighbour-selection heuristic with reverse links by k_hnsw_prune).  Prints one JSON line.

  python scripts/hnsw_bench.py [--rows 100000] [--d 4096] [--dtype bf16] [--nq 256] [--reps 5]
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

from photo_search_engine_amd.hnsw import HNSWGraph  # noqa: E402
from photo_search_engine_amd.vector_store import VectorStore  # noqa: E402

SEED_QUERIES = 20260418


def recall_at(I, Ie, k):
    return float(np.mean([len(set(a[:k]) & set(b[:k])) / k for a, b in zip(I, Ie)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=4096)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=48)
    ap.add_argument("--ef", type=int, default=192)
    ap.add_argument("--efc", type=int, default=320)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--data", default="mixture", choices=["mixture", "iso"],
                    help="mixture: unit rows around 1000 random centres (cosine ~0.8 to their centre), "
                         "queries from the same mixture; iso: isotropic unit rows (no structure)")
    args = ap.parse_args()
    N, d, k, M = args.rows, args.d, args.k, args.m
    os.environ["VECTOR_DTYPE"] = args.dtype
    os.environ["VECTOR_HNSW_SEARCH"] = "graph"
    store = VectorStore(dimension=d, index_path="/tmp/hnsw_bench.index", metadata_path="/tmp/hnsw_bench.json",
                        metric="cosine", index_type="hnsw", hnsw_m=M, hnsw_ef_construction=args.efc, hnsw_ef_search=args.ef)
    rng = np.random.default_rng(SEED_QUERIES)
    centres = rng.standard_normal((1000, d)).astype(np.float32)
    centres /= np.linalg.norm(centres, axis=1, keepdims=True)

    def draw(m):
        if args.data == "iso":
            return rng.standard_normal((m, d)).astype(np.float32)
        x = centres[rng.integers(0, 1000, m)] + (0.75 / np.sqrt(d)) * rng.standard_normal((m, d)).astype(np.float32)
        return x / np.linalg.norm(x, axis=1, keepdims=True)

    for r0 in range(0, N, 16384):
        m = min(16384, N - r0)
        store.add(draw(m).astype(np.float32), [{}] * m)  # (the store normalises rows, cosine)
    q = draw(args.nq).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    ix = store.index

    t = time.perf_counter()
    store._graph_arrays = store._build_graph(N)
    build_s = time.perf_counter() - t
    g = store._graph_arrays
    hg = HNSWGraph(ix, g, args.ef)

    hg.search(q, k)  # warm-up (module load, workspaces)
    ix.search(q, k)
    tg = []
    for _ in range(args.reps):
        t = time.perf_counter()
        D, I = hg.search(q, k)
        tg.append(time.perf_counter() - t)
    te = []
    for _ in range(args.reps):
        t = time.perf_counter()
        De, Ie = ix.search(q, k)
        te.append(time.perf_counter() - t)
    lat = []
    for j in range(min(32, args.nq)):
        t = time.perf_counter()
        hg.search(q[j:j + 1], k)
        lat.append(time.perf_counter() - t)
    tg_ms, te_ms = 1e3 * float(np.median(tg)), 1e3 * float(np.median(te))
    out = {
        "workload": f"hnsw graph search N={N} d={d} {args.dtype} M={M} efSearch={args.ef} k={k} batch={args.nq}",
        "graph": f"VectorStore._build_graph: {int(g['max_level']) + 1} levels, faiss heuristic over "
                 f"exact efConstruction={args.efc} candidates, reverse links",
        "graph_build_s": round(build_s, 3),
        "hnsw_batch_ms": round(tg_ms, 3),
        "hnsw_qps": round(args.nq / (tg_ms / 1e3), 1),
        "hnsw_single_query_ms_p50": round(1e3 * float(np.median(lat)), 3),
        "exact_batch_ms": round(te_ms, 3),
        "exact_qps": round(args.nq / (te_ms / 1e3), 1),
        f"hnsw_recall_at_{k}_vs_exact": round(recall_at(I, Ie, k), 4),
        "data": ("synthetic unit rows around 1000 centres, queries from the same mixture" if args.data == "mixture"
                 else "synthetic isotropic unit rows") + "; host API end to end",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()

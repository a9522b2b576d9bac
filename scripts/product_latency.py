"""Per-call latency of the product path: VectorStore.search (one query, the Searcher's call shape,
core/searcher.py:1195) over the reference's configured dimension (EMBEDDING_DIMENSION 4096,
config.py:142), fp32 storage (the reference's precision).  Host API end to end: normalisation,
H2D, screen, refine, certificate, D2H, result dicts.  The CPU column is the faiss IndexFlatIP
restatement (oracle/vs_oracle.c, nq < 20 path = faiss' sequential SIMD scan) on the same rows.

    python scripts/product_latency.py [--rows 100000] [--calls 200] [--screen native|int8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--dim", type=int, default=4096)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--screen", default="native", choices=["native", "int8"],
                    help="VECTOR_SCREEN of the store (int8: the certified int8 GEMV screen)")
    args = ap.parse_args()
    os.environ["VECTOR_SCREEN"] = args.screen
    from oracle import oracle as O
    from photo_search_engine_amd.vector_store import VectorStore

    N, d = args.rows, args.dim
    x = O.synth_rows(O.SEED_CORPUS, 0, N, d, False, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, args.calls, d, False, "f32")
    tmp = tempfile.mkdtemp()
    store = VectorStore(dimension=d, index_path=os.path.join(tmp, "i"), metadata_path=os.path.join(tmp, "m"))
    store.add(x, [{"photo_path": f"/{i}"} for i in range(N)])
    out = {"rows": N, "dim": d, "dtype": "f32", "screen": args.screen}
    for top_k in (10, 50, 500):
        for i in range(5):
            store.search(q[i].tolist(), top_k)  # warm
        t = []
        for i in range(args.calls):
            t0 = time.perf_counter()
            store.search(q[i].tolist(), top_k)
            t.append(time.perf_counter() - t0)
        out[f"gpu_ms_p50_k{top_k}"] = round(float(np.median(t)) * 1e3, 3)
        out[f"gpu_ms_p99_k{top_k}"] = round(float(np.percentile(t, 99)) * 1e3, 3)
    out["uncertified_first_pass"] = store.index.uncertified_count()
    xs = store.index.reconstruct_n(0, N)
    qn = store._normalize_rows(q[:20])
    t = []
    for i in range(20):
        t0 = time.perf_counter()
        O.knn_faiss_fp32(xs, qn[i:i + 1], 50, "ip", 1)
        t.append(time.perf_counter() - t0)
    out["cpu_faiss_restatement_ms_p50_k50_1thread"] = round(float(np.median(t)) * 1e3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

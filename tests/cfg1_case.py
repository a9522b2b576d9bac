"""BASELINE cfg1 (N=10k, d=1536, one query per call, top-10) through a ``VectorStore`` class,
checked against tests/golden/cfg1_wrapper_golden.npz -- the reference wrapper
(/root/reference/utils/vector_store.py) run on the same raw rows (tests/golden/make_goldens.py
``make_cfg1_golden``).  Shared by the CPU host test (checker-backed index) and the GPU test (the HIP
index through the C ABI)."""
from __future__ import annotations

import hashlib
import os

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg1_wrapper_golden.npz")
N, D, NQ, NQ_L2 = 10000, 1536, 32, 8
TOPKS = (10, 1, 50)
TAIL = 16  # rows added one add_item at a time after the bulk add (the indexer's own call)


def load_golden():
    g = np.load(GOLDEN)
    assert int(g["N"]) == N and int(g["d"]) == D
    return g


def corpus():
    """The raw (un-normalised) rows and queries the golden was recorded on."""
    x = O.synth_rows(O.SEED_CORPUS, 0, N, D, False, "f32")
    q = O.synth_rows(O.SEED_QUERIES, 0, NQ, D, False, "f32")
    return x, q


def meta(i: int) -> dict:
    return {"photo_path": f"/photos/{i:05d}.jpg", "row": i}


def build_store(VS, tmp_path, metric: str, x: np.ndarray):
    store = VS(dimension=D, index_path=str(tmp_path / f"{metric}.index"),
               metadata_path=str(tmp_path / f"{metric}.metadata.json"), metric=metric)
    store.add(x[:N - TAIL], [meta(i) for i in range(N - TAIL)])
    for i in range(N - TAIL, N):
        store.add_item(x[i].tolist(), meta(i))
    assert store.get_total_items() == N
    return store


def check_store(store, g, metric: str, q: np.ndarray, prefix: str | None = None, topks=TOPKS, files: bool = True):
    """Every golden search of ``metric`` (one query per call), the probe embeddings and the saved
    file's bytes."""
    prefix = prefix or metric
    nq = NQ if metric == "cosine" else NQ_L2
    for top_k in topks:
        want_I, want_D = g[f"{prefix}_top{top_k}_I"], g[f"{prefix}_top{top_k}_D"]
        for a in range(nq):
            res = store.search(q[a].tolist(), top_k)
            assert [r["metadata"]["row"] for r in res] == want_I[a].tolist(), (prefix, top_k, a)
            assert [r["distance"] for r in res] == want_D[a].tolist(), (prefix, top_k, a)
    if not files:
        return
    for i, emb in zip(g[f"{metric}_probe_rows"].tolist(), g[f"{metric}_probe_emb"]):
        assert store.get_embedding_by_photo_path(meta(i)["photo_path"]) == emb.tolist()
    store.save()
    with open(store.index_path, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == str(g[f"{metric}_index_sha256"])
